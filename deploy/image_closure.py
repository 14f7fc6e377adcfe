#!/usr/bin/env python3
"""The runtime image's file closure: the exporter binary, everything it and the libraries it
dlopens need at run time, and nothing else (no Python, no ROCm development image).

Reference: the production image is `python:3` + `requests` + one script + a vendored libltdl
(/root/reference/Dockerfile:1-7). Here the runtime stage of deploy/Dockerfile is a plain Ubuntu
base plus exactly this closure, staged by the build stage:

  * bin/gpumon-exporter and its DT_NEEDED closure (ldd);
  * what it dlopen()s: libamd_smi (csrc/core/amdsmi_backend.cpp), librocm_smi64 (rsmi_backend.cpp),
    libssl / libcrypto for an https:// INFLUXDB_URL (csrc/core/tls.cpp), the ROCTx library
    (--roctx), each with its own DT_NEEDED closure; the CA bundle;
  * --overlays (deploy/k8s/overlays/pmc, ondevice): lib/libgpumon_pmc.so, lib/libgpumon_probe.so,
    lib/gpumon-ondevice-helper, the libraries the ROCm runtimes dlopen (aqlprofile), and
    rocprofiler-sdk's counter definitions.

Files keep their absolute paths (ROCm libraries stay under /opt/rocm/lib, where the plugins' RUNPATH
and rocprofiler-sdk's share/ lookup expect them); the product goes to /opt/gpumon/{bin,lib} (the
exporter finds its plugins in ../lib). glibc itself comes from the base image.

    python3 deploy/image_closure.py list [--overlays]          # JSON: files, sizes
    python3 deploy/image_closure.py stage --root DIR [--overlays]
    python3 deploy/image_closure.py check --root DIR [--backend mock] [--overlays]   # run + /proc maps
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time
import urllib.request

TREE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
PREFIX = "/opt/gpumon"
LIB_DIRS = [f"{ROCM}/lib", "/lib/x86_64-linux-gnu", "/usr/lib/x86_64-linux-gnu", "/usr/local/lib", "/lib64"]
# From the base image (glibc): never copied, always allowed in /proc/<pid>/maps.
SYSTEM = {"linux-vdso.so.1", "ld-linux-x86-64.so.2", "libc.so.6", "libm.so.6", "libpthread.so.0", "libdl.so.2",
          "librt.so.1", "libutil.so.1", "libresolv.so.2", "libnss_files.so.2", "libnss_dns.so.2",
          "libmvec.so.1"}

PRODUCT = {"bin/gpumon-exporter": f"{PREFIX}/bin/gpumon-exporter"}
PRODUCT_OVERLAYS = {"lib/libgpumon_pmc.so": f"{PREFIX}/lib/libgpumon_pmc.so",
                    "lib/libgpumon_probe.so": f"{PREFIX}/lib/libgpumon_probe.so",
                    "lib/gpumon-ondevice-helper": f"{PREFIX}/lib/gpumon-ondevice-helper"}
# dlopen()ed by name (not in any DT_NEEDED): each name is kept as the path it resolves to, with its
# symlink chain, so the loader finds it under the name the code asks for
DLOPEN = ["libamd_smi.so.26", "libamd_smi.so", "librocm_smi64.so.1", "librocm_smi64.so", "libssl.so.3",
          "libcrypto.so.3", "librocprofiler-sdk-roctx.so.1",
          # libamd_smi dlopens the DRM libraries at init (seen mapped on MI355X, profiles/r5_gpu_runs.md)
          "libdrm.so.2", "libdrm_amdgpu.so.1"]
DLOPEN_OVERLAYS = ["libhsa-amd-aqlprofile64.so.1", "libhsa-amd-aqlprofile64.so"]
DATA = ["/etc/ssl/certs/ca-certificates.crt"]
# optional data: staged when the build image has it (libdrm_amdgpu's marketing-name table)
DATA_OPTIONAL = ["/usr/share/libdrm/amdgpu.ids", "/opt/amdgpu/share/libdrm/amdgpu.ids"]
DATA_OVERLAYS = [f"{ROCM}/share/rocprofiler-sdk/counter_defs.yaml", f"{ROCM}/share/rocprofiler-sdk/basic_counters.xml",
                 f"{ROCM}/share/rocprofiler-sdk/derived_counters.xml"]


def resolve(name: str) -> str | None:
    if name.startswith("/"):
        return name if os.path.exists(name) else None
    for d in LIB_DIRS:
        p = os.path.join(d, name)
        if os.path.exists(p):
            return p
    return None


def needed(path: str) -> list[tuple[str, str | None]]:
    """(soname, resolved path) of every library `path` loads (ldd: the whole DT_NEEDED tree)."""
    r = subprocess.run(["ldd", path], capture_output=True, text=True)
    out = []
    for line in r.stdout.splitlines():
        parts = line.split()
        if not parts:
            continue
        if "=>" in parts:
            i = parts.index("=>")
            so = parts[0]
            p = parts[i + 1] if i + 1 < len(parts) and parts[i + 1].startswith("/") else None
            out.append((so, p))
        elif parts[0].startswith("/"):
            out.append((os.path.basename(parts[0]), parts[0]))
        else:
            out.append((parts[0], None))
    return out


def closure(overlays: bool = False) -> dict:
    """{"files": {image path: source path}, "missing": [...]} (symlinks recorded as links)."""
    files, links, missing = {}, {}, []

    def add_path(p: str):
        # the name asked for, every link on the way, and the real file, at their own paths
        while os.path.islink(p):
            t = os.readlink(p)
            links[p] = t
            p = os.path.normpath(os.path.join(os.path.dirname(p), t))
        files[p] = p

    def add_elf(src: str, dest: str | None = None):
        if dest:
            files[dest] = src
        else:
            add_path(src)
        for so, p in needed(src):
            if so in SYSTEM or os.path.basename(p or "") in SYSTEM:
                continue
            if p is None:
                if so.startswith("libgpumon_pmc"):  # the helper's sibling: staged with the overlays
                    continue
                missing.append(f"{so} (needed by {os.path.basename(src)})")
                continue
            if p.startswith(TREE + "/"):
                continue  # our own plugin (staged under PREFIX)
            add_path(p)

    prod = dict(PRODUCT, **(PRODUCT_OVERLAYS if overlays else {}))
    for rel, dest in prod.items():
        src = os.path.join(TREE, rel)
        if not os.path.exists(src):
            missing.append(f"{rel} (run make all)")
            continue
        add_elf(src, dest)
    for name in DLOPEN + (DLOPEN_OVERLAYS if overlays else []):
        p = resolve(name)
        if p is None:
            missing.append(f"{name} (dlopen)")
            continue
        add_elf(p)
    for d in DATA + (DATA_OVERLAYS if overlays else []):
        if os.path.exists(d):
            add_path(d)
        else:
            missing.append(d)
    for d in DATA_OPTIONAL:
        if os.path.exists(d):
            add_path(d)
    return {"files": dict(sorted(files.items())), "links": dict(sorted(links.items())), "missing": missing}


def stage(root: str, overlays: bool = False) -> dict:
    c = closure(overlays)
    for dest, src in c["files"].items():
        out = root + dest
        os.makedirs(os.path.dirname(out), exist_ok=True)
        shutil.copy2(os.path.realpath(src), out)
    for link, target in c["links"].items():
        out = root + link
        os.makedirs(os.path.dirname(out), exist_ok=True)
        if os.path.lexists(out):
            os.remove(out)
        os.symlink(target, out)
    os.makedirs(root + "/etc/ld.so.conf.d", exist_ok=True)
    with open(root + "/etc/ld.so.conf.d/gpumon-rocm.conf", "w") as fh:
        fh.write(f"{ROCM}/lib\n")
    c["bytes"] = sum(os.path.getsize(root + d) for d in c["files"])
    return c


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _children(pid: int) -> list[int]:
    out = []
    for p in os.listdir("/proc"):
        if p.isdigit():
            try:
                with open(f"/proc/{p}/stat") as fh:
                    if int(fh.read().rsplit(")", 1)[1].split()[1]) == pid:
                        out.append(int(p))
            except (OSError, ValueError, IndexError):
                pass
    return out


def mapped_files(pid: int) -> set[str]:
    out = set()
    with open(f"/proc/{pid}/maps") as fh:
        for line in fh:
            parts = line.split(None, 5)
            if len(parts) == 6 and parts[5].startswith("/"):
                out.add(parts[5].strip().replace(" (deleted)", ""))
    return out


def environment_maps(env: dict) -> set[str]:
    """Files any program started with `env` maps before it runs a line of its own (whatever the
    environment preloads): measured on a trivial child with the same environment, not guessed."""
    p = subprocess.Popen(["sleep", "5"], env=env)
    try:
        time.sleep(0.2)
        return mapped_files(p.pid) - {os.path.realpath("/bin/sleep"), "/usr/bin/sleep", "/bin/sleep"}
    except OSError:
        return set()
    finally:
        p.kill()
        p.wait()


def outside(paths, root: str) -> list[str]:
    """Mapped shared objects / executables that are neither staged nor glibc."""
    bad = []
    for p in sorted(paths):
        if p.startswith("/dev/") or p.startswith("/sys/") or p.startswith("/memfd:") or p.startswith("/proc/"):
            continue
        if p.startswith(root + "/") or os.path.basename(p) in SYSTEM:
            continue
        if ".so" in os.path.basename(p) or os.access(p, os.X_OK):
            bad.append(p)
    return bad


def run_check(root: str, args: list[str], env_extra: dict | None = None, settle_s: float = 3.0,
              want_children: int = 0) -> dict:
    """Start the staged exporter with the library search limited to the staged tree, wait for
    /healthz, then list every file its process (and helper children) mapped."""
    port = _free_port()
    libpath = ":".join(root + d for d in (f"{ROCM}/lib", "/lib/x86_64-linux-gnu", "/usr/lib/x86_64-linux-gnu"))
    env = {k: v for k, v in os.environ.items() if k not in ("LD_LIBRARY_PATH", "GPUMON_PLUGIN_DIR", "GPUMON_AMDSMI_LIB",
                                                              "PYTHONPATH")}
    env.update({"LD_LIBRARY_PATH": libpath, "SSL_CERT_FILE": root + "/etc/ssl/certs/ca-certificates.crt"},
               **(env_extra or {}))
    exe = root + PREFIX + "/bin/gpumon-exporter"
    p = subprocess.Popen([exe, "--listen", f"127.0.0.1:{port}", "--no-pod-resources", "--no-cri", "--interval", "0.5",
                          "--log-level", "warn", *args], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                         text=True)
    res = {"args": args, "ok": False}
    try:
        deadline = time.time() + 60
        up = False
        while time.time() < deadline and p.poll() is None:
            try:
                urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=2).read()
                up = True
                break
            except OSError:
                time.sleep(0.2)
        if not up:
            res["error"] = "exporter did not serve /healthz: " + (p.stderr.read()[-2000:] if p.poll() is not None else "")
            return res
        time.sleep(settle_s)
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
        maps = mapped_files(p.pid) - environment_maps(env)
        kids = _children(p.pid)
        kid_maps = set()
        for k in kids:
            try:
                kid_maps |= mapped_files(k) - environment_maps(env)
            except OSError:
                pass
        res.update({"pid_maps": len(maps), "children": len(kids), "outside": outside(maps | kid_maps, root),
                    "staged_libs_mapped": sorted({os.path.basename(m) for m in maps | kid_maps
                                                  if m.startswith(root + "/") and ".so" in m}),
                    "gpu_up": [l for l in body.splitlines() if l.startswith("gpu_up{")][:8],
                    "backend_up": [l for l in body.splitlines() if l.startswith("gpumon_backend_up{")]})
        res["ok"] = not res["outside"] and len(kids) >= want_children
        return res
    finally:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
            try:
                p.wait(30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["list", "stage", "check"])
    ap.add_argument("--root", default="")
    ap.add_argument("--overlays", action="store_true")
    ap.add_argument("--backend", default="mock:gpus=1")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.cmd == "list":
        c = closure(a.overlays)
        c["bytes"] = sum(os.path.getsize(os.path.realpath(s)) for s in c["files"].values())
        print(json.dumps(c, indent=1))
        return 1 if c["missing"] else 0
    if a.cmd == "stage":
        if not a.root:
            ap.error("stage needs --root")
        c = stage(a.root, a.overlays)
        print(json.dumps({"files": len(c["files"]), "links": len(c["links"]), "bytes": c["bytes"],
                          "missing": c["missing"]}))
        return 1 if c["missing"] else 0
    root = a.root or tempfile.mkdtemp(prefix="gpumon-closure-")
    try:
        if not a.root:
            stage(root, a.overlays)
        runs = [run_check(root, ["--backend", a.backend], settle_s=2.0)]
        if a.overlays:
            runs.append(run_check(root, ["--backend", a.backend, "--pmc"], settle_s=6.0, want_children=1))
        out = {"root": root, "ok": all(r["ok"] for r in runs), "runs": runs}
        print(json.dumps(out, indent=1))
        if a.out:
            with open(a.out, "w") as fh:
                json.dump(out, fh, indent=1)
        return 0 if out["ok"] else 1
    finally:
        if not a.root:
            shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())

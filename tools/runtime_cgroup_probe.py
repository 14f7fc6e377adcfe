#!/usr/bin/env python3
"""What the PID -> container attributor sees on a real container runtime (VERDICT r3 missing #2).

The reference resolved container PIDs with `docker top <cid> -eo pid` (/root/reference/gpu.py:177);
gpumon reads /proc/<pid>/cgroup (+ mountinfo) instead (csrc/core/attribution.cpp). This records,
on whatever box it runs on (the gpurun GPU box is itself a container):

* /proc/self/cgroup, /proc/1/cgroup, the cgroup namespace inode, the first mountinfo lines;
* the attributor's resolve() for this process and for a GPU tenant subprocess (a torch process
  holding a HIP context), and the pod_gpu rows the exporter builds for the tenant;
* whether a cgroup namespace hides the container path (`0::/`).

    python tools/runtime_cgroup_probe.py [OUTDIR]      -> OUTDIR/runtime.json (+ raw files)
"""

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _read(path, limit=None):
    try:
        with open(path) as fh:
            lines = fh.read().splitlines()
    except OSError as e:
        return [f"<{type(e).__name__}: {e}>"]
    return lines[:limit] if limit else lines


def _ns(pid, kind):
    try:
        return os.readlink(f"/proc/{pid}/ns/{kind}")
    except OSError as e:
        return f"<{e}>"


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/runtime"
    os.makedirs(out, exist_ok=True)
    from gpumon import core

    tenant_code = ("import torch, time, sys; x = torch.ones(1 << 20, device='cuda'); torch.cuda.synchronize(); "
                   "print('ready', flush=True); time.sleep(float(sys.argv[1]))")
    tenant = subprocess.Popen([sys.executable, "-c", tenant_code, "30"], stdout=subprocess.PIPE, text=True)
    try:
        line = tenant.stdout.readline().strip()
        ex = core().Exporter({"backend": "auto", "serve_http": False, "interval_s": 0, "host": "probe",
                              "cri_socket": "", "pod_resources_socket": "", "log_level": "warn"})
        err = ex.start()
        rows, resolved = [], {}
        if not err:
            deadline = time.time() + 10
            while time.time() < deadline:
                ex.tick()
                rows = [r for r in ex.pod_rows() if str(r.get("pid")) == str(tenant.pid)]
                if rows:
                    break
                time.sleep(0.2)
            for name, pid in (("self", os.getpid()), ("tenant", tenant.pid), ("init", 1)):
                resolved[name] = dict(ex.resolve_pid(pid), pid=pid)
        ex.stop()
        # the cgroup parse alone (no /dev/kfd ownership check): what the path says for each pid
        ex = core().Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0, "verify_kfd": False,
                              "log_level": "warn"})
        ex.start()
        parsed = {name: dict(ex.resolve_pid(pid), pid=pid)
                  for name, pid in (("self", os.getpid()), ("tenant", tenant.pid), ("init", 1))}
        ex.stop()
        res = {
            "tenant_ready": line,
            "exporter_error": err,
            "self_cgroup": _read("/proc/self/cgroup"),
            "tenant_cgroup": _read(f"/proc/{tenant.pid}/cgroup"),
            "init_cgroup": _read("/proc/1/cgroup"),
            "cgroup_ns": {"self": _ns("self", "cgroup"), "init": _ns(1, "cgroup")},
            "pid_ns": {"self": _ns("self", "pid"), "init": _ns(1, "pid")},
            "mountinfo_head": _read("/proc/self/mountinfo", 40),
            "cgroup_mounts": [l for l in _read("/proc/self/mountinfo") if " - cgroup" in l],
            "uid": os.getuid(),
            "resolved": resolved,
            "parsed_without_kfd_check": parsed,
            "tenant_rows": [{k: r.get(k) for k in ("dev", "pid", "idle", "containerid", "podname", "namespace",
                                                   "procressname", "used_memory_bytes", "source")} for r in rows],
        }
        res["cgroup_namespaced_root"] = any(l.endswith("::/") for l in res["self_cgroup"])
    finally:
        tenant.kill()
        tenant.wait()
    with open(os.path.join(out, "runtime.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: res[k] for k in ("exporter_error", "self_cgroup", "cgroup_namespaced_root", "resolved")}))


if __name__ == "__main__":
    main()

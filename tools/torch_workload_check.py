"""Cross-check the exporter's PMC-derived series against a REAL PyTorch workload, not the repo's own
burn kernels: a tenant process runs back-to-back torch GEMMs (hipBLASLt kernels) in bf16 / f16 /
fp8, event-timed, while the deployed exporter (bin/gpumon-exporter --pmc, 1 Hz) counts them from
another process. Reports, per dtype, the exported gpu_mfma_tflops{dtype} and gpu_mfma_util_percent
(median over the ticks fully inside the run) against the tenant's own FLOP count / event time, and
the tenant's per-process busy % and CU-equivalents (KFD).

The reference had no compute-side signal at all: device util copied onto every process row
(/root/reference/gpu.py:205).

    python tools/torch_workload_check.py [--seconds 8] [--dtypes bf16,f16,fp8] > out.json
    python tools/torch_workload_check.py --shared [--seconds 10] > out.json

--shared: two bf16 GEMM tenants (8192^3, then 4096^3 4 s later) on the same GPU, the reference
dashboard's "(共享)" shared-GPU case. The exported device TFLOP/s must equal the sum of the two
tenants' FLOPs over wall time; each tenant gets its own row (busy %, CU-equivalents), and
pod_gpu_mfma_util_percent is absent (the device's MFMA util is not one pod's when shared).
"""

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TENANT = r"""
import json, sys, time, torch
dtype, seconds, n = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
dev = torch.device("cuda:0")
if dtype == "fp8":
    a = torch.randn(n, n, device=dev).to(torch.float8_e4m3fn)
    b = torch.randn(n, n, device=dev).to(torch.float8_e4m3fn).t()  # column-major B for _scaled_mm
    one = torch.ones((), device=dev)
    mm = lambda: torch._scaled_mm(a, b, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
else:
    dt = {"bf16": torch.bfloat16, "f16": torch.float16}[dtype]
    a = torch.randn(n, n, device=dev, dtype=dt)
    b = torch.randn(n, n, device=dev, dtype=dt)
    mm = lambda: a @ b
for _ in range(20):
    mm()
torch.cuda.synchronize()
batch, flops, busy_ms, batches = 20, 0.0, 0.0, 0
t0 = time.time()
while time.time() - t0 < seconds:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(batch):
        mm()
    e1.record()
    e1.synchronize()
    busy_ms += e0.elapsed_time(e1)
    flops += 2.0 * n ** 3 * batch
    batches += 1
t1 = time.time()
print(json.dumps({"dtype": dtype, "n": n, "t0": t0, "t1": t1, "batches": batches, "flops": flops,
                  "tflops": flops / (busy_ms * 1e-3) / 1e12, "busy": busy_ms * 1e-3 / (t1 - t0)}), flush=True)
"""


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shared(port, seconds):
    from gpumon.export import promtext

    sizes = (8192, 4096)
    # staggered: the big tenant first, the small (~10 % resident) one `stagger` s later -- the
    # arrival the exporter must not miss (GPUTEST_r02: one tick read 1 active process and gave the
    # big tenant's row the device MFMA util while the small one already held VRAM)
    stagger = 4.0
    spawn = lambda n, secs: subprocess.Popen([sys.executable, "-c", TENANT, "bf16", str(secs), str(n)],
                                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    # processes already holding the GPU (the test runner itself when earlier tests used torch): not
    # tenants -- they make the GPU look shared only for their arrival window (5 ticks / 5 s)
    fam0 = promtext.parse(urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode())
    background = {l["pid"] for _, l, _ in fam0.get("pod_gpu_used_memory", {}).get("samples", [])}
    ts = [spawn(sizes[0], seconds + stagger)]
    t_second = time.time() + stagger
    ticks = []
    deadline = time.time() + seconds + stagger + 60
    while any(t.poll() is None for t in ts) and time.time() < deadline:
        if len(ts) == 1 and time.time() >= t_second:
            ts.append(spawn(sizes[1], seconds))
        fam = promtext.parse(urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode())
        busy = {l["pid"]: v for _, l, v in fam.get("pod_gpu_proc_gfx_util", {}).get("samples", [])}
        cu = {l["pid"]: v for _, l, v in fam.get("pod_gpu_proc_cu_occupancy", {}).get("samples", [])}
        mem = {l["pid"]: v for _, l, v in fam.get("pod_gpu_used_memory", {}).get("samples", [])}
        ticks.append({"t": time.time(),
                      "tflops": (promtext.values(fam, "gpu_mfma_tflops", gpu_id="0", dtype="bf16") or [None])[0],
                      "pod_mfma_util_rows": len(promtext.values(fam, "pod_gpu_mfma_util_percent", gpu_id="0")),
                      "active": (promtext.values(fam, "gpu_active_processes", gpu_id="0") or [None])[0],
                      "vram_rows": sum(1 for p, v in mem.items() if v > 0 and p not in background),
                      # KFD reports host PIDs (not the tenants' pids inside a PID namespace): rows
                      # ranked by busy share, the bigger tenant first
                      "rows": sorted(({"busy": busy.get(p), "cu": cu.get(p), "mib": mem.get(p)} for p in busy
                                      if p not in background),
                                     key=lambda r: -(r["busy"] or 0))})
        time.sleep(0.5)
    res = []
    for t in ts:
        so, se = t.communicate(timeout=120)
        if t.returncode != 0:
            return {"error": se.strip().splitlines()[-1] if se.strip() else f"rc {t.returncode}"}
        res.append(json.loads(so.strip().splitlines()[-1]))
    t0, t1 = max(r["t0"] for r in res) + 2.0, min(r["t1"] for r in res)
    inside = [k for k in ticks if t0 <= k["t"] <= t1]
    wall = [r["flops"] / (r["t1"] - r["t0"]) / 1e12 for r in res]
    tf = [k["tflops"] for k in inside if k["tflops"] is not None]
    rows = [k["rows"] for k in inside if len(k["rows"]) >= 2]
    return {"tenants": [{"n": r["n"], "wall_tflops": round(w, 1), "busy": round(r["busy"], 3)}
                        for r, w in zip(res, wall)],
            "tenants_sum_wall_tflops": round(sum(wall), 1), "ticks_inside": len(inside),
            "exported_tflops_median": round(statistics.median(tf), 1) if tf else None,
            "exported_vs_sum": round(statistics.median(tf) / sum(wall), 4) if tf else None,
            "rows_median": [{"busy": statistics.median([r[i]["busy"] for r in rows if r[i]["busy"] is not None] or [0]),
                             "cu": round(statistics.median([r[i]["cu"] for r in rows if r[i]["cu"] is not None] or [0]), 1)}
                            for i in range(2)] if rows else None,
            "background_pids": sorted(background),
            "pod_mfma_util_rows_max": max((k["pod_mfma_util_rows"] for k in inside), default=None),
            # every scrape (not only those inside the timed window) with two tenants holding VRAM
            "scrapes_two_vram_tenants": sum(1 for k in ticks if k["vram_rows"] >= 2),
            "pod_mfma_rows_while_two_vram_tenants": sum(k["pod_mfma_util_rows"] for k in ticks if k["vram_rows"] >= 2),
            "pod_mfma_rows_single_tenant": sum(k["pod_mfma_util_rows"] for k in ticks if k["vram_rows"] == 1),
            "active_processes": [k["active"] for k in inside]}


def main() -> int:
    from gpumon.export import promtext

    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--dtypes", default="bf16,f16,fp8")
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--shared", action="store_true", help="two concurrent bf16 tenants on one GPU")
    args = ap.parse_args()

    port = _port()
    ex = subprocess.Popen([os.path.join(ROOT, "bin", "gpumon-exporter"), "--backend", "amdsmi", "--interval", "1",
                           "--pmc", "--listen", f"127.0.0.1:{port}", "--no-pod-resources", "--no-cri",
                           "--log-level", "warn"], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    out = {"exporter": "bin/gpumon-exporter --pmc --interval 1", "n": args.n, "runs": {}}
    try:
        time.sleep(3)
        if ex.poll() is not None:
            raise SystemExit("exporter exited: " + ex.stderr.read()[-2000:])
        if args.shared:
            out["shared"] = _shared(port, args.seconds)
            print("shared", out["shared"], file=sys.stderr)
        for dtype in ([] if args.shared else args.dtypes.split(",")):
            tenant = subprocess.Popen([sys.executable, "-c", TENANT, dtype, str(args.seconds), str(args.n)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
            ticks = []
            deadline = time.time() + args.seconds + 60
            while tenant.poll() is None and time.time() < deadline:
                body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
                fam = promtext.parse(body)
                # the tenant's row: the process with the most resident waves (KFD reports host PIDs,
                # which differ from tenant.pid when this runs inside a PID namespace)
                occ = sorted(fam.get("pod_gpu_proc_cu_occupancy", {}).get("samples", []), key=lambda r: -r[2])[:1]
                rows = [r for r in fam.get("pod_gpu_proc_gfx_util", {}).get("samples", [])
                        if occ and r[1].get("pid") == occ[0][1].get("pid")]
                ticks.append({"t": time.time(),
                              "tflops": {k["dtype"]: v for _, k, v in fam.get("gpu_mfma_tflops", {}).get("samples", [])
                                         if k.get("gpu_id") == "0"},
                              "mfma_util": (promtext.values(fam, "gpu_mfma_util_percent", gpu_id="0") or [None])[0],
                              "proc_busy": rows[0][2] if rows else None,
                              "active": (promtext.values(fam, "gpu_active_processes", gpu_id="0") or [None])[0],
                              "proc_cu": occ[0][2] if occ else None})
                time.sleep(1.0)
            so, se = tenant.communicate(timeout=120)
            if tenant.returncode != 0:
                out["runs"][dtype] = {"error": se.strip().splitlines()[-1] if se.strip() else f"rc {tenant.returncode}"}
                print(dtype, out["runs"][dtype], file=sys.stderr)
                continue
            t = json.loads(so.strip().splitlines()[-1])
            # ticks whose whole counted second lies inside the tenant's timed loop
            inside = [k for k in ticks if t["t0"] + 2.0 <= k["t"] <= t["t1"]]
            key = {"bf16": "bf16", "f16": "f16", "fp8": "f8"}[dtype]
            exp_tf = [k["tflops"].get(key) for k in inside if k["tflops"].get(key) is not None]
            util = [k["mfma_util"] for k in inside if k["mfma_util"] is not None]
            busy = [k["proc_busy"] for k in inside if k["proc_busy"] is not None]
            cu = [k["proc_cu"] for k in inside if k["proc_cu"] is not None]
            r = {"tenant_tflops_event_timed": round(t["tflops"], 1), "tenant_busy": round(t["busy"], 3),
                 "ticks_inside": len(inside),
                 "exported_tflops_median": round(statistics.median(exp_tf), 1) if exp_tf else None,
                 "exported_mfma_util_median": round(statistics.median(util), 1) if util else None,
                 "exported_proc_busy_median": round(statistics.median(busy), 1) if busy else None,
                 "exported_proc_cu_median": round(statistics.median(cu), 1) if cu else None,
                 "active_processes": [k["active"] for k in inside]}
            if r["exported_tflops_median"]:
                # the tenant's rate is over its GPU-busy time; the exporter's over wall time
                r["exported_vs_tenant"] = round(r["exported_tflops_median"] / (t["tflops"] * t["busy"]), 4)
            out["runs"][dtype] = r
            print(dtype, r, file=sys.stderr)
            time.sleep(2.0)
    finally:
        ex.terminate()
        ex.wait(20)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())

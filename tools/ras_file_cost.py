"""Per-file cost of the kernel ras/ files on a loaded MI355X (profiles/r1_ras.md "open item").

For each file: the read time when it is the first ras/ read after 200 ms of quiet ("cold") and when
it follows a read of aca_gfx ("warm"). If warm << cold for the ACA files, one firmware query is
shared by a burst and whole passes are cheaper than slices. Load: a bf16 matmul loop on cuda:0.
"""
import glob
import json
import os
import statistics
import threading
import time

import torch


def _read(p):
    t = time.perf_counter()
    with open(p, "rb") as f:
        f.read()
    return (time.perf_counter() - t) * 1e6


def main():
    stop = threading.Event()

    def load():
        a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
        while not stop.is_set():
            for _ in range(20):
                a = (a @ a).clamp_(-1, 1)
            torch.cuda.synchronize()

    th = threading.Thread(target=load, daemon=True)
    th.start()
    time.sleep(2)
    dirs = [d for d in glob.glob("/sys/bus/pci/devices/*/ras") if os.path.exists(d + "/aca_gfx")]
    d = dirs[0]
    files = sorted(f for f in os.listdir(d) if f.startswith("aca_")) + ["event_state", "gpu_vram_bad_pages"]
    out = {"dir": d, "files": {}}
    for f in files:
        cold, warm = [], []
        for _ in range(15):
            time.sleep(0.2)
            cold.append(_read(f"{d}/{f}"))
            time.sleep(0.2)
            _read(f"{d}/aca_gfx")
            warm.append(_read(f"{d}/{f}"))
        out["files"][f] = {"cold_us": round(statistics.median(cold), 1), "warm_us": round(statistics.median(warm), 1)}
    passes = []
    for _ in range(15):
        time.sleep(0.2)
        t = time.perf_counter()
        for f in files:
            _read(f"{d}/{f}")
        passes.append((time.perf_counter() - t) * 1e6)
    out["full_pass_us"] = round(statistics.median(passes), 1)
    stop.set()
    th.join()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

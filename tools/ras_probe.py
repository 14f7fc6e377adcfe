#!/usr/bin/env python3
"""Box probe: what RAS / ECC data an MI355X exposes to a non-root exporter, and what it costs.
sysfs ras/ directory (per-block err_count files, bad pages, features) and the amdsmi ECC calls.
Prints one JSON object."""
import glob
import json
import os
import sys
import time

sys.path.insert(0, "/opt/rocm/share/amd_smi")


def rd(p):
    try:
        with open(p) as f:
            return f.read()
    except Exception as e:  # noqa: BLE001
        return "ERR %r" % (e,)


def main():
    out = {"sysfs": {}, "amdsmi": {}}
    for dev in sorted(glob.glob("/sys/class/drm/card*/device"))[:2]:
        ras = os.path.join(dev, "ras")
        d = {"exists": os.path.isdir(ras), "files": {}}
        if d["exists"]:
            for f in sorted(os.listdir(ras)):
                p = os.path.join(ras, f)
                if os.path.isfile(p):
                    t = time.perf_counter()
                    v = rd(p)
                    d["files"][f] = {"v": v[:300], "us": round((time.perf_counter() - t) * 1e6, 1),
                                     "mode": oct(os.stat(p).st_mode & 0o777)}
        for f in ("mem_info_vram_used", "ecc_count", "umc_err_count"):
            if os.path.exists(os.path.join(dev, f)):
                d["files"]["../" + f] = rd(os.path.join(dev, f))[:200]
        out["sysfs"][os.path.realpath(dev)] = d
    try:
        import amdsmi as A

        A.amdsmi_init(A.AmdSmiInitFlags.INIT_AMD_GPUS)
        h = A.amdsmi_get_processor_handles()[0]
        for name, args in [("amdsmi_get_gpu_ecc_enabled", ()), ("amdsmi_get_gpu_total_ecc_count", ()),
                           ("amdsmi_get_gpu_ras_feature_info", ()), ("amdsmi_get_gpu_bad_page_info", ()),
                           ("amdsmi_get_gpu_bad_page_threshold", ()), ("amdsmi_get_gpu_ecc_status", ())]:
            f = getattr(A, name, None)
            if f is None:
                out["amdsmi"][name] = "MISSING"
                continue
            t = time.perf_counter()
            try:
                r = f(h, *args) if name != "amdsmi_get_gpu_ecc_status" else f(h, A.AmdSmiGpuBlock.UMC)
            except Exception as e:  # noqa: BLE001
                r = "ERR %r" % (e,)
            out["amdsmi"][name] = {"r": str(r)[:400], "ms": round((time.perf_counter() - t) * 1e3, 3)}
        blocks = {}
        for b in A.AmdSmiGpuBlock:
            if b.name in ("INVALID", "RESERVED", "FIRST", "LAST"):
                continue
            t = time.perf_counter()
            try:
                r = A.amdsmi_get_gpu_ecc_count(h, b)
            except Exception as e:  # noqa: BLE001
                r = "ERR %s" % (type(e).__name__,)
            blocks[b.name] = {"r": str(r)[:200], "ms": round((time.perf_counter() - t) * 1e3, 3)}
        out["amdsmi"]["ecc_count"] = blocks
    except Exception as e:  # noqa: BLE001
        out["amdsmi"]["error"] = repr(e)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Box probe for the xGMI peer map: dump amdsmi_get_link_metrics entries (peer BDF,
read/write KB, bit rate, max bandwidth, type) next to the gpu_metrics table's per-slot xGMI
accumulators and link status, twice `--gap` seconds apart, so the entry -> slot pairing can be
read off the accumulator deltas on real hardware.

    python tools/xgmi_link_probe.py [--gap 1.0] > links.json
"""

import argparse
import json
import sys
import time

sys.path.insert(0, "/opt/rocm/share/amd_smi")


def snap(A, h):
    out = {"t": time.time()}
    try:
        lm = A.amdsmi_get_link_metrics(h)
        out["link_metrics"] = lm if isinstance(lm, (dict, list)) else repr(lm)
    except Exception as e:  # NOT_SUPPORTED etc.
        out["link_metrics"] = "ERR %r" % (e,)
    m = A.amdsmi_get_gpu_metrics_info(h)
    out["gm"] = {k: m.get(k) for k in ("xgmi_read_data_acc", "xgmi_write_data_acc", "xgmi_link_status",
                                       "xgmi_link_width", "xgmi_link_speed")}
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gap", type=float, default=1.0)
    args = ap.parse_args()
    import amdsmi as A

    A.amdsmi_init(A.AmdSmiInitFlags.INIT_AMD_GPUS)
    res = []
    try:
        for i, h in enumerate(A.amdsmi_get_processor_handles()):
            a = snap(A, h)
            time.sleep(args.gap)
            b = snap(A, h)
            res.append({"gpu": i, "bdf": A.amdsmi_get_gpu_device_bdf(h), "before": a, "after": b})
    finally:
        A.amdsmi_shut_down()
    print(json.dumps(res, default=str, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())

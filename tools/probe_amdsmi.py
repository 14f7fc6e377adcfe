"""Box probe: time every amdsmi call we plan to use and dump gpu_metrics fields."""
import sys, time
sys.path.insert(0, "/opt/rocm/share/amd_smi")
import amdsmi as A

A.amdsmi_init(A.AmdSmiInitFlags.INIT_AMD_GPUS)
hs = A.amdsmi_get_processor_handles()
print("n handles", len(hs))
for i, h in enumerate(hs):
    print("=== gpu", i)
    for name in ["amdsmi_get_gpu_enumeration_info", "amdsmi_get_gpu_device_uuid", "amdsmi_get_gpu_device_bdf",
                 "amdsmi_get_gpu_asic_info", "amdsmi_get_gpu_vram_usage", "amdsmi_get_gpu_activity",
                 "amdsmi_get_power_info", "amdsmi_get_gpu_process_list", "amdsmi_get_gpu_compute_partition",
                 "amdsmi_get_gpu_memory_partition", "amdsmi_get_link_metrics", "amdsmi_get_gpu_kfd_info",
                 "amdsmi_get_pcie_info", "amdsmi_get_violation_status", "amdsmi_get_gpu_board_info",
                 "amdsmi_get_gpu_driver_info", "amdsmi_get_gpu_vram_info", "amdsmi_get_energy_count"]:
        f = getattr(A, name, None)
        if f is None:
            print(name, "MISSING"); continue
        t = time.perf_counter()
        try:
            r = f(h)
        except Exception as e:
            r = "ERR %r" % (e,)
        print(name, "%.3f ms" % ((time.perf_counter() - t) * 1e3), r)
    t = time.perf_counter()
    for _ in range(20):
        m = A.amdsmi_get_gpu_metrics_info(h)
    print("gpu_metrics x20 avg %.3f ms" % ((time.perf_counter() - t) * 1e3 / 20))
    for k, v in m.items():
        print("  ", k, v)
    # refresh rate of the firmware table
    ts = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        mm = A.amdsmi_get_gpu_metrics_info(h)
        ts.append((mm.get("firmware_timestamp"), mm.get("system_clock_counter")))
    print("distinct fw ts in 1s:", len(set(x[0] for x in ts)), "calls", len(ts), "distinct sys", len(set(x[1] for x in ts)))
    for ct in ["GFX", "MEM", "SOC"]:
        try:
            print("clock", ct, A.amdsmi_get_clock_info(h, getattr(A.AmdSmiClkType, ct)))
        except Exception as e:
            print("clock", ct, "ERR", e)
    for tt in ["EDGE", "HOTSPOT", "VRAM"]:
        try:
            print("temp", tt, A.amdsmi_get_temp_metric(h, getattr(A.AmdSmiTemperatureType, tt), A.AmdSmiTemperatureMetric.CURRENT))
        except Exception as e:
            print("temp", tt, "ERR", e)
A.amdsmi_shut_down()

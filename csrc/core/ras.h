// RAS / ECC readers shared by the backends.
//
// The reference exports no device-health data (/root/reference/gpu.py:104-109 queries utilisation
// and memory only). A production MI355X exporter must surface HBM / GFX / xGMI error counters:
// the kernel publishes them per RAS block under /sys/bus/pci/devices/<bdf>/ras/ as plain text
// (measured on MI355X, profiles/r1_ras.md):
//   aca_<block>         "ue: N\nce: N\nde: N\n"   (ACA, MI300 / MI355X: umc gfx sdma mmhub xgmi_wafl vcn jpeg)
//   <block>_err_count   "ue: N\nce: N\n"          (older ASICs / kernels)
//   event_state         fatal-error and poison creation / consumption counters
//   gpu_vram_bad_pages  one "0xPFN : 0xSIZE : R|P|F" line per retired / pending page
// Files are world-readable (0444) and cost 10-130 us each, so a non-root exporter reads them every
// `ras_every` ticks without libamd_smi.
#pragma once

#include <string>

#include "sample.h"

namespace gpumon {

// "ue: 1\nce: 2\n[de: 3\n]" -> counts; false if neither ue nor ce is present.
bool parse_err_count(const std::string& text, RasCount* out);

// "Fatal Error: count:N, ..." / "Poison Creation: count:N" / "Poison Consumption: count:N".
void parse_event_state(const std::string& text, RasSample* out);

// Number of page records in gpu_vram_bad_pages.
int count_bad_pages(const std::string& text);

// Reads <sys_root>/bus/pci/devices/<bdf>/ras; false (out untouched) when the directory has no
// error-count files (RAS disabled, VM guest, or no such device).
bool read_ras_sysfs(const std::string& sys_root, const std::string& bdf, RasSample* out);

}  // namespace gpumon

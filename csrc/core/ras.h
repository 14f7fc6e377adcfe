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
// Files are world-readable (0444) and cost 10-130 us each, so a non-root exporter reads them without
// libamd_smi, one slice per tick (RasSysfsReader), a full pass every `ras_every` ticks.
#pragma once

#include <algorithm>
#include <string>
#include <utility>
#include <vector>

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

// Incremental reader for one device. A full refresh costs 0.24 ms idle and ~0.5 ms under load on
// MI355X (aca_gfx alone 0.13 ms: the driver queries firmware per file), which made every
// `ras_every`-th tick the slowest. read(slice, nslices) re-reads only the files whose index is
// slice (mod nslices) and merges them into the last reading, so a full pass is spread over
// nslices ticks. The first call always reads everything.
class RasSysfsReader {
 public:
  RasSysfsReader(const std::string& sys_root, const std::string& bdf);
  // false (out untouched) when the directory has no error-count files. A due file that fails to
  // read keeps its last value and counts in out->stale_items (the caller reports the call failed).
  bool read(int slice, int nslices, RasSample* out);
  int items() const { return static_cast<int>(files_.size()) + 2; }  // + event_state, bad pages
  // The last directory scan found no error-count files (RAS off, VM guest, no such device): the
  // only reason to stop reading. A false read() with files listed is transient (retry with backoff).
  bool missing() const { return listed_ && files_.empty(); }

 private:
  bool list();
  std::string dir_;
  bool listed_ = false;
  std::vector<std::pair<std::string, std::string>> files_;  // (block, file), one per block
  bool has_events_ = false, has_bad_pages_ = false;         // listed at the last directory scan
  RasSample cur_;
};

// Backoff after transient RAS read failures: skip 1, 3, 7, ... up to 63 refreshes, reset on success.
struct RasRetry {
  int fails = 0, skip = 0;
  bool due() {
    if (skip > 0) {
      --skip;
      return false;
    }
    return true;
  }
  void failed() {
    ++fails;
    skip = (1 << std::min(fails, 6)) - 1;
  }
  void ok() { fails = skip = 0; }
};

}  // namespace gpumon

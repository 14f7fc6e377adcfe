// Fake librocm_smi64 for CPU tests of the REAL RocmSmiBackend through its dlopen table (the
// rocm_smi_lib fallback of SURVEY.md D6). Same MI355X-shaped firmware table as the fake
// libamd_smi (fake_metrics.h). Scripted by environment variables read at rsmi_init():
//   FAKE_RSMI_GPUS=N          number of GPUs (default 2)
//   FAKE_RSMI_PROCS=N         GPU processes per device (default 1; >64 exercises the resize path)
//   FAKE_RSMI_FAIL_METRICS=K  gpu_metrics fails (RSMI_STATUS_BUSY) on device K
//   FAKE_RSMI_INIT_FAIL=1     rsmi_init returns RSMI_STATUS_INIT_ERROR
//   FAKE_RSMI_NO_METRICS=1    gpu_metrics NOT_SUPPORTED (exercises the busy_percent fallback)
#include <rocm_smi/rocm_smi.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "fake_metrics.h"

namespace {
int g_gpus = 2, g_procs = 1, g_fail_metrics = -1;
bool g_no_metrics = false;
std::atomic<uint64_t> g_calls[64];
int env_int(const char* k, int d) {
  const char* v = getenv(k);
  return v ? atoi(v) : d;
}
bool bad(uint32_t dv) { return dv >= static_cast<uint32_t>(g_gpus); }
uint32_t pid_of(uint32_t dv, uint32_t i) { return 200000 + 1000 * dv + i; }
}  // namespace

extern "C" {

rsmi_status_t rsmi_init(uint64_t) {
  if (env_int("FAKE_RSMI_INIT_FAIL", 0)) return RSMI_STATUS_INIT_ERROR;
  g_gpus = env_int("FAKE_RSMI_GPUS", 2);
  g_procs = env_int("FAKE_RSMI_PROCS", 1);
  g_fail_metrics = env_int("FAKE_RSMI_FAIL_METRICS", -1);
  g_no_metrics = env_int("FAKE_RSMI_NO_METRICS", 0) != 0;
  for (auto& c : g_calls) c = 0;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_shut_down(void) { return RSMI_STATUS_SUCCESS; }

rsmi_status_t rsmi_num_monitor_devices(uint32_t* n) {
  *n = static_cast<uint32_t>(g_gpus);
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_version_get(rsmi_version_t* v) {
  v->major = 77;
  v->minor = 1;
  v->patch = 2;
  v->build = "fake";
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_name_get(uint32_t dv, char* name, size_t len) {
  if (bad(dv)) return RSMI_STATUS_INVALID_ARGS;
  snprintf(name, len, "AMD Instinct MI355 OAM (fake rocm_smi)");
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_serial_number_get(uint32_t dv, char* s, uint32_t len) {
  snprintf(s, len, "0xFAKE%u", dv);
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_pci_id_get(uint32_t dv, uint64_t* bdfid) {
  // domain 0, bus 0x26 + 0x20*dv, device 0, function 0
  *bdfid = static_cast<uint64_t>(0x26 + 0x20 * dv) << 8;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_unique_id_get(uint32_t dv, uint64_t* id) {
  *id = 0x8bff75a3cf9c0000ull + dv;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_compute_partition_get(uint32_t, char* p, uint32_t len) {
  snprintf(p, len, "SPX");
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_memory_partition_get(uint32_t, char* p, uint32_t len) {
  snprintf(p, len, "NPS1");
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_partition_id_get(uint32_t, uint32_t* id) {
  *id = 0;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_power_cap_get(uint32_t, uint32_t, uint64_t* cap) {
  *cap = 1400000000ull;  // microwatts
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_energy_count_get(uint32_t, uint64_t* e, float* res, uint64_t* ts) {
  *e = 1000;
  *res = 15.3f;
  *ts = 0;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_memory_total_get(uint32_t dv, rsmi_memory_type_t t, uint64_t* total) {
  if (bad(dv) || t != RSMI_MEM_TYPE_VRAM) return RSMI_STATUS_NOT_SUPPORTED;
  *total = 288ull << 30;  // 288 GiB
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_memory_usage_get(uint32_t dv, rsmi_memory_type_t t, uint64_t* used) {
  if (bad(dv) || t != RSMI_MEM_TYPE_VRAM) return RSMI_STATUS_NOT_SUPPORTED;
  *used = (283ull + 1024ull * dv) << 20;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_busy_percent_get(uint32_t dv, uint32_t* p) {
  *p = 11 + dv;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_memory_busy_percent_get(uint32_t, uint32_t* p) {
  *p = 5;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_gpu_metrics_info_get(uint32_t dv, rsmi_gpu_metrics_t* m) {
  if (bad(dv)) return RSMI_STATUS_INVALID_ARGS;
  if (g_no_metrics) return RSMI_STATUS_NOT_SUPPORTED;
  if (static_cast<int>(dv) == g_fail_metrics) return RSMI_STATUS_BUSY;
  fake::fill_metrics(m, static_cast<int>(dv), ++g_calls[dv]);
  return RSMI_STATUS_SUCCESS;
}

// All compute processes on the node (each GPU runs g_procs of its own).
rsmi_status_t rsmi_compute_process_info_get(rsmi_process_info_t* procs, uint32_t* num) {
  const uint32_t total = static_cast<uint32_t>(g_gpus * g_procs);
  if (!procs) {
    *num = total;
    return RSMI_STATUS_SUCCESS;
  }
  const uint32_t cap = *num;
  uint32_t k = 0;
  for (uint32_t d = 0; d < static_cast<uint32_t>(g_gpus); ++d)
    for (uint32_t i = 0; i < static_cast<uint32_t>(g_procs); ++i, ++k)
      if (k < cap) {
        memset(&procs[k], 0, sizeof procs[k]);
        procs[k].process_id = pid_of(d, i);
      }
  *num = total;  // like rocm_smi_lib: the full count, so callers can resize
  return total > cap ? RSMI_STATUS_INSUFFICIENT_SIZE : RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_compute_process_info_by_device_get(uint32_t pid, uint32_t dv, rsmi_process_info_t* p) {
  if (bad(dv)) return RSMI_STATUS_INVALID_ARGS;
  const uint32_t base = pid_of(dv, 0);
  if (pid < base || pid >= base + static_cast<uint32_t>(g_procs)) return RSMI_STATUS_NOT_FOUND;
  const uint32_t i = pid - base;
  memset(p, 0, sizeof *p);
  p->process_id = pid;
  p->vram_usage = (1ull << 30) * (i + 1);
  p->cu_occupancy = 64;
  return RSMI_STATUS_SUCCESS;
}

}  // extern "C"

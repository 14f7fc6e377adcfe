// Fake libamd_smi for CPU tests of the REAL AmdSmiBackend ("a C++ fake with the
// same dlopen function-table signature, so the C++ sampler is testable without ROCm").
//
// Exports the amdsmi C API subset gpumon resolves, with MI355X-shaped values (gpu_metrics v1.8:
// 8 XCC, 7 xGMI peer links + N/A slot 0, 288 GiB HBM3E, N/A edge temperature, 15.3 uJ energy
// resolution). Behaviour is scripted by environment variables read at amdsmi_init():
//   FAKE_AMDSMI_GPUS=N            number of GPUs (default 2)
//   FAKE_AMDSMI_PROCS=N           GPU processes per device (default 1; >64 exercises the
//                                 OUT_OF_RESOURCES resize path)
//   FAKE_AMDSMI_FAIL_METRICS=K    gpu_metrics fails (AMDSMI_STATUS_BUSY) on device K
//   FAKE_AMDSMI_INIT_FAIL=1       amdsmi_init returns AMDSMI_STATUS_INIT_ERROR
//   FAKE_AMDSMI_NO_METRICS=1      gpu_metrics NOT_SUPPORTED (exercises the activity/power fallback)
//   FAKE_AMDSMI_CPX=1             CPX compute partitioning: every socket exposes 8 logical GPUs (one
//                                 XCD each); partition k's busy counters live in xcp_stats[k]
//   FAKE_AMDSMI_ECC_UMC_CE=N      correctable UMC errors on device 0 (other ECC blocks: 0; only UMC,
//                                 SDMA, GFX, MMHUB, XGMI_WAFL answer, as measured on MI355X)
//   FAKE_AMDSMI_BAD_PAGES=N       bad-page records on device 0
//   FAKE_AMDSMI_LINK_SLOTS=a,b,.. the gpu_metrics xGMI slot each amdsmi_get_link_metrics entry
//                                 describes, in entry order (0 = self: no peer). Default
//                                 0,1,2,3,4,5,6,7: what ROCm 7.2 returns on MI355X (self + 7 peers,
//                                 positional, counters equal to the table's)
//   FAKE_AMDSMI_LINK_NUM=N        num_links reported (default: entries - 1, i.e. 7 for 8 entries,
//                                 as measured: the count leaves out the self entry it fills)
//   FAKE_AMDSMI_UNSUPPORTED=a,b   these calls return NOT_SUPPORTED (activity, power, vram, procs,
//                                 links): firmware / partition modes without the query
//   FAKE_AMDSMI_BUSY=a,b          these calls fail with AMDSMI_STATUS_BUSY (a transient error)
// Counters advance deterministically per call so rates are checkable.
#include <amd_smi/amdsmi.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fake_metrics.h"

namespace {
int g_gpus = 2, g_procs = 1, g_fail_metrics = -1, g_parts = 1;
std::vector<int> g_link_slots;
int g_link_num = -1;
bool g_no_metrics = false;
std::string g_unsupported, g_busy;  // ",name1,name2,"
std::vector<uintptr_t> g_handles;
std::atomic<uint64_t> g_calls[64];
int env_int(const char* k, int d) {
  const char* v = getenv(k);
  return v ? atoi(v) : d;
}
std::string env_list(const char* k) {
  const char* v = getenv(k);
  return std::string(",") + (v ? v : "") + ",";
}
// NOT_SUPPORTED / BUSY when the call is listed in FAKE_AMDSMI_UNSUPPORTED / FAKE_AMDSMI_BUSY.
amdsmi_status_t scripted(const char* call) {
  const std::string k = std::string(",") + call + ",";
  if (g_unsupported.find(k) != std::string::npos) return AMDSMI_STATUS_NOT_SUPPORTED;
  if (g_busy.find(k) != std::string::npos) return AMDSMI_STATUS_BUSY;
  return AMDSMI_STATUS_SUCCESS;
}
int dev_of(amdsmi_processor_handle h) {
  uintptr_t x = reinterpret_cast<uintptr_t>(h);
  return (x >= 0x1000 && x < 0x1000 + static_cast<uintptr_t>(g_gpus * g_parts)) ? static_cast<int>(x - 0x1000) : -1;
}
int part_of(int d) { return d % g_parts; }
int sock_of(int d) { return d / g_parts; }
}  // namespace

extern "C" {

amdsmi_status_t amdsmi_init(uint64_t) {
  if (env_int("FAKE_AMDSMI_INIT_FAIL", 0)) return AMDSMI_STATUS_INIT_ERROR;
  g_gpus = env_int("FAKE_AMDSMI_GPUS", 2);
  g_procs = env_int("FAKE_AMDSMI_PROCS", 1);
  g_fail_metrics = env_int("FAKE_AMDSMI_FAIL_METRICS", -1);
  g_no_metrics = env_int("FAKE_AMDSMI_NO_METRICS", 0) != 0;
  g_unsupported = env_list("FAKE_AMDSMI_UNSUPPORTED");
  g_busy = env_list("FAKE_AMDSMI_BUSY");
  g_parts = env_int("FAKE_AMDSMI_CPX", 0) ? 8 : 1;
  g_link_slots = {0, 1, 2, 3, 4, 5, 6, 7};
  g_link_num = env_int("FAKE_AMDSMI_LINK_NUM", -1);
  if (const char* ls = getenv("FAKE_AMDSMI_LINK_SLOTS")) {
    g_link_slots.clear();
    for (const char* p = ls; *p;) {
      char* end = nullptr;
      const long v = strtol(p, &end, 10);
      if (end == p) break;
      g_link_slots.push_back(static_cast<int>(v));
      p = *end == ',' ? end + 1 : end;
    }
  }
  g_handles.clear();
  for (int i = 0; i < g_gpus * g_parts; ++i) g_handles.push_back(0x1000 + i);
  for (auto& c : g_calls) c = 0;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_shut_down(void) { return AMDSMI_STATUS_SUCCESS; }

amdsmi_status_t amdsmi_get_lib_version(amdsmi_version_t* v) {
  v->major = 99;
  v->minor = 0;
  v->release = 1;
  v->build = "fake";
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* count, amdsmi_socket_handle* socks) {
  // one socket per GPU, as on MI355X OAM platforms
  if (!socks) {
    *count = static_cast<uint32_t>(g_gpus);
    return AMDSMI_STATUS_SUCCESS;
  }
  for (uint32_t i = 0; i < *count && i < static_cast<uint32_t>(g_gpus); ++i)
    socks[i] = reinterpret_cast<amdsmi_socket_handle>(0x100 + i);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle s, uint32_t* count,
                                             amdsmi_processor_handle* hs) {
  const uintptr_t si = reinterpret_cast<uintptr_t>(s) - 0x100;
  if (!hs) {
    *count = static_cast<uint32_t>(g_parts);
    return AMDSMI_STATUS_SUCCESS;
  }
  // reverse socket order on purpose: the backend must sort by hip_id
  const int sock = g_gpus - 1 - static_cast<int>(si);
  for (int k = 0; k < g_parts && k < static_cast<int>(*count); ++k)
    hs[k] = reinterpret_cast<amdsmi_processor_handle>(g_handles[sock * g_parts + k]);
  *count = static_cast<uint32_t>(g_parts);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_type(amdsmi_processor_handle, processor_type_t* t) {
  *t = AMDSMI_PROCESSOR_TYPE_AMD_GPU;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_enumeration_info(amdsmi_processor_handle h, amdsmi_enumeration_info_t* e) {
  int d = dev_of(h);
  if (d < 0) return AMDSMI_STATUS_INVAL;
  memset(e, 0, sizeof *e);
  e->hip_id = d;
  e->drm_card = 24 + d;
  e->drm_render = 152 + d;
  e->hsa_id = 2 + d;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_uuid(amdsmi_processor_handle h, unsigned int* len, char* uuid) {
  int d = dev_of(h);
  snprintf(uuid, *len, "8bff75a3-0000-1000-80d2-cf9ceac6%04x", d);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle h, amdsmi_bdf_t* b) {
  int d = dev_of(h);
  b->as_uint = 0;
  b->bus_number = 0x26 + 0x20 * sock_of(d);
  b->function_number = part_of(d);  // CPX partitions: one PCI function each
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_asic_info(amdsmi_processor_handle, amdsmi_asic_info_t* a) {
  memset(a, 0, sizeof *a);
  strcpy(a->market_name, "AMD Instinct MI355 OAM (fake amdsmi)");
  strcpy(a->asic_serial, "0xFAKE");
  a->num_of_compute_units = 256;
  a->target_graphics_version = 0x950;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_kfd_info(amdsmi_processor_handle h, amdsmi_kfd_info_t* k) {
  k->kfd_id = 36622 + dev_of(h);
  k->node_id = 2 + dev_of(h);
  k->current_partition_id = static_cast<uint32_t>(part_of(dev_of(h)));
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_driver_info(amdsmi_processor_handle, amdsmi_driver_info_t* i) {
  memset(i, 0, sizeof *i);
  strcpy(i->driver_name, "amdgpu");
  // FAKE_AMDSMI_DRIVER_VERSION: what libamd_smi returned on the pool's MI355X boxes (in-kernel
  // amdgpu: /proc/version with its spaces removed, profiles/data/r4/cm_base.prom:24)
  const char* v = getenv("FAKE_AMDSMI_DRIVER_VERSION");
  snprintf(i->driver_version, sizeof i->driver_version, "%s", v ? v : "6.18.0-fake");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_compute_partition(amdsmi_processor_handle, char* p, uint32_t len) {
  snprintf(p, len, g_parts > 1 ? "CPX" : "SPX");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_memory_partition(amdsmi_processor_handle, char* p, uint32_t len) {
  snprintf(p, len, "NPS1");
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_power_info(amdsmi_processor_handle, amdsmi_power_info_t* p) {
  if (amdsmi_status_t st = scripted("power"); st != AMDSMI_STATUS_SUCCESS) return st;
  memset(p, 0xFF, sizeof *p);
  p->socket_power = 250;
  p->current_socket_power = 250;
  p->power_limit = 1400000000;  // ROCm 7.2 reports microwatts here (measured on MI355X)
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_energy_count(amdsmi_processor_handle, uint64_t* e, float* res, uint64_t* ts) {
  *e = 1000;
  *res = 15.3f;
  *ts = 0;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_vram_usage(amdsmi_processor_handle h, amdsmi_vram_usage_t* v) {
  if (amdsmi_status_t st = scripted("vram"); st != AMDSMI_STATUS_SUCCESS) return st;
  v->vram_total = 294896;
  v->vram_used = 283 + 1024 * dev_of(h);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_activity(amdsmi_processor_handle h, amdsmi_engine_usage_t* u) {
  if (amdsmi_status_t st = scripted("activity"); st != AMDSMI_STATUS_SUCCESS) return st;
  memset(u, 0, sizeof *u);
  u->gfx_activity = 11 + dev_of(h);
  u->umc_activity = 5;
  u->mm_activity = 0xFFFFFFFF;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_metrics_info(amdsmi_processor_handle h, amdsmi_gpu_metrics_t* m) {
  int d = dev_of(h);
  if (g_no_metrics) return AMDSMI_STATUS_NOT_SUPPORTED;
  if (d == g_fail_metrics) return AMDSMI_STATUS_BUSY;
  const uint64_t n = ++g_calls[d];  // advances once per tick
  fake::fill_metrics(m, sock_of(d), n);
  if (g_parts > 1) {
    // CPX: every logical GPU returns the socket table; XCP k holds partition k's single XCC
    const int k = part_of(d);
    memset(m->xcp_stats, 0xFF, sizeof m->xcp_stats);
    m->xcp_stats[k].gfx_busy_inst[0] = static_cast<uint32_t>(10 * k + 5);
    m->xcp_stats[k].gfx_busy_acc[0] = n * (10 * k + 5) * 1000;
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_process_list(amdsmi_processor_handle h, uint32_t* max, amdsmi_proc_info_t* list) {
  if (amdsmi_status_t st = scripted("procs"); st != AMDSMI_STATUS_SUCCESS) return st;
  int d = dev_of(h);
  const uint32_t n = static_cast<uint32_t>(g_procs);
  const uint32_t cap = *max;
  for (uint32_t i = 0; i < n && i < cap; ++i) {
    amdsmi_proc_info_t& p = list[i];
    memset(&p, 0, sizeof p);
    snprintf(p.name, sizeof p.name, "worker-%u", i);
    p.pid = 100000 + 1000 * d + i;
    p.mem = (1ull << 30) * (i + 1);
    p.memory_usage.vram_mem = (1ull << 30) * (i + 1);
    p.engine_usage.gfx = g_calls[d] * 500000000ull;  // 50 % of a 1 s tick
    p.cu_occupancy = 64;
  }
  *max = n;
  return n > cap ? AMDSMI_STATUS_OUT_OF_RESOURCES : AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_link_metrics(amdsmi_processor_handle h, amdsmi_link_metrics_t* lm) {
  if (amdsmi_status_t st = scripted("links"); st != AMDSMI_STATUS_SUCCESS) return st;
  const int d = dev_of(h);
  if (d < 0) return AMDSMI_STATUS_INVAL;
  memset(lm, 0, sizeof *lm);
  const uint64_t n = g_calls[d];  // the table this tick's gpu_metrics call returned
  lm->num_links = static_cast<uint32_t>(g_link_num >= 0 ? g_link_num : std::max<int>(0, g_link_slots.size() - 1));
  for (size_t j = 0; j < g_link_slots.size(); ++j) {
    const int k = g_link_slots[j];  // slot k of the table: k GB/s read, k/2 GB/s write (fake_metrics.h)
    auto& L = lm->links[j];
    if (k == 0) {
      L.bdf.as_uint = ~0ull;  // self / unknown, as on MI355X
    } else {
      L.bdf.bus_number = 0x40 + k;
      L.read = n * 1000000ull * k;
      L.write = n * 500000ull * k;
    }
    L.bit_rate = 38;
    L.max_bandwidth = 608;
    L.link_type = AMDSMI_LINK_TYPE_XGMI;
  }
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_ecc_count(amdsmi_processor_handle h, amdsmi_gpu_block_t block,
                                         amdsmi_error_count_t* ec) {
  const int d = dev_of(h);
  if (d < 0 || !ec) return AMDSMI_STATUS_INVAL;
  switch (block) {
    case AMDSMI_GPU_BLOCK_UMC: case AMDSMI_GPU_BLOCK_SDMA: case AMDSMI_GPU_BLOCK_GFX:
    case AMDSMI_GPU_BLOCK_MMHUB: case AMDSMI_GPU_BLOCK_XGMI_WAFL: break;
    default: return AMDSMI_STATUS_API_FAILED;  // what libamd_smi answers for untracked blocks
  }
  memset(ec, 0, sizeof *ec);
  if (d == 0 && block == AMDSMI_GPU_BLOCK_UMC) ec->correctable_count = env_int("FAKE_AMDSMI_ECC_UMC_CE", 0);
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_bad_page_info(amdsmi_processor_handle h, uint32_t* num_pages,
                                             amdsmi_retired_page_record_t* info) {
  const int d = dev_of(h);
  if (d < 0 || !num_pages) return AMDSMI_STATUS_INVAL;
  *num_pages = d == 0 ? env_int("FAKE_AMDSMI_BAD_PAGES", 0) : 0;
  (void)info;
  return AMDSMI_STATUS_SUCCESS;
}

}  // extern "C"

// Which HSA step pins the ~173 MB host blocks? Brings the probe's raw-HSA path up one step at a time
// (hsa_init -> executable load -> hsa_queue_create -> first dispatch) and prints, after each step,
// the process's resident memory and its anonymous mappings of >= 100 MB resident (smaps).
//
//   make bin/hsa_stages       (g++, -lhsa-runtime64)
//   bin/hsa_stages build/obj/hip/probe_gfx950.hsaco     # one JSON line per step
//
// Bounded: one dispatch of gpumon_probe_reset (one workgroup, 4 counters), waited for <= 10 s.
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

static void mem(const char* step) {
  std::ifstream f("/proc/self/smaps");
  std::string line;
  long rss_kb = 0, kb = 0;
  bool anon = false;
  std::vector<long> big;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    std::string a;
    is >> a;
    if (a.find('-') != std::string::npos && a.back() != ':') {
      std::string perms, off, dev, inode, path;
      is >> perms >> off >> dev >> inode >> path;
      anon = path.empty();
    } else if (a == "Rss:") {
      is >> kb;
      rss_kb += kb;
      if (anon && kb >= (100 << 10)) big.push_back(kb >> 10);
    }
  }
  printf("{\"step\": \"%s\", \"rss_mb\": %ld, \"anon_blocks_ge_100mb\": [", step, rss_kb >> 10);
  for (size_t i = 0; i < big.size(); ++i) printf("%s%ld", i ? ", " : "", big[i]);
  printf("]}\n");
  fflush(stdout);
}

#define CK(x)                                                   \
  do {                                                          \
    hsa_status_t s_ = (x);                                      \
    if (s_ != HSA_STATUS_SUCCESS) {                             \
      fprintf(stderr, "%s failed: %d\n", #x, static_cast<int>(s_)); \
      return 1;                                                 \
    }                                                           \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: hsa_stages CODE_OBJECT\n");
    return 2;
  }
  std::ifstream co(argv[1], std::ios::binary);
  std::string bytes((std::istreambuf_iterator<char>(co)), std::istreambuf_iterator<char>());
  mem("start");
  CK(hsa_init());
  mem("hsa_init");
  hsa_agent_t gpu{}, cpu{};
  hsa_agent_t agents[2];
  memset(agents, 0, sizeof agents);
  hsa_iterate_agents(
      [](hsa_agent_t a, void* p) {
        hsa_device_type_t t;
        hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
        auto* g = static_cast<hsa_agent_t*>(p);
        if (t == HSA_DEVICE_TYPE_GPU && g[0].handle == 0) g[0] = a;
        if (t == HSA_DEVICE_TYPE_CPU && g[1].handle == 0) g[1] = a;
        return HSA_STATUS_SUCCESS;
      },
      agents);
  gpu = agents[0];
  cpu = agents[1];
  if (!gpu.handle) {
    fprintf(stderr, "no GPU agent\n");
    return 1;
  }
  // the memory pools of both agents (segment / global flags / size), for the kernarg placement
  for (int ai = 0; ai < 2; ++ai)
    hsa_amd_agent_iterate_memory_pools(
        agents[ai],
        [](hsa_amd_memory_pool_t pool, void* d) {
          hsa_amd_segment_t seg;
          uint32_t flags = 0;
          size_t size = 0;
          bool alloc = false;
          hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
          hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
          hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SIZE, &size);
          hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
          printf("{\"pool_of\": \"%s\", \"segment\": %d, \"global_flags\": %u, \"size_gb\": %.1f, \"alloc\": %d}\n",
                 *static_cast<int*>(d) == 0 ? "gpu" : "cpu", static_cast<int>(seg), flags, size / 1e9, alloc ? 1 : 0);
          return HSA_STATUS_SUCCESS;
        },
        &ai);
  hsa_code_object_reader_t rd;
  hsa_executable_t exe;
  CK(hsa_code_object_reader_create_from_memory(bytes.data(), bytes.size(), &rd));
  CK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  CK(hsa_executable_load_agent_code_object(exe, gpu, rd, nullptr, nullptr));
  CK(hsa_executable_freeze(exe, nullptr));
  mem("executable_loaded");
  hsa_executable_symbol_t sym;
  uint64_t kobj = 0;
  CK(hsa_executable_get_symbol_by_name(exe, "gpumon_probe_reset.kd", &gpu, &sym));
  CK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
  // memory: counters in VRAM, kernargs in the kernarg pool
  struct P {
    uint32_t want;
    hsa_amd_memory_pool_t pool;
    bool found;
  };
  auto find = [](hsa_agent_t ag, uint32_t want) {
    P p{want, {}, false};
    hsa_amd_agent_iterate_memory_pools(
        ag,
        [](hsa_amd_memory_pool_t pool, void* d) {
          auto* q = static_cast<P*>(d);
          hsa_amd_segment_t seg;
          uint32_t flags = 0;
          bool alloc = false;
          hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
          hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
          hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
          if (!q->found && seg == HSA_AMD_SEGMENT_GLOBAL && alloc && (flags & q->want) == q->want) {
            q->pool = pool;
            q->found = true;
          }
          return HSA_STATUS_SUCCESS;
        },
        &p);
    return p;
  };
  P vram = find(gpu, HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED);
  P karg = find(cpu, HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT);
  if (!vram.found || !karg.found) {
    fprintf(stderr, "pools missing\n");
    return 1;
  }
  void *counters = nullptr, *ka = nullptr;
  CK(hsa_amd_memory_pool_allocate(vram.pool, 16, 0, &counters));
  CK(hsa_amd_memory_pool_allocate(karg.pool, 256, 0, &ka));
  CK(hsa_amd_agents_allow_access(1, &gpu, nullptr, ka));
  mem("memory_allocated");
  hsa_queue_t* q = nullptr;
  uint32_t qmin = 64;
  hsa_agent_get_info(gpu, HSA_AGENT_INFO_QUEUE_MIN_SIZE, &qmin);
  CK(hsa_queue_create(gpu, qmin < 64 ? 64 : qmin, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  mem("queue_created");
  hsa_signal_t done;
  CK(hsa_signal_create(1, 0, nullptr, &done));
  const uint32_t n = 4;
  memcpy(static_cast<char*>(ka), &counters, 8);
  memcpy(static_cast<char*>(ka) + 8, &n, 4);
  const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
  hsa_queue_store_write_index_relaxed(q, idx + 1);
  auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
  memset(reinterpret_cast<char*>(pkt) + 4, 0, sizeof(*pkt) - 4);
  pkt->workgroup_size_x = 64;
  pkt->workgroup_size_y = pkt->workgroup_size_z = 1;
  pkt->grid_size_x = 64;
  pkt->grid_size_y = pkt->grid_size_z = 1;
  pkt->kernel_object = kobj;
  pkt->kernarg_address = ka;
  pkt->completion_signal = done;
  const uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                       (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                       (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), hdr | (1u << 16), __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(10);
  while (hsa_signal_load_scacquire(done) > 0) {
    if (std::chrono::steady_clock::now() > t_end) {
      fprintf(stderr, "dispatch did not complete in 10 s\n");
      return 1;  // the queue and memory stay allocated: nothing is freed under a running kernel
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  mem("first_dispatch_done");
  hsa_signal_destroy(done);
  hsa_queue_destroy(q);
  mem("queue_destroyed");
  hsa_amd_memory_pool_free(counters);
  hsa_amd_memory_pool_free(ka);
  hsa_executable_destroy(exe);
  hsa_code_object_reader_destroy(rd);
  hsa_shut_down();
  return 0;
}

// K1 probe over the raw HSA runtime (probe_hsa.h).
#include "probe_hsa.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>

// The unbundled gfx950 code object of csrc/hip/probe_co.hip (Makefile: GPUMON_PROBE_HSACO).
asm(".section .rodata\n"
    ".p2align 12\n"
    ".global gpumon_probe_hsaco_begin\n"
    ".hidden gpumon_probe_hsaco_begin\n"
    "gpumon_probe_hsaco_begin:\n"
    ".incbin \"" GPUMON_PROBE_HSACO "\"\n"
    ".global gpumon_probe_hsaco_end\n"
    ".hidden gpumon_probe_hsaco_end\n"
    "gpumon_probe_hsaco_end:\n"
    ".previous\n");
extern "C" const char gpumon_probe_hsaco_begin[];
extern "C" const char gpumon_probe_hsaco_end[];

namespace gpumon_hsa {

namespace {

int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void ck(hsa_status_t s, const char* what) {
  if (s == HSA_STATUS_SUCCESS) return;
  const char* msg = nullptr;
  hsa_status_string(s, &msg);
  throw std::runtime_error(std::string(what) + ": " + (msg ? msg : "HSA error"));
}

struct Agents {
  bool up = false;
  hsa_agent_t cpu{};
  std::vector<hsa_agent_t> gpus;
};

Agents& agents() {
  static Agents a;
  static std::once_flag once;
  std::call_once(once, [] {
    if (hsa_init() != HSA_STATUS_SUCCESS) return;  // stays up for the life of the process
    hsa_iterate_agents(
        [](hsa_agent_t ag, void* p) {
          auto* A = static_cast<Agents*>(p);
          hsa_device_type_t t;
          if (hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
          if (t == HSA_DEVICE_TYPE_GPU) A->gpus.push_back(ag);
          else if (t == HSA_DEVICE_TYPE_CPU && A->cpu.handle == 0) A->cpu = ag;
          return HSA_STATUS_SUCCESS;
        },
        &a);
    a.up = a.cpu.handle != 0;
  });
  return a;
}

// First pool of `agent` in the global segment whose flags contain `want`, runtime-allocatable.
hsa_amd_memory_pool_t find_pool(hsa_agent_t agent, uint32_t want) {
  struct Q {
    uint32_t want;
    hsa_amd_memory_pool_t pool{};
    bool found = false;
  } q{want};
  hsa_amd_agent_iterate_memory_pools(
      agent,
      [](hsa_amd_memory_pool_t pool, void* p) {
        auto* Q_ = static_cast<Q*>(p);
        if (Q_->found) return HSA_STATUS_SUCCESS;
        hsa_amd_segment_t seg;
        uint32_t flags = 0;
        bool alloc = false;
        if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
            seg != HSA_AMD_SEGMENT_GLOBAL)
          return HSA_STATUS_SUCCESS;
        hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
        hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
        if (alloc && (flags & Q_->want) == Q_->want) {
          Q_->pool = pool;
          Q_->found = true;
        }
        return HSA_STATUS_SUCCESS;
      },
      &q);
  if (!q.found) throw std::runtime_error("no HSA memory pool with flags " + std::to_string(want));
  return q.pool;
}

// AQL dispatch header: kernel dispatch, barrier bit so slots retire in order, system-scope acquire
// (invalidates the L2 lines of the coarse-grained host kernargs written since the last launch of
// the slot) and system-scope release (the records and the arrival flag land in host memory). An
// agent-scope acquire measured the same on fine-grained kernargs but would not cover coarse ones.
constexpr uint16_t kHeader = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                             (1 << HSA_PACKET_HEADER_BARRIER) |
                             (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                             (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);

struct Kernel {
  uint64_t object = 0;
  uint32_t kernarg_size = 0, group = 0, priv = 0;
};

}  // namespace

int gpu_count() { return agents().up ? static_cast<int>(agents().gpus.size()) : 0; }

std::string gpu_pci(int index) {
  const Agents& a = agents();
  if (!a.up || index < 0 || index >= static_cast<int>(a.gpus.size())) return "";
  uint32_t bdf = 0, domain = 0;
  if (hsa_agent_get_info(a.gpus[index], static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf) !=
      HSA_STATUS_SUCCESS)
    return "";
  if (hsa_agent_get_info(a.gpus[index], static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &domain) !=
      HSA_STATUS_SUCCESS)
    domain = 0;
  char buf[32];  // BDFID: bus[15:8] device[7:3] function[2:0]
  snprintf(buf, sizeof buf, "%04x:%02x:%02x.%x", domain & 0xffff, (bdf >> 8) & 0xff, (bdf >> 3) & 0x1f, bdf & 0x7);
  return buf;
}

std::string gpu_arch(int index) {
  const Agents& a = agents();
  if (!a.up || index < 0 || index >= static_cast<int>(a.gpus.size())) return "";
  std::string name;
  hsa_agent_iterate_isas(
      a.gpus[index],
      [](hsa_isa_t isa, void* p) {
        uint32_t len = 0;
        if (hsa_isa_get_info_alt(isa, HSA_ISA_INFO_NAME_LENGTH, &len) != HSA_STATUS_SUCCESS || !len)
          return HSA_STATUS_SUCCESS;
        std::string s(len, '\0');
        hsa_isa_get_info_alt(isa, HSA_ISA_INFO_NAME, &s[0]);
        s.resize(strnlen(s.c_str(), s.size()));
        auto* out = static_cast<std::string*>(p);
        if (out->empty()) *out = s;
        return HSA_STATUS_SUCCESS;
      },
      &name);
  const std::string prefix = "amdgcn-amd-amdhsa--";
  return name.compare(0, prefix.size(), prefix) == 0 ? name.substr(prefix.size()) : name;
}

struct HsaProbe::Impl {
  hsa_agent_t gpu{};
  hsa_queue_t* queue = nullptr;
  hsa_executable_t exe{};
  hsa_code_object_reader_t reader{};
  bool have_exe = false, have_reader = false;
  Kernel probe, reset;
  gpumon_hip::ProbeRecord* ring = nullptr;  // fine-grained system memory, GPU-accessible
  uint32_t* arrivals = nullptr;              // ditto, one flag per slot
  uint32_t* counters = nullptr;              // GPU VRAM, one self re-arming counter per slot
  char* kernargs = nullptr;                  // kernarg pool, kKernargStride per slot (+ 1 for reset)
  std::vector<hsa_signal_t> done;            // per slot (+ 1 for reset): 1 while the dispatch runs
  std::vector<uint32_t> slot_seq;
  std::vector<int64_t> slot_launch_ns;
  uint32_t seq = 0;
  int next = 0;
  static constexpr size_t kKernargStride = 256;

  void dispatch(const Kernel& k, int sig_index, uint32_t grid_wgs) {
    // Single producer (one sampler thread owns a probe): claim the packet slot only once it is
    // free, so a full queue never leaves a reserved slot without a valid header behind (the
    // command processor would wait on it forever). Never more than slots + 1 packets are in flight
    // and the queue holds >= 64, so this wait is a guard.
    const uint64_t idx = hsa_queue_load_write_index_relaxed(queue);
    const int64_t deadline = mono_ns() + 1'000'000'000;
    while (idx - hsa_queue_load_read_index_scacquire(queue) >= queue->size) {
      if (mono_ns() > deadline) throw std::runtime_error("HSA probe queue full");
      std::this_thread::yield();
    }
    hsa_queue_store_write_index_relaxed(queue, idx + 1);
    auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(queue->base_address) + (idx & (queue->size - 1));
    pkt->workgroup_size_x = 64;
    pkt->workgroup_size_y = 1;
    pkt->workgroup_size_z = 1;
    pkt->reserved0 = 0;
    pkt->grid_size_x = grid_wgs * 64u;
    pkt->grid_size_y = 1;
    pkt->grid_size_z = 1;
    pkt->private_segment_size = k.priv;
    pkt->group_segment_size = k.group;
    pkt->kernel_object = k.object;
    pkt->kernarg_address = kernargs + static_cast<size_t>(sig_index) * kKernargStride;
    pkt->reserved2 = 0;
    pkt->completion_signal = done[sig_index];
    const uint32_t setup = 1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;  // 1-D grid
    __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), kHeader | (setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(queue->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
  }

  bool wait_signal(int i, double timeout_s) {
    const int64_t deadline = mono_ns() + static_cast<int64_t>(timeout_s * 1e9);
    while (hsa_signal_load_scacquire(done[i]) > 0) {
      if (mono_ns() > deadline) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    return true;
  }
};

HsaProbe::HsaProbe(int gpu, int blocks, int slots, int spin_ticks)
    : d_(new Impl), blocks_(std::max(1, blocks)), slots_(std::max(1, slots)), spin_(std::max(1, spin_ticks)) {
  try {
    const Agents& a = agents();
    if (!a.up) throw std::runtime_error("hsa_init failed");
    if (gpu < 0 || gpu >= static_cast<int>(a.gpus.size()))
      throw std::runtime_error("no HSA GPU agent " + std::to_string(gpu));
    d_->gpu = a.gpus[gpu];
    // code object -> executable -> the two kernel descriptors
    const size_t co_size = static_cast<size_t>(gpumon_probe_hsaco_end - gpumon_probe_hsaco_begin);
    ck(hsa_code_object_reader_create_from_memory(gpumon_probe_hsaco_begin, co_size, &d_->reader),
       "hsa_code_object_reader_create_from_memory");
    d_->have_reader = true;
    ck(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &d_->exe),
       "hsa_executable_create_alt");
    d_->have_exe = true;
    ck(hsa_executable_load_agent_code_object(d_->exe, d_->gpu, d_->reader, nullptr, nullptr),
       "hsa_executable_load_agent_code_object (is the GPU gfx950?)");
    ck(hsa_executable_freeze(d_->exe, nullptr), "hsa_executable_freeze");
    auto sym = [&](const char* name, Kernel* k, uint32_t want_kernarg) {
      hsa_executable_symbol_t s;
      ck(hsa_executable_get_symbol_by_name(d_->exe, name, &d_->gpu, &s), name);
      ck(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->object), name);
      ck(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kernarg_size),
         name);
      ck(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->group), name);
      ck(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->priv), name);
      // the argument block written below must be the one the code object declares
      if (k->kernarg_size != want_kernarg || k->kernarg_size > Impl::kKernargStride)
        throw std::runtime_error(std::string(name) + ": kernarg segment " + std::to_string(k->kernarg_size) +
                                 " B, expected " + std::to_string(want_kernarg));
    };
    sym("gpumon_probe_kernel.kd", &d_->probe, 36);
    sym("gpumon_probe_reset.kd", &d_->reset, 12);
    // memory
    const hsa_amd_memory_pool_t host_fine = find_pool(a.cpu, HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED);
    // Kernargs: every probe wave reads its 36-byte block. From the kernarg pool (fine-grained,
    // not cached in L2) those reads cross to host memory from every CU: a 32 us kernel with a
    // 28 us wave spread on MI355X. From coarse-grained system memory the first read per XCD fills
    // its L2 (the dispatch's system-scope acquire invalidates it before each launch): 16 us and
    // 6.6 us, as on the HIP path (profiles/r3_probe_hsa.md). GPUMON_PROBE_KERNARG=kernarg selects
    // the kernarg pool; without a coarse-grained system pool it is used anyway.
    hsa_amd_memory_pool_t kernarg{};
    {
      const char* k = getenv("GPUMON_PROBE_KERNARG");
      bool coarse = !(k && !strcmp(k, "kernarg"));
      if (coarse) {
        try {
          kernarg = find_pool(a.cpu, HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED);
        } catch (const std::exception&) {
          coarse = false;
        }
      }
      if (!coarse) kernarg = find_pool(a.cpu, HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT);
    }
    const hsa_amd_memory_pool_t vram = find_pool(d_->gpu, HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED);
    const size_t ring_bytes = sizeof(gpumon_hip::ProbeRecord) * static_cast<size_t>(blocks_) * slots_;
    auto host_alloc = [&](hsa_amd_memory_pool_t pool, size_t bytes, void** p, const char* what) {
      ck(hsa_amd_memory_pool_allocate(pool, bytes, 0, p), what);
      ck(hsa_amd_agents_allow_access(1, &d_->gpu, nullptr, *p), what);
      memset(*p, 0, bytes);
    };
    host_alloc(host_fine, ring_bytes, reinterpret_cast<void**>(&d_->ring), "ring");
    host_alloc(host_fine, sizeof(uint32_t) * slots_, reinterpret_cast<void**>(&d_->arrivals), "arrivals");
    host_alloc(kernarg, Impl::kKernargStride * (slots_ + 1), reinterpret_cast<void**>(&d_->kernargs), "kernargs");
    ck(hsa_amd_memory_pool_allocate(vram, sizeof(uint32_t) * slots_, 0, reinterpret_cast<void**>(&d_->counters)),
       "counters");
    for (int i = 0; i <= slots_; ++i) {
      hsa_signal_t s;
      ck(hsa_signal_create(0, 0, nullptr, &s), "hsa_signal_create");
      d_->done.push_back(s);
    }
    // one hardware queue; its size is the agent's minimum (>= 64 packets)
    uint32_t qmin = 64;
    hsa_agent_get_info(d_->gpu, HSA_AGENT_INFO_QUEUE_MIN_SIZE, &qmin);
    ck(hsa_queue_create(d_->gpu, std::max<uint32_t>(qmin, 64), HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX,
                        UINT32_MAX, &d_->queue),
       "hsa_queue_create");
    // zero the counters on the same queue, wait for it (bounded)
    char* ka = d_->kernargs + static_cast<size_t>(slots_) * Impl::kKernargStride;
    void* cptr = d_->counters;
    const uint32_t n = static_cast<uint32_t>(slots_);
    memcpy(ka + 0, &cptr, 8);
    memcpy(ka + 8, &n, 4);
    hsa_signal_store_screlease(d_->done[slots_], 1);
    d_->dispatch(d_->reset, slots_, 1);
    if (!d_->wait_signal(slots_, 10.0)) throw std::runtime_error("probe counter reset did not complete in 10 s");
    d_->slot_seq.assign(slots_, 0);
    d_->slot_launch_ns.assign(slots_, 0);
  } catch (...) {
    release(d_);
    d_ = nullptr;
    throw;
  }
}

void HsaProbe::release(Impl* d) {
  if (!d) return;
  // nothing may be freed under a running dispatch: wait (bounded), else leak rather than fault
  bool idle = true;
  for (size_t i = 0; i < d->done.size(); ++i) idle = d->wait_signal(static_cast<int>(i), 5.0) && idle;
  if (idle) {
    if (d->queue) hsa_queue_destroy(d->queue);
    for (hsa_signal_t s : d->done) hsa_signal_destroy(s);
    if (d->ring) hsa_amd_memory_pool_free(d->ring);
    if (d->arrivals) hsa_amd_memory_pool_free(d->arrivals);
    if (d->kernargs) hsa_amd_memory_pool_free(d->kernargs);
    if (d->counters) hsa_amd_memory_pool_free(d->counters);
    if (d->have_exe) hsa_executable_destroy(d->exe);
    if (d->have_reader) hsa_code_object_reader_destroy(d->reader);
  }
  delete d;
}

HsaProbe::~HsaProbe() { release(d_); }

int HsaProbe::launch() {
  const int slot = d_->next;
  // A slot is reusable only when its previous launch fully arrived and its dispatch retired
  // (the kernarg block and the completion signal are the slot's own).
  if (d_->slot_seq[slot] != 0 &&
      (__atomic_load_n(&d_->arrivals[slot], __ATOMIC_ACQUIRE) < static_cast<uint32_t>(blocks_) ||
       hsa_signal_load_scacquire(d_->done[slot]) > 0))
    return -1;
  d_->next = (d_->next + 1) % slots_;
  const uint32_t seq = ++d_->seq;
  __atomic_store_n(&d_->arrivals[slot], 0u, __ATOMIC_RELEASE);
  d_->slot_seq[slot] = seq;
  char* ka = d_->kernargs + static_cast<size_t>(slot) * Impl::kKernargStride;
  void* recs = d_->ring + static_cast<size_t>(slot) * blocks_;
  void* arr = d_->arrivals + slot;
  void* cnt = d_->counters + slot;
  const uint32_t spin = static_cast<uint32_t>(spin_), nb = static_cast<uint32_t>(blocks_);
  memcpy(ka + 0, &recs, 8);
  memcpy(ka + 8, &arr, 8);
  memcpy(ka + 16, &cnt, 8);
  memcpy(ka + 24, &seq, 4);
  memcpy(ka + 28, &spin, 4);
  memcpy(ka + 32, &nb, 4);
  hsa_signal_store_screlease(d_->done[slot], 1);
  d_->slot_launch_ns[slot] = mono_ns();
  d_->dispatch(d_->probe, slot, nb);
  return slot;
}

bool HsaProbe::poll(int slot, gpumon_hip::ProbeResult* out) {
  if (slot < 0 || slot >= slots_) return false;
  const uint32_t arrived = __atomic_load_n(&d_->arrivals[slot], __ATOMIC_ACQUIRE);
  out->seq = d_->slot_seq[slot];
  out->blocks = blocks_;
  out->arrived = static_cast<int>(arrived);
  out->host_launch_ns = d_->slot_launch_ns[slot];
  if (arrived < static_cast<uint32_t>(blocks_)) {
    out->complete = false;
    return false;
  }
  out->complete = true;
  out->host_done_ns = mono_ns();
  gpumon_hip::probe_collect(d_->ring + static_cast<size_t>(slot) * blocks_, blocks_, out);
  return true;
}

bool HsaProbe::wait(int slot, double timeout_s, gpumon_hip::ProbeResult* out) {
  const int64_t deadline = mono_ns() + static_cast<int64_t>(timeout_s * 1e9);
  while (!poll(slot, out)) {
    if (mono_ns() > deadline) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  return true;
}

}  // namespace gpumon_hsa

// K1 probe over the raw HSA runtime: the probe's code object (csrc/hip/probe_co.hip, embedded in
// this library) loaded into an hsa_executable and dispatched as AQL kernel-dispatch packets on ONE
// hardware queue of its own.
//
// Why: every hardware queue pins a ~173 MB host context-save area on MI355X (256 CUs of wave state,
// profiles/r2_footprint.md), and the HIP runtime brings up two queues for a device even when the
// probe runs on its null stream (profiles/r3_helper_memory.md). A process that only needs the
// probe therefore pays one queue here instead of two. The records, their publication and their
// analysis are the HIP path's (csrc/hip/probe_kernel.h, csrc/hip/probe_collect.h).
//
// Memory: ring + arrival flags in fine-grained system memory (the CPU agent's fine-grained pool,
// made accessible to the GPU), the self re-arming per-slot counters in the GPU's coarse-grained
// VRAM pool (zeroed once by gpumon_probe_reset on the same queue: a copy engine or blit kernel
// would bring up another queue), one kernarg block per slot in coarse-grained system memory (cached
// in L2 after the first read per XCD) and one completion signal per slot.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../hip/probe_collect.h"

namespace gpumon_hsa {

// HSA runtime view of the GPUs, in HSA enumeration order (= HIP device order when no
// HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES / GPU_DEVICE_ORDINAL reorders HIP's view).
int gpu_count();                   // brings HSA up on first use (hsa_init); 0 when it cannot
std::string gpu_arch(int index);   // "gfx950:sramecc+:xnack-", "" for a bad index
std::string gpu_pci(int index);    // "0000:75:00.0" (HSA_AMD_AGENT_INFO_DOMAIN / _BDFID), "" if unknown

class HsaProbe {
 public:
  HsaProbe(int gpu, int blocks, int slots, int spin_ticks);  // throws std::runtime_error
  ~HsaProbe();
  HsaProbe(const HsaProbe&) = delete;
  HsaProbe& operator=(const HsaProbe&) = delete;
  int launch();  // slot, or -1 when the slot to use is still in flight
  bool poll(int slot, gpumon_hip::ProbeResult* out);
  bool wait(int slot, double timeout_s, gpumon_hip::ProbeResult* out);
  int blocks() const { return blocks_; }

 private:
  struct Impl;
  static void release(Impl* d);
  Impl* d_;
  int blocks_, slots_, spin_;
};

}  // namespace gpumon_hsa

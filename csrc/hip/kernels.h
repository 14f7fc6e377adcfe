// gfx950 (MI355X / CDNA4) kernels for gpumon:
//
//   K1 probe  — on-device sampling microkernel. One 64-lane wave per workgroup stamps
//               s_memrealtime (100 MHz constant clock), s_memtime (shader clock), HW_REG_XCC_ID
//               and HW_REG_HW_ID, spins a fixed realtime window to measure the effective shader
//               clock, and publishes a record into a PINNED host ring buffer with system-scope
//               stores + a per-slot arrival counter. The host polls the counter; it never calls
//               hipDeviceSynchronize (no host-side stall, no interference with the workload's
//               streams). SQ/GRBM perf counters are not readable from shader code on CDNA4 (they
//               are privileged MMIO programmed by the driver); MFMA-busy / occupancy come from
//               rocprofiler-sdk device counting (tests/oracles/ops/pmc.py), the probe supplies the
//               per-XCD liveness, clock and dispatch-latency signals.
//   K2 load   — synthetic loads that validate the exporter under known conditions:
//               bf16 MFMA burn (v_mfma_f32_32x32x16_bf16, 4 independent accumulators per wave,
//               operands in VGPRs) and an HBM stream (16-B per lane non-temporal loads/stores,
//               grid-stride, >>256 workgroups to fill all 8 XCDs).
//
// The reference (/root/reference) has no GPU code at all; these kernels are [new] per SURVEY.md
// §2.3 (K1, K2).
#pragma once

#include <cstdint>

namespace gpumon_hip {

struct ProbeRecord {
  uint32_t xcc_id;     // HW_REG_XCC_ID[3:0]
  uint32_t hw_id;      // HW_REG_HW_ID raw (wave, simd, cu, sh, se ...)
  uint64_t t0_real;    // s_memrealtime at block start (100 MHz)
  uint64_t t1_real;    // s_memrealtime at block end
  uint64_t c0;         // s_memtime at block start (shader clock)
  uint64_t c1;         // s_memtime at block end
  uint32_t seq;        // launch sequence number (matches the slot's expected seq when valid)
  uint32_t block;
};
static_assert(sizeof(ProbeRecord) == 48, "ProbeRecord layout");

}  // namespace gpumon_hip

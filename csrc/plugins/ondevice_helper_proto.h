// Wire protocol between the exporter and lib/gpumon-ondevice-helper, the process that runs every
// GPU-runtime-facing piece of the on-device samplers: the rocprofiler-sdk device counting contexts
// (libgpumon_pmc.so) and the K1 probe (libgpumon_probe.so, HIP). Both ends are built from this tree
// for the same machine: fixed-size structs over a pipe pair, no versioning beyond the magic.
//
// Why a separate process:
//  * rocprofiler-sdk's device counting service leaves an HSA async-events thread polling (ioctl +
//    calloc in a loop, one full CPU core, measured on MI355X with tools/thread_cpu.py +
//    tools/ip_sample). The exporter freezes the helper (SIGSTOP) between requests; the hardware
//    keeps counting while it is stopped (tools/pmc_stop_probe.py: identical MFMA busy over stopped
//    and running intervals), so the poller costs nothing between samples.
//  * the exporter process itself never loads HIP, HSA or rocprofiler (9 MB RSS); the runtimes share
//    one HSA instance in the helper, and a wedged GPU runtime is a helper to kill, not an exporter.
#pragma once

#include <stdint.h>

#include "ondevice_abi.h"

#define GPUMON_PMC_PROTO_MAGIC 0x474d5043u  // "GMPC"

enum gpumon_pmc_op : uint32_t {
  GPUMON_PMC_OP_INIT = 1,          // -> rc = agent count (or -1, err)
  GPUMON_PMC_OP_AGENT = 2,         // agents[0] = index -> payload gpumon_pmc_agent_t
  GPUMON_PMC_OP_SAMPLE_MANY = 3,   // agents, counters, window_s -> values + ok
  GPUMON_PMC_OP_READ_RUNNING = 4,  // agents, counters -> values + ok + started
  GPUMON_PMC_OP_STOP_RUNNING = 5,
  GPUMON_PMC_OP_QUIT = 6,
  // K1 probe (libgpumon_probe.so, dlopen'd by the helper on first use)
  GPUMON_PROBE_OP_COUNT = 10,      // -> rc = HIP device count (or -1, err)
  GPUMON_PROBE_OP_CREATE = 11,     // agents = {hip_dev, blocks, slots, spin_ticks} -> rc = handle id
  GPUMON_PROBE_OP_LAUNCH = 12,     // agents = {handle} -> rc = slot (-1: every slot in flight)
  GPUMON_PROBE_OP_WAIT = 13,       // agents = {handle, slot}, window_s = timeout -> rc 1 + gpumon_probe_result_t | 0
  GPUMON_PROBE_OP_DESTROY = 14,    // agents = {handle}
  // one sampler step in one request: agents = {handle, pending slot (-1: launch now)} per probe,
  // window_s = timeout -> rc = n, payload gpumon_probe_cycle_t[n]. Launch and completion are seen
  // within one awake period, so host_latency_s never includes the time the helper was stopped.
  GPUMON_PROBE_OP_CYCLE = 15,
  GPUMON_PROBE_OP_PCI = 16,        // agents = {hip_dev} -> rc = bytes, payload = "dddd:bb:dd.f" (rc 0: unknown)
};

typedef struct {
  int32_t pending;  // slot still in flight after the step (-1: completed or nothing launched)
  int32_t got;      // 1: `result` holds the completed launch
  gpumon_probe_result_t result;
} gpumon_probe_cycle_t;

// request: header, int32 agents[n_agents], char counters[counters_len] ('\n'-separated)
typedef struct {
  uint32_t magic;
  uint32_t op;
  uint32_t n_agents;
  uint32_t counters_len;
  double window_s;
} gpumon_pmc_req_t;

// response: header, char err[err_len], payload[payload_len]
//   AGENT: gpumon_pmc_agent_t
//   SAMPLE_MANY / READ_RUNNING: gpumon_pmc_value_t[n_agents * n_counters], int32 ok[n_agents]
//   PROBE_WAIT (rc 1): gpumon_probe_result_t
//   PROBE_CYCLE: gpumon_probe_cycle_t[n]
typedef struct {
  uint32_t magic;
  int32_t rc;
  int32_t started;
  uint32_t err_len;
  uint32_t payload_len;
} gpumon_pmc_resp_t;

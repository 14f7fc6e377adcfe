// Wire protocol between the exporter and bin/gpumon-pmc-helper (the process that owns the
// rocprofiler-sdk device counting contexts). Both ends are built from this tree for the same
// machine: fixed-size little-endian structs over a pipe pair, no versioning beyond the magic.
//
// Why a separate process: rocprofiler-sdk's device counting service leaves an HSA async-events
// thread polling (ioctl + calloc in a loop, one full CPU core, measured on MI355X with
// tools/thread_cpu.py + tools/ip_sample). The exporter freezes the helper (SIGSTOP) between reads;
// the hardware keeps counting while it is stopped (tools/pmc_stop_probe.py: identical MFMA busy
// over stopped and running intervals), so the poller costs nothing between samples.
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
};

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
typedef struct {
  uint32_t magic;
  int32_t rc;
  int32_t started;
  uint32_t err_len;
  uint32_t payload_len;
} gpumon_pmc_resp_t;

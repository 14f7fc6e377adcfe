// Exporter internals shared by its translation units (exporter.cpp, dev_workers.cpp,
// pod_rows.cpp, exporter_http.cpp). Not part of the public API (exporter.h).
#pragma once

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "exporter.h"

namespace gpumon {

// ---------------------------------------------------------------------------------------------
// Per-device sampling workers with a watchdog.
//
// Each GPU gets its own thread; a tick hands every idle worker a request and waits until all
// answer or `device_timeout_s` passes. A device whose call has not returned by then (a hung
// driver/SMU call) is exported as gpu_up 0 with gpumon_device_timeouts_total incremented, and is not
// asked again until its call returns -- the other GPUs keep their 1 Hz cadence (the reference
// stalled the whole node on any slow nvidia-smi, gpu.py:104-116). Workers only touch their own
// heap state and the backend, so a worker stuck at shutdown can be detached safely (the backend is
// then deliberately leaked instead of destroyed under it).
// ---------------------------------------------------------------------------------------------
struct Exporter::DoneSignal {
  std::mutex mu;
  std::condition_variable cv;
};

struct Exporter::DevWorker {
  std::mutex mu;
  std::condition_variable cv;
  bool quit = false;
  bool pending = false;          // request posted, not yet picked up
  bool busy = false;             // request in flight (posted or running)
  uint64_t req = 0;              // tick id of the current request
  std::atomic<uint64_t> done{0}; // tick id whose results are stored below
  bool want_links = false, want_procs = false, want_ras = false;
  bool ras_async = false;        // read the RAS slice AFTER publishing this tick (applied next tick)
  int ras_slice = 0, ras_n = 1;
  int64_t started_ns = 0;
  int64_t picked_ns = 0, device_ns = 0;  // pickup time and device-call time of the stored tick
  DeviceSample sample;
  std::vector<ProcSample> procs;
  int64_t proc_ns = 0;
  std::thread th;
};

// SCHED_FIFO for the calling thread (rt_priority); counted in `rt` while the thread lives.
bool apply_rt(int prio, const std::string& who, std::atomic<int>* rt);

}  // namespace gpumon

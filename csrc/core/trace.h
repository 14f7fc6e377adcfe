// Optional ROCTx ranges around the sampler phases (tracing row).
//
// The reference traced nothing beyond print() per line (gpu.py:144,146,217,219). Here every tick
// can be bracketed with ROCTx ranges ("gpumon.tick" > "gpumon.sample" / "gpumon.attrib" /
// "gpumon.render" / "gpumon.gzip", plus "gpumon.sample_dev" per device task) so
// `rocprofv3 --marker-trace` places the exporter's host work on the same timeline as the GPU
// kernels it observes. librocprofiler-sdk-roctx is dlopen'ed only when enabled (config `roctx` /
// GPUMON_ROCTX=1): no link-time ROCm dependency, zero cost (one relaxed load) when off.
#pragma once

#include <dlfcn.h>

#include <atomic>
#include <cstdint>

namespace gpumon {

class Roctx {
 public:
  using PushFn = int (*)(const char*);
  using PopFn = int (*)();
  using MarkFn = void (*)(const char*);

  // Returns true if ROCTx is active after the call.
  static bool enable(bool on) {
    Roctx& r = get();
    if (!on) {
      r.on_.store(false, std::memory_order_relaxed);
      return false;
    }
    if (!r.push_) {
      const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                            "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so.4"};
      for (const char* l : libs) {
        void* h = dlopen(l, RTLD_NOW | RTLD_LOCAL);
        if (!h) continue;
        auto push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
        auto pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
        if (push && pop) {
          r.mark_ = reinterpret_cast<MarkFn>(dlsym(h, "roctxMarkA"));
          r.pop_ = pop;
          r.push_ = push;
          break;
        }
        dlclose(h);
      }
    }
    r.on_.store(r.push_ != nullptr, std::memory_order_relaxed);
    return r.push_ != nullptr;
  }
  static bool active() { return get().on_.load(std::memory_order_relaxed); }
  static void push(const char* name) {
    if (get().push_) get().push_(name);
  }
  static void pop() {
    if (get().pop_) get().pop_();
  }
  static void mark(const char* name) {
    if (active() && get().mark_) get().mark_(name);
  }
  // Ranges pushed/popped so far (tests check the bracketing without a profiler attached).
  static uint64_t ranges() { return get().n_.load(std::memory_order_relaxed); }
  static void count() { get().n_.fetch_add(1, std::memory_order_relaxed); }

 private:
  static Roctx& get() {
    static Roctx r;
    return r;
  }
  std::atomic<bool> on_{false};
  std::atomic<uint64_t> n_{0};
  PushFn push_ = nullptr;
  PopFn pop_ = nullptr;
  MarkFn mark_ = nullptr;
};

// RAII range; `active` is sampled once so a toggle mid-range cannot unbalance push/pop.
class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(Roctx::active()) {
    if (on_) {
      Roctx::push(name);
      Roctx::count();
    }
  }
  ~TraceRange() {
    if (on_) Roctx::pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

}  // namespace gpumon

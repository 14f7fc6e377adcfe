// Shared utilities for the gpumon C++ core: clocks, logging, small string helpers.
//
// The reference agent (/root/reference/gpu.py:21-22,144,146) logs with bare print() calls and
// has no time base other than time.sleep(10) (gpu.py:263). Here every component stamps with a
// monotonic ns clock for rates/latencies and a realtime ns clock for exported timestamps.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <string>
#include <string_view>
#include <vector>

namespace gpumon {

inline int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

inline int64_t wall_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

enum class LogLevel : int { kDebug = 0, kInfo = 1, kWarn = 2, kError = 3, kOff = 4 };

// Global log threshold; set from config (--log-level). Structured "key=value" lines to stderr.
extern std::atomic<int> g_log_level;

void log_line(LogLevel lvl, const char* component, const std::string& msg);

// Names the calling thread (<= 15 chars) so per-thread CPU is attributable in /proc/<pid>/task,
// top -H and perf (tools/thread_cpu.py).
void set_thread_name(const std::string& name);
// Blocks SIGPIPE on the calling thread. OpenSSL writes to its sockets with write(), which has no
// MSG_NOSIGNAL: on a connection the peer has reset, a second write would raise SIGPIPE and, in a host
// process that has not ignored it (an embedding service; CPython and the native binary do ignore
// it), end the process. Blocked, the write fails with EPIPE and the signal stays pending on this
// thread, where it is never delivered.
void block_sigpipe();

#define GPUMON_LOG(lvl, comp, msg)                                              \
  do {                                                                          \
    if (static_cast<int>(lvl) >= ::gpumon::g_log_level.load(std::memory_order_relaxed)) \
      ::gpumon::log_line(lvl, comp, msg);                                       \
  } while (0)

// Splits on a single character; empty fields kept.
std::vector<std::string> split(std::string_view s, char sep);
std::string_view trim(std::string_view s);
bool starts_with(std::string_view s, std::string_view p);
bool ends_with(std::string_view s, std::string_view p);

// Canonical PCI address "dddd:bb:dd.f", lower case; a missing domain is 0000 ("75:00.0" ->
// "0000:75:00.0"). "" if `s` is not a BDF. hipDeviceGetPCIBusId, libamd_smi and sysfs agree on it.
std::string normalize_bdf(std::string_view s);

// Reads a whole (small) file; returns false if it cannot be opened.
bool read_file(const std::string& path, std::string* out, size_t max_bytes = 1 << 20);

// The gpu_info driver_version label. `module_version` (<sysfs>/module/amdgpu/version, present for
// an out-of-tree / DKMS amdgpu) wins; otherwise libamd_smi's string, which for an in-kernel amdgpu
// is the kernel's /proc/version (seen on MI355X with its spaces removed: "Linuxversion6.18.51-ant.1
// (nixbld@localhost)(gcc(GCC)15.3.0,GNUld..."): then the release token ("6.18.51-ant.1", uname -r
// when the library gave nothing). Long library strings are cut at a separator, never inside a
// token (the reference's Q6 -- spaces stripped out of values, /root/reference/gpu.py:87 -- is
// what produced the garbage). *source: "module" | "kernel" | "library".
std::string driver_version_label(const std::string& raw, const std::string& module_version, std::string* source);

}  // namespace gpumon

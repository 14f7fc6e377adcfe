// Exposition renderers: Prometheus text format 0.0.4 and InfluxDB line protocol.
//
// Reference parity: the reference hand-builds two InfluxDB measurements with string
// concatenation and no escaping (/root/reference/gpu.py:136-143 node_gpu, gpu.py:206-216 and
// 240-250 pod_gpu; quirks Q7/Q8). Here both sinks are rendered from the same sample set once per
// tick into a buffer that scrapes / pushes only copy:
//   - Prometheus: node_gpu_* / pod_gpu_* keep the reference field names (dashboard compat) and
//     gpu_* families carry the MI355X extras.
//   - Influx:     byte-compatible node_gpu / pod_gpu measurements (tags/fields as the reference,
//     properly escaped, with timestamps) plus an optional gpu_ext measurement.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "sample.h"

namespace gpumon {

// One pod_gpu series: an attributed GPU process, or an allocated-but-idle GPU (pid "-").
struct PodRow {
  int dev = 0;                      // device index
  bool idle = false;
  std::string pid = "-";
  std::string procname = "-";
  std::string pod_namespace = "-";
  std::string pod_name = "-";
  std::string container = "-";
  std::string containerid = "-";    // 12-char short id (reference docker short id)
  std::string user_name = "-";
  double used_memory_bytes = 0;
  double gpu_util = 0;              // device-wide util (reference semantics, Q4)
  double proc_gfx_util = kNaN;      // true per-process util from engine_usage.gfx ns
  double cu_occupancy = kNaN;
  int occ_samples = 0;  // cu_occupancy reads behind the interval mean
  int queues = -1;      // hardware queues on the GPU (KFD queue list; -1 unknown)
  // the device's wall-time MFMA utilisation (PMC) when this process was the only one on the GPU
  // with waves resident this interval (exclusive use); NaN when the GPU was shared or PMC is off
  double mfma_util = kNaN;
  std::vector<std::pair<std::string, std::string>> extra_labels;  // allowlisted pod labels (label_<key>)
};

// A GPU context of a tick's process lists that is not a pod_gpu row, and why (/debug/procs).
struct HiddenCtx {
  int dev;
  uint32_t pid;
  const char* why;  // "empty", "peer", "helper", "not opted in"
};

// Histogram with fixed upper bounds (seconds).
struct HistSnapshot {
  std::vector<double> bounds;
  std::vector<uint64_t> counts;     // cumulative-ready: per-bucket (non-cumulative) counts
  uint64_t count = 0;
  double sum = 0;
};

struct SelfStats {
  std::string version;
  std::string backend;
  std::string backend_version;
  bool backend_up = false;
  int fast_path_devices = -1;        // amdsmi sysfs fast path (-1: not applicable)
  std::string fast_path_status;
  uint64_t backend_reinits = 0;
  uint64_t ticks = 0;
  uint64_t samples = 0;
  uint64_t stale_samples = 0;
  uint64_t frozen_samples = 0;       // ... of those, repeats older than stale_hold_s (rates withheld)
  uint64_t occupancy_reads = 0;     // KFD cu_occupancy sub-sample reads by the device workers
  uint64_t process_list_failures = 0;  // failed process lists (the last good one held kProcHoldTicks)
  uint64_t occupancy_scan_failures = 0;  // ... process listings that failed (retried with a backoff)
  uint64_t hidden_contexts = 0;     // GPU contexts without VRAM or waves left out of pod_gpu rows
  uint64_t hidden_peer_contexts = 0;  // peer contexts of multi-GPU processes left out of pod_gpu rows
  int rt_threads = 0;               // sampler / device-worker threads running SCHED_FIFO (rt_priority)
  int http_rt_loops = -1;            // HTTP loops at SCHED_FIFO now (-1: http_rt_priority off)
  int64_t http_evicted = -1;         // connections closed to make room at the cap (-1: no server)
  int64_t http_max_conns = -1;       // connection cap over all HTTP loops (from RLIMIT_NOFILE)
  int64_t http_tls_failures = -1;    // /metrics over HTTPS: failed / timed-out handshakes (-1: plain HTTP)
  int64_t http_tls_client_cert_refused = -1;  // mutual TLS: /metrics without a client certificate (-1: not mTLS)
  int64_t http_tls_not_after = 0;     // ... the serving certificate's expiry (unix s; 0 unknown)
  uint64_t http_tls_reloads_ok = 0, http_tls_reloads_failed = 0;  // ... certificate rotations picked up / refused
  int64_t http_auth_failures = -1;    // http_auth_token_file: /metrics requests refused (-1: no token)
  uint64_t http_auth_failures_by[3] = {0, 0, 0};  // ... by reason: no header, not Bearer, wrong token
  uint64_t http_auth_reloads_ok = 0, http_auth_reloads_failed = 0;  // ... token rotations picked up / refused
  int64_t http_rt_demotions = -1;    // ... times a loop spent its CPU budget and was demoted
  uint64_t overruns = 0;
  double last_tick_wall_s = 0;
  double interval_s = 1.0;
  HistSnapshot sample_hist;         // whole-tick duration
  HistSnapshot scrape_hist;         // server-side /metrics latency
  uint64_t scrapes = 0;
  uint64_t http_connections = 0;
  uint64_t pods_attributed = 0;
  uint64_t attribution_cache_hits = 0, attribution_cache_misses = 0;
  uint64_t influx_ok = 0, influx_fail = 0, influx_dropped = 0;
  uint64_t gzip_eager = 0, gzip_lazy = 0, gzip_unused = 0, gzip_predicted = 0;  // snapshot compressions
  uint64_t kfd_files_open = 0, kfd_reads_cached = 0;        // sysfs fast path: kept KFD per-pid files
  bool influx_enabled = false;  // a push URL is configured
  int influx_up = 0;            // the last push attempt succeeded
  int64_t influx_last_ok_wall_ns = 0;
  struct Call {
    std::string call;
    uint64_t n = 0, errors = 0;
    double seconds = 0;
  };
  std::vector<Call> backend_calls;  // per backend call kind (amdsmi_get_gpu_metrics_info, ...)
  // process collector (the reference forked ~4+2C+P subprocesses per cycle; this is the whole cost)
  double cpu_seconds = -1, rss_bytes = -1, start_time_s = -1;
  int threads = -1, open_fds = -1;
  std::vector<uint64_t> device_errors;  // per device
  std::vector<uint64_t> device_timeouts;  // per device: hung calls caught by the watchdog
};

// Values supplied from outside the sampler (probe kernel, PMC device counting, plugins).
struct ExtraSeries {
  std::string name;                 // full metric name
  std::string help;
  std::string type = "gauge";
  int dev = -1;                     // -1 = node-level (no device labels)
  std::vector<std::pair<std::string, std::string>> labels;
  double value = 0;
};

struct RenderInput {
  std::string host;
  const std::vector<DeviceStatic>* statics = nullptr;
  const std::vector<DeviceSample>* samples = nullptr;
  const std::vector<DeviceRates>* rates = nullptr;
  const std::vector<PodRow>* pod_rows = nullptr;
  const std::vector<size_t>* proc_counts = nullptr;  // per device
  const std::vector<ExtraSeries>* extras = nullptr;
  const SelfStats* self = nullptr;
  bool compat_families = true;      // node_gpu_* / pod_gpu_*
  bool extended_families = true;    // gpu_* MI355X extras
  // false: device series carry only host + gpu_id (the reference's tags, gpu.py:137); uuid / bdf /
  // model live once on gpu_info (join on gpu_id). true: uuid + bdf on every device series.
  bool full_device_labels = false;
  // family filter (ExporterConfig::metrics_include / metrics_exclude); null or empty = no filter
  const std::vector<std::string>* metrics_include = nullptr;
  const std::vector<std::string>* metrics_exclude = nullptr;
};

// Whether render_prometheus emits family `name` under the input's include / exclude globs.
bool family_selected(const RenderInput& in, const char* name);
// Shell glob: '*', '?', '[abc]' / '[a-z]' / '[!x]' classes, '\\' escapes. Time O(|glob| x |name|)
// (one backtrack point: the last '*'), never exponential -- request globs reach it from the
// network, and glibc fnmatch recurses per '*' (ADVICE r3).
bool glob_match(const char* glob, const char* name);
// The same rule on plain lists: with a non-empty include list only matching names pass, then
// exclude drops matching ones (glob_match).
bool family_matches(const std::vector<std::string>& include, const std::vector<std::string>& exclude,
                    const char* name);
// Filters a rendered exposition by family: every line from a family's "# HELP" up to the next one
// (its TYPE line and samples, histogram _bucket/_sum/_count included) is kept or dropped as a unit.
// Sample lines before any HELP are kept. Used for per-request filters (/metrics?include=&exclude=).
void filter_exposition(const std::string& body, const std::vector<std::string>& include,
                       const std::vector<std::string>& exclude, std::string* out);

void render_prometheus(const RenderInput& in, std::string* out);
// Line protocol; one line per node_gpu / pod_gpu row (+ gpu_ext when extended), ns timestamps.
// schema: 2019 = the reference's current node_gpu/pod_gpu layout (gpu.py:136-143,206-216,240-250);
// 2018 = the older pod_gpu layout of img/influxdb.png (node_gpu unchanged).
void render_influx(const RenderInput& in, int64_t ts_ns, bool extended, std::string* out, int schema = 2019);

// Escapers (exposed for tests).
void escape_label_value(std::string_view v, std::string* out);
void escape_influx_tag(const std::string& v, std::string* out);
void escape_influx_field_str(const std::string& v, std::string* out);
void append_double(double v, std::string* out);

}  // namespace gpumon

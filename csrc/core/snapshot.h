// Pre-rendered exposition snapshot shared between the sampler (writer) and HTTP workers (readers).
//
// The reference has no scrape endpoint (push-only, /root/reference/gpu.py:145). The design goal
// for /metrics p99 is that a scrape never touches the device or re-renders: the sampler renders
// (and gzips) once per tick, then publishes an immutable Snapshot; a scrape takes a reference
// under a tiny critical section and writes the bytes.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace gpumon {

struct Snapshot {
  std::string body;       // text/plain; version=0.0.4
  uint64_t seq = 0;
  int64_t wall_ns = 0;
  bool gzip = false;      // compression enabled for this exporter

  // The gzip of `body`, made at most once per snapshot: by the tick thread right after publication
  // when recent snapshots were scraped with gzip (Prometheus scraping every tick), otherwise by the
  // first gzip scrape of this snapshot (a 15 s scrape of a 1 Hz exporter compresses 1 tick in 15,
  // not all of them: gzip was 2/3 of the tick thread's CPU at 8 GPUs, profiles/r5_cpu_8dev.md).
  // nullptr = serve the identity body (compression disabled, failed, or another thread is
  // compressing right now -- HTTP lets a server ignore Accept-Encoding).
  const std::string* gzipped(bool compress_now) const;
  static constexpr int64_t kGzipWaitNs = 1'000'000;  // longest wait for another thread's compression
  // The tick thread's eager compression (does not count as a gzip request). false = not made
  // here: a scrape is compressing or has compressed it (or compression is off or failed).
  bool precompress() const;
  // A scrape asked this snapshot for gzip (the tick thread's eager / lazy decision).
  bool gzip_asked() const { return gz_asked_.load(std::memory_order_relaxed); }
  // Whether this snapshot was compressed (by either path).
  bool compressed() const { return gz_state_.load(std::memory_order_acquire) == 2; }
  // A thread is compressing it right now (tests).
  bool compressing() const { return gz_state_.load(std::memory_order_acquire) == 1; }

 private:
  // 0 -> 1: this thread compresses. false = another thread got there first (*st = its state).
  bool claim(int* st) const;
  const std::string* compress_claimed() const;  // after a successful claim
  mutable std::atomic<int> gz_state_{0};  // 0 none, 1 compressing, 2 done, 3 failed
  mutable std::atomic<bool> gz_asked_{false};
  mutable std::string gz_;
};

class SnapshotStore {
 public:
  std::shared_ptr<const Snapshot> get() const {
    std::lock_guard<std::mutex> g(mu_);
    return cur_;
  }
  void publish(std::shared_ptr<const Snapshot> s) {
    std::lock_guard<std::mutex> g(mu_);
    cur_ = std::move(s);
  }

 private:
  mutable std::mutex mu_;
  std::shared_ptr<const Snapshot> cur_;
};

// Lock-free fixed-bucket histogram (observations in seconds).
class Histogram {
 public:
  explicit Histogram(std::vector<double> bounds);
  void observe(double seconds);
  void snapshot(std::vector<double>* bounds, std::vector<uint64_t>* counts, uint64_t* count,
                double* sum) const;
  // Quantile of the last kRecent observations, exact (the exported buckets are what Prometheus
  // aggregates; a bucket-interpolated p99 between 1 and 2.5 ms says little about a 1.1 ms tick).
  double quantile(double q) const;

  // Observations with index >= `from` (0-based, in arrival order) still held by the ring, and the
  // index one past the newest: an exact window quantile for a caller that noted observed() first.
  std::vector<float> since(uint64_t from, uint64_t* end) const;
  uint64_t observed() const { return recent_n_.load(std::memory_order_relaxed); }

  static constexpr size_t kRecent = 16384;

 private:
  std::vector<double> bounds_;
  std::unique_ptr<std::atomic<uint64_t>[]> counts_;  // bounds_.size() + 1 (overflow)
  std::atomic<uint64_t> count_{0};
  std::atomic<uint64_t> sum_ns_{0};
  std::unique_ptr<std::atomic<float>[]> recent_;  // ring of the last kRecent observations (seconds)
  std::atomic<uint64_t> recent_n_{0};
};

std::vector<double> latency_buckets();  // 50us .. 10s

// gzip (RFC 1952) of `in`; returns false if zlib fails.
bool gzip_compress(const std::string& in, std::string* out, int level = 1);

}  // namespace gpumon

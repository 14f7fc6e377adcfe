#include "snapshot.h"

#include "common.h"

#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cmath>

namespace gpumon {

Histogram::Histogram(std::vector<double> bounds)
    : bounds_(std::move(bounds)), counts_(new std::atomic<uint64_t>[bounds_.size() + 1]),
      recent_(new std::atomic<float>[kRecent]) {
  for (size_t i = 0; i <= bounds_.size(); ++i) counts_[i].store(0);
  for (size_t i = 0; i < kRecent; ++i) recent_[i].store(0.f);
}

void Histogram::observe(double s) {
  const uint64_t slot = recent_n_.fetch_add(1, std::memory_order_relaxed);
  recent_[slot % kRecent].store(static_cast<float>(s), std::memory_order_relaxed);
  size_t i = std::lower_bound(bounds_.begin(), bounds_.end(), s) - bounds_.begin();
  counts_[i].fetch_add(1, std::memory_order_relaxed);
  count_.fetch_add(1, std::memory_order_relaxed);
  sum_ns_.fetch_add(static_cast<uint64_t>(std::max(0.0, s) * 1e9), std::memory_order_relaxed);
}

void Histogram::snapshot(std::vector<double>* bounds, std::vector<uint64_t>* counts,
                         uint64_t* count, double* sum) const {
  *bounds = bounds_;
  counts->resize(bounds_.size());
  uint64_t total = 0;
  for (size_t i = 0; i < bounds_.size(); ++i) {
    (*counts)[i] = counts_[i].load(std::memory_order_relaxed);
    total += (*counts)[i];
  }
  total += counts_[bounds_.size()].load(std::memory_order_relaxed);
  *count = total;
  *sum = sum_ns_.load(std::memory_order_relaxed) * 1e-9;
}

double Histogram::quantile(double q) const {
  const uint64_t n = std::min<uint64_t>(recent_n_.load(std::memory_order_relaxed), kRecent);
  if (!n) return NAN;
  std::vector<float> v(n);
  for (uint64_t k = 0; k < n; ++k) v[k] = recent_[k].load(std::memory_order_relaxed);
  const size_t idx = std::min<size_t>(n - 1, static_cast<size_t>(std::ceil(q * n)) - (q > 0 ? 1 : 0));
  std::nth_element(v.begin(), v.begin() + idx, v.end());
  return v[idx];
}

std::vector<float> Histogram::since(uint64_t from, uint64_t* end) const {
  const uint64_t n = recent_n_.load(std::memory_order_acquire);
  if (end) *end = n;
  const uint64_t lo = std::max<uint64_t>(from, n > kRecent ? n - kRecent : 0);
  std::vector<float> v;
  v.reserve(n > lo ? n - lo : 0);
  for (uint64_t k = lo; k < n; ++k) v.push_back(recent_[k % kRecent].load(std::memory_order_relaxed));
  return v;
}

std::vector<double> latency_buckets() {
  return {50e-6, 100e-6, 250e-6, 500e-6, 1e-3, 2.5e-3, 5e-3, 10e-3, 25e-3,
          50e-3, 100e-3, 250e-3, 500e-3, 1.0,  2.5,    5.0,  10.0};
}

namespace {
// One deflate state per thread, reset between bodies: deflateInit2 allocates ~270 KB and clears
// the window and hash tables each time, about a third of a 20-30 KB exposition's compression.
struct Deflater {
  z_stream zs{};
  int level = -1;  // -1: not initialised
  ~Deflater() {
    if (level >= 0) deflateEnd(&zs);
  }
};
}  // namespace

bool gzip_compress(const std::string& in, std::string* out, int level) {
  thread_local Deflater d;
  if (d.level != level) {
    if (d.level >= 0) deflateEnd(&d.zs);
    d.zs = z_stream{};
    d.level = -1;
    if (deflateInit2(&d.zs, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    d.level = level;
  } else if (deflateReset(&d.zs) != Z_OK) {
    return false;
  }
  z_stream& zs = d.zs;
  out->resize(deflateBound(&zs, in.size()) + 32);
  zs.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data()));
  zs.avail_in = static_cast<uInt>(in.size());
  zs.next_out = reinterpret_cast<Bytef*>(&(*out)[0]);
  zs.avail_out = static_cast<uInt>(out->size());
  const int r = deflate(&zs, Z_FINISH);
  if (r != Z_STREAM_END) return false;  // the next call resets the stream
  out->resize(zs.total_out);
  return true;
}

const std::string* Snapshot::gzipped(bool compress_now) const {
  if (!gzip) return nullptr;
  gz_asked_.store(true, std::memory_order_relaxed);
  int st = gz_state_.load(std::memory_order_acquire);
  if (st == 0 && compress_now) {
    if (claim(&st)) return compress_claimed();
    // lost the claim to a concurrent compression: st is its state now (1, 2 or 3)
  }
  if (st == 1) {
    // another thread (the tick thread's eager / predicted compression, or a concurrent scrape) is
    // compressing this snapshot right now: wait for it (0.1-0.8 ms for 1-8 GPUs) rather than answer
    // with the 5-10x larger identity body -- but at most kGzipWaitNs: this runs on an HTTP loop
    // (possibly at SCHED_FIFO), and every other connection of the loop waits with it (it
    // was 20 ms). Past the budget the identity body goes out.
    const int64_t until = mono_ns() + kGzipWaitNs;
    while ((st = gz_state_.load(std::memory_order_acquire)) == 1 && mono_ns() < until)
      std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  return st == 2 ? &gz_ : nullptr;
}

bool Snapshot::precompress() const {
  if (!gzip) return false;
  int st = gz_state_.load(std::memory_order_acquire);
  return st == 0 && claim(&st) && compress_claimed() != nullptr;
}

bool Snapshot::claim(int* st) const {
  return gz_state_.compare_exchange_strong(*st, 1, std::memory_order_acq_rel);
}

const std::string* Snapshot::compress_claimed() const {
  const bool ok = gzip_compress(body, &gz_, 1);
  gz_state_.store(ok ? 2 : 3, std::memory_order_release);
  return ok ? &gz_ : nullptr;
}

}  // namespace gpumon

#include "xgmi_map.h"

#include <algorithm>

namespace gpumon {

namespace {

uint64_t absdiff(uint64_t a, uint64_t b) { return a > b ? a - b : b - a; }

bool close_abs(uint64_t a, uint64_t b) {
  return absdiff(a, b) <= XgmiSlotMap::kAbsTolKB + std::max(a, b) / 10000;
}

bool close_delta(uint64_t a, uint64_t b) {
  return static_cast<double>(absdiff(a, b)) <= 1024.0 + 0.03 * static_cast<double>(std::max(a, b));
}

}  // namespace

void XgmiSlotMap::update(const DeviceSample& s) {
  const auto& e = s.link_entries;
  const Accumulators& a = s.acc;
  const size_t n = e.size();
  const int nslots = std::min(a.n_links_acc, kMaxLinks);
  if (slot_.size() != n) {  // first refresh, or the entry list changed shape: positional start
    slot_.assign(n, -1);
    for (size_t j = 0; j < n && j < static_cast<size_t>(kMaxLinks); ++j) slot_[j] = static_cast<int>(j);
    verified_.assign(n, 0);
    have_base_ = false;
  }
  has_peer_.assign(n, 0);
  peer_.resize(n);
  for (size_t j = 0; j < n; ++j) {
    has_peer_[j] = !e[j].peer_bdf.empty();
    if (e[j].peer_bdf != peer_[j]) {  // the entry now names another peer: earlier evidence is void
      verified_[j] = 0;
      slot_[j] = j < static_cast<size_t>(kMaxLinks) ? static_cast<int>(j) : -1;
      peer_[j] = e[j].peer_bdf;
    }
  }
  // slots that can carry a peer: listed in the table (status known) with counters
  auto slot_ok = [&](int k) { return a.valid && k < nslots && s.links[k].status >= 0; };
  std::vector<int> match(n, -1);
  for (size_t j = 0; j < n; ++j) {
    if (!has_peer_[j] || !e[j].has_acc) continue;
    // 1. absolute counters: libamd_smi fills the entries from the same firmware table (measured on
    // MI355X: every entry equals its slot to the KB), so one slot with IDENTICAL counters pairs it
    // (idle links keep their counts between the two reads); else one slot within the traffic the
    // link can move between the reads
    int found = -1, count = 0;
    if (e[j].read_kb + e[j].write_kb > 0) {
      for (int k = 0; k < nslots; ++k)
        if (slot_ok(k) && e[j].read_kb == a.xgmi_rd_kb[k] && e[j].write_kb == a.xgmi_wr_kb[k]) {
          found = k;
          ++count;
        }
      if (count == 1) {
        match[j] = found;
        continue;
      }
    }
    found = -1;
    count = 0;
    for (int k = 0; k < nslots; ++k)
      if (slot_ok(k) && close_abs(e[j].read_kb, a.xgmi_rd_kb[k]) && close_abs(e[j].write_kb, a.xgmi_wr_kb[k])) {
        found = k;
        ++count;
      }
    if (count == 1) {
      match[j] = found;
      continue;
    }
    // 2. deltas since the last refresh (a source whose counters have another origin)
    if (!have_base_ || j >= base_ok_.size() || !base_ok_[j] || !base_.valid) continue;
    if (e[j].read_kb < base_erd_[j] || e[j].write_kb < base_ewr_[j]) continue;  // wrapped / reset
    const uint64_t dr = e[j].read_kb - base_erd_[j], dw = e[j].write_kb - base_ewr_[j];
    if (dr + dw < kMinDeltaKB) continue;  // too little traffic to tell links apart
    found = -1;
    count = 0;
    for (int k = 0; k < nslots && k < base_.n_links_acc; ++k) {
      if (!slot_ok(k) || a.xgmi_rd_kb[k] < base_.xgmi_rd_kb[k] || a.xgmi_wr_kb[k] < base_.xgmi_wr_kb[k]) continue;
      if (close_delta(dr, a.xgmi_rd_kb[k] - base_.xgmi_rd_kb[k]) && close_delta(dw, a.xgmi_wr_kb[k] - base_.xgmi_wr_kb[k])) {
        found = k;
        ++count;
      }
    }
    if (count == 1) match[j] = found;
  }
  // two entries claiming one slot: neither is evidence
  for (size_t j = 0; j < n; ++j)
    for (size_t m = j + 1; m < n; ++m)
      if (match[j] >= 0 && match[j] == match[m]) match[j] = match[m] = -2;
  for (size_t j = 0; j < n; ++j)
    if (match[j] >= 0) {
      slot_[j] = match[j];
      verified_[j] = 1;
    } else if (match[j] == -2) {
      verified_[j] = 0;
    }
  // Slots held by verified entries (this refresh or an earlier one; this refresh's evidence wins
  // over an older pairing of the same slot). An unverified entry on such a slot, or a verified one
  // that lost its slot to newer evidence, has its peer withheld, not guessed.
  std::vector<int> owner(kMaxLinks, -1);
  for (size_t j = 0; j < n; ++j)
    if (match[j] >= 0) owner[match[j]] = static_cast<int>(j);
  for (size_t j = 0; j < n; ++j)
    if (verified_[j] && match[j] < 0 && slot_[j] >= 0 && owner[slot_[j]] < 0) owner[slot_[j]] = static_cast<int>(j);
  for (size_t j = 0; j < n; ++j)
    if (slot_[j] >= 0 && owner[slot_[j]] >= 0 && owner[slot_[j]] != static_cast<int>(j)) {
      slot_[j] = -1;
      verified_[j] = 0;
    }
  base_erd_.assign(n, 0);
  base_ewr_.assign(n, 0);
  base_ok_.assign(n, 0);
  for (size_t j = 0; j < n; ++j) {
    base_erd_[j] = e[j].read_kb;
    base_ewr_[j] = e[j].write_kb;
    base_ok_[j] = e[j].has_acc;
  }
  base_ = a;
  have_base_ = true;
}

void XgmiSlotMap::apply(const std::vector<LinkEntry>& e, DeviceSample* s) const {
  for (size_t j = 0; j < e.size() && j < slot_.size(); ++j) {
    const int k = slot_[j];
    if (k < 0 || k >= kMaxLinks) continue;
    LinkInfo& L = s->links[k];
    L.peer_bdf = e[j].peer_bdf;
    L.bit_rate_gbps = e[j].bit_rate_gbps;
    L.max_bandwidth_gbps = e[j].max_bandwidth_gbps;
    L.link_type = e[j].link_type;
    if (k + 1 > s->n_links) s->n_links = k + 1;
  }
}

int XgmiSlotMap::verified() const {
  int c = 0;
  for (size_t j = 0; j < slot_.size(); ++j) c += has_peer_.size() > j && has_peer_[j] && verified_[j] ? 1 : 0;
  return c;
}

int XgmiSlotMap::mismatched() const {
  int c = 0;
  for (size_t j = 0; j < slot_.size(); ++j)
    c += has_peer_.size() > j && has_peer_[j] && verified_[j] && slot_[j] != static_cast<int>(j) ? 1 : 0;
  return c;
}

int XgmiSlotMap::unverified() const {
  int c = 0;
  for (size_t j = 0; j < slot_.size(); ++j) c += has_peer_.size() > j && has_peer_[j] && !verified_[j] ? 1 : 0;
  return c;
}

}  // namespace gpumon

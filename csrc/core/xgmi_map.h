// xGMI peer identity: which gpu_metrics link slot does each amdsmi_get_link_metrics entry describe?
//
// The exporter takes per-link traffic and status from the firmware table's slots
// (gpu_metrics.xgmi_read/write_data_acc[8], xgmi_link_status[8]; read every tick) and the peer BDF /
// bit rate / max bandwidth from amdsmi_get_link_metrics (read every `link_every` ticks). The two
// lists differ in length on MI355X (7 entries vs 8 slots) and nothing documents that their orders
// agree -- pairing them by position would export every per-peer rate under the wrong peer the
// moment they do not. Each link-metrics entry carries its own read/write KB
// accumulators, so an entry is paired with the slot whose accumulators it matches:
//   1. absolute: the entry's counters equal one slot's (both sources read within ~1 ms), or
//   2. delta: over the interval between two refreshes, the entry's Δread/Δwrite equal one slot's.
// A pairing is taken only when exactly one slot fits (idle or perfectly balanced traffic, e.g. a
// ring all-reduce loading every link alike, cannot tell links apart); unpaired entries keep their
// previous slot (initially the positional one) unless a paired entry claims it, in which case
// their peer is withheld rather than guessed. The reference never looked at NVLink at all
// (/root/reference/gpu.py:104-116); SURVEY D7 names these fields.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "sample.h"

namespace gpumon {

class XgmiSlotMap {
 public:
  // One link-refresh tick of a device: s.link_entries are the link-metrics entries, s.acc / s.links
  // the firmware slots' accumulators / status from the same sample. Updates the pairing.
  void update(const DeviceSample& s);
  // Writes each paired entry's identity onto its slot of `s` (peer BDF, bit rate, max bandwidth,
  // type); slots no entry describes keep what they had.
  void apply(const std::vector<LinkEntry>& e, DeviceSample* s) const;

  int slot_of(size_t entry) const { return entry < slot_.size() ? slot_[entry] : -1; }
  // entries with a peer whose slot was confirmed by traffic / differs from their position
  int verified() const;
  int mismatched() const;
  int unverified() const;  // entries with a peer not (yet) confirmed by traffic
  bool empty() const { return slot_.empty(); }

  // Tolerances (KB). Absolute: both sources are read within ~1 ms, at most ~64 MB of traffic apart
  // on a busy link; delta: 3 % of the interval's traffic + 1 MB, and at least 64 MB moved.
  static constexpr uint64_t kAbsTolKB = 65536;
  static constexpr uint64_t kMinDeltaKB = 65536;

 private:
  std::vector<int> slot_;          // per entry, -1 = no slot
  std::vector<char> verified_;     // per entry: slot confirmed by traffic at least once
  std::vector<char> has_peer_;
  std::vector<std::string> peer_;  // per entry: peer BDF at the last refresh
  bool have_base_ = false;
  std::vector<uint64_t> base_erd_, base_ewr_;
  std::vector<char> base_ok_;  // per entry: counters present at the base refresh
  Accumulators base_;
};

}  // namespace gpumon

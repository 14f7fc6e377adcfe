// RAS / ECC sysfs readers (see ras.h).
#include "ras.h"

#include <dirent.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.h"

namespace gpumon {

namespace {

// Value after `key` (e.g. "ue:") on its line, or -1.
long long field_after(const std::string& text, const char* key) {
  size_t p = text.find(key);
  if (p == std::string::npos) return -1;
  p += strlen(key);
  while (p < text.size() && (text[p] == ' ' || text[p] == '\t')) ++p;
  if (p >= text.size() || text[p] < '0' || text[p] > '9') return -1;
  return strtoll(text.c_str() + p, nullptr, 10);
}

}  // namespace

bool parse_err_count(const std::string& text, RasCount* out) {
  const long long ue = field_after(text, "ue:"), ce = field_after(text, "ce:"), de = field_after(text, "de:");
  if (ue < 0 && ce < 0) return false;
  out->ue = ue > 0 ? static_cast<uint64_t>(ue) : 0;
  out->ce = ce > 0 ? static_cast<uint64_t>(ce) : 0;
  out->has_de = de >= 0;
  out->de = de > 0 ? static_cast<uint64_t>(de) : 0;
  return true;
}

void parse_event_state(const std::string& text, RasSample* out) {
  for (const auto& line : split(text, '\n')) {
    const std::string l(trim(line));
    const long long c = field_after(l, "count:");
    if (c < 0) continue;
    if (starts_with(l, "Fatal Error")) out->fatal = static_cast<double>(c);
    else if (starts_with(l, "Poison Creation")) out->poison_created = static_cast<double>(c);
    else if (starts_with(l, "Poison Consumption")) out->poison_consumed = static_cast<double>(c);
  }
}

int count_bad_pages(const std::string& text) {
  int n = 0;
  for (const auto& line : split(text, '\n'))
    if (starts_with(trim(line), "0x")) ++n;
  return n;
}

RasSysfsReader::RasSysfsReader(const std::string& sys_root, const std::string& bdf)
    : dir_(bdf.empty() ? std::string() : sys_root + "/bus/pci/devices/" + bdf + "/ras") {}

bool RasSysfsReader::list() {
  listed_ = true;
  files_.clear();
  if (dir_.empty()) return false;
  DIR* d = opendir(dir_.c_str());
  if (!d) return false;
  has_events_ = has_bad_pages_ = false;
  while (dirent* e = readdir(d)) {
    const std::string f = e->d_name;
    if (f == "event_state") has_events_ = true;
    else if (f == "gpu_vram_bad_pages") has_bad_pages_ = true;
    else if (starts_with(f, "aca_")) files_.emplace_back(f.substr(4), f);
    else if (ends_with(f, "_err_count")) files_.emplace_back(f.substr(0, f.size() - 10), f);
  }
  closedir(d);
  // an ACA file and a legacy file for the same block: keep the ACA one (it carries deferred);
  // "aca_x" sorts before "x_err_count" within a block once keyed by block name
  std::sort(files_.begin(), files_.end(), [](const auto& a, const auto& b) {
    if (a.first != b.first) return a.first < b.first;
    return starts_with(a.second, "aca_") && !starts_with(b.second, "aca_");
  });
  files_.erase(std::unique(files_.begin(), files_.end(),
                           [](const auto& a, const auto& b) { return a.first == b.first; }),
               files_.end());
  return !files_.empty();
}

bool RasSysfsReader::read(int slice, int nslices, RasSample* out) {
  const bool full = !cur_.valid;
  if (full && !list()) return false;
  if (nslices < 1) nslices = 1;
  auto mine = [&](size_t k) { return full || static_cast<int>(k % static_cast<size_t>(nslices)) == slice; };
  RasSample r;
  r.source = "sysfs";
  std::string text;
  int failed = 0;
  for (size_t k = 0; k < files_.size(); ++k) {
    RasCount c;
    c.block = files_[k].first;
    const RasCount* prev = nullptr;
    for (const auto& p : cur_.blocks)
      if (p.block == c.block) prev = &p;
    if (mine(k)) {
      if (read_file(dir_ + "/" + files_[k].second, &text, 4096) && parse_err_count(text, &c)) {
        r.blocks.push_back(c);
      } else {
        failed++;
        if (prev) r.blocks.push_back(*prev);  // transient read failure: keep the last count
      }
    } else if (prev) {
      r.blocks.push_back(*prev);
    }
  }
  if (r.blocks.empty()) return false;
  // event_state and bad pages: carried from the last reading when not due OR when the read fails
  // (a failed read must not blank the fatal / poison / bad-page series for a cycle)
  r.fatal = cur_.fatal;
  r.poison_created = cur_.poison_created;
  r.poison_consumed = cur_.poison_consumed;
  r.bad_pages = cur_.bad_pages;
  const size_t ev = files_.size(), bp = files_.size() + 1;
  if (mine(ev) && has_events_) {
    if (read_file(dir_ + "/event_state", &text, 4096)) parse_event_state(text, &r);
    else failed++;
  }
  if (mine(bp) && has_bad_pages_) {
    if (read_file(dir_ + "/gpu_vram_bad_pages", &text, 1 << 20)) r.bad_pages = count_bad_pages(text);
    else failed++;
  }
  r.valid = true;
  r.stale_items = failed;
  cur_ = r;
  *out = std::move(r);
  return true;
}

bool read_ras_sysfs(const std::string& sys_root, const std::string& bdf, RasSample* out) {
  RasSysfsReader r(sys_root, bdf);
  return r.read(0, 1, out);
}

}  // namespace gpumon

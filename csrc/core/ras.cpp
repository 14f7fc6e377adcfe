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

bool read_ras_sysfs(const std::string& sys_root, const std::string& bdf, RasSample* out) {
  if (bdf.empty()) return false;
  const std::string dir = sys_root + "/bus/pci/devices/" + bdf + "/ras";
  DIR* d = opendir(dir.c_str());
  if (!d) return false;
  std::vector<std::pair<std::string, std::string>> files;  // (block, file)
  while (dirent* e = readdir(d)) {
    const std::string f = e->d_name;
    if (starts_with(f, "aca_")) files.emplace_back(f.substr(4), f);
    else if (ends_with(f, "_err_count")) files.emplace_back(f.substr(0, f.size() - 10), f);
  }
  closedir(d);
  if (files.empty()) return false;
  std::sort(files.begin(), files.end());
  RasSample r;
  r.source = "sysfs";
  std::string text;
  for (const auto& bf : files) {
    // an ACA file and a legacy file for the same block: keep the ACA one (it carries deferred)
    if (!r.blocks.empty() && r.blocks.back().block == bf.first) continue;
    RasCount c;
    c.block = bf.first;
    if (read_file(dir + "/" + bf.second, &text, 4096) && parse_err_count(text, &c)) r.blocks.push_back(c);
  }
  if (r.blocks.empty()) return false;
  if (read_file(dir + "/event_state", &text, 4096)) parse_event_state(text, &r);
  if (read_file(dir + "/gpu_vram_bad_pages", &text, 1 << 20)) r.bad_pages = count_bad_pages(text);
  r.valid = true;
  *out = std::move(r);
  return true;
}

}  // namespace gpumon

#include "sysfs_fast.h"

#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace gpumon {

namespace {

int open_ro(const std::string& p) { return ::open(p.c_str(), O_RDONLY | O_CLOEXEC); }

// pread at offset 0 re-runs the attribute's show() (kernfs restarts the seq_file at pos 0). kernfs
// hands out at most a page per read and a show() fills its whole content at once, so a read that
// returns less than a request of at most a page is the whole file: no second pread() just to see
// EOF (one syscall per small read instead of two).
ssize_t pread_all(int fd, void* buf, size_t cap) {
  constexpr size_t kPage = 4096;
  size_t got = 0;
  while (got < cap) {
    const size_t want = cap - got;
    ssize_t r = ::pread(fd, static_cast<char*>(buf) + got, want, static_cast<off_t>(got));
    if (r < 0) return -1;
    if (r == 0) break;
    got += static_cast<size_t>(r);
    if (static_cast<size_t>(r) < want && want <= kPage) break;  // short read of <= a page: the end
  }
  return static_cast<ssize_t>(got);
}

bool pread_u64(int fd, uint64_t* v) {
  char b[64];
  ssize_t n = pread_all(fd, b, sizeof b - 1);
  if (n <= 0) return false;
  b[n] = 0;
  char* end = nullptr;
  unsigned long long x = strtoull(b, &end, 10);
  if (end == b) return false;
  *v = x;
  return true;
}

bool read_small(const std::string& p, char* b, size_t cap, size_t* n) {
  int fd = open_ro(p);
  if (fd < 0) return false;
  ssize_t r = pread_all(fd, b, cap - 1);
  ::close(fd);
  if (r < 0) return false;
  b[r] = 0;
  *n = static_cast<size_t>(r);
  return true;
}

// "key:\t123 unit" -> 123 ; returns false if the key is absent.
bool fdinfo_value(const char* text, const char* key, uint64_t* v) {
  const char* p = strstr(text, key);
  while (p && p != text && p[-1] != '\n') p = strstr(p + 1, key);
  if (!p) return false;
  p += strlen(key);
  while (*p == ' ' || *p == '\t') ++p;
  char* end = nullptr;
  unsigned long long x = strtoull(p, &end, 10);
  if (end == p) return false;
  while (*end == ' ') ++end;
  if (!strncmp(end, "KiB", 3)) x *= 1024ull;
  else if (!strncmp(end, "MiB", 3)) x *= 1048576ull;
  *v = x;
  return true;
}

}  // namespace

SysfsGpu::~SysfsGpu() {
  for (int fd : {fd_metrics_, fd_vram_used_, fd_vram_total_, fd_gtt_used_})
    if (fd >= 0) ::close(fd);
  std::lock_guard<std::mutex> g(kfd_fds_mu_);
  for (auto& [k, fd] : kfd_fds_) ::close(fd);
}

bool SysfsGpu::read_kfd(uint32_t pid, KfdFile kind, char* b, size_t cap, size_t* n) {
  const uint64_t key = (static_cast<uint64_t>(pid) << 1) | static_cast<uint64_t>(kind);
  int fd = -1;
  {
    std::lock_guard<std::mutex> g(kfd_fds_mu_);
    auto it = kfd_fds_.find(key);
    if (it != kfd_fds_.end()) {
      fd = it->second;
      kfd_fds_.erase(it);  // taken out while read: a concurrent caller opens its own
    }
  }
  if (fd >= 0) {
    const ssize_t r = pread_all(fd, b, cap - 1);
    if (r > 0) {
      b[r] = 0;
      *n = static_cast<size_t>(r);
      std::lock_guard<std::mutex> g(kfd_fds_mu_);
      if (!kfd_fds_.emplace(key, fd).second) ::close(fd);
      kfd_reads_cached_.fetch_add(1, std::memory_order_relaxed);
      return true;
    }
    // the process exited (its kobject is gone: ENODEV) or the pid was reused: a fresh open below
    ::close(fd);
  }
  const std::string path = sys_root_ + "/class/kfd/kfd/proc/" + std::to_string(pid) +
                           (kind == KfdFile::kVram ? "/vram_" + std::to_string(kfd_gpu_id_)
                                                   : "/stats_" + std::to_string(kfd_gpu_id_) + "/cu_occupancy");
  fd = open_ro(path);
  if (fd < 0) return false;
  const ssize_t r = pread_all(fd, b, cap - 1);
  if (r < 0) {
    ::close(fd);
    return false;
  }
  b[r] = 0;
  *n = static_cast<size_t>(r);
  std::lock_guard<std::mutex> g(kfd_fds_mu_);
  if (kfd_fds_.size() >= kMaxKfdFds || !kfd_fds_.emplace(key, fd).second) ::close(fd);
  return true;
}

void SysfsGpu::retain_kfd(const std::vector<uint32_t>& listed_sorted) {
  std::lock_guard<std::mutex> g(kfd_fds_mu_);
  for (auto it = kfd_fds_.begin(); it != kfd_fds_.end();) {
    if (!std::binary_search(listed_sorted.begin(), listed_sorted.end(), static_cast<uint32_t>(it->first >> 1))) {
      ::close(it->second);
      it = kfd_fds_.erase(it);
    } else {
      ++it;
    }
  }
}

size_t SysfsGpu::kfd_fds() {
  std::lock_guard<std::mutex> g(kfd_fds_mu_);
  return kfd_fds_.size();
}

bool SysfsGpu::open(const std::string& sys_root, const std::string& proc_root, const std::string& bdf,
                    uint64_t kfd_gpu_id, int drm_render, std::string* why) {
  sys_root_ = sys_root.empty() ? "/sys" : sys_root;
  proc_root_ = proc_root.empty() ? "/proc" : proc_root;
  dev_dir_ = sys_root_ + "/bus/pci/devices/" + bdf;
  kfd_gpu_id_ = kfd_gpu_id;
  if (drm_render >= 0) render_path_ = "/dev/dri/renderD" + std::to_string(drm_render);
  fd_metrics_ = open_ro(dev_dir_ + "/gpu_metrics");
  if (fd_metrics_ < 0) {
    if (why) *why = dev_dir_ + "/gpu_metrics: " + strerror(errno);
    return false;
  }
  fd_vram_used_ = open_ro(dev_dir_ + "/mem_info_vram_used");
  fd_vram_total_ = open_ro(dev_dir_ + "/mem_info_vram_total");
  fd_gtt_used_ = open_ro(dev_dir_ + "/mem_info_gtt_used");
  return true;
}

bool SysfsGpu::prewarm() {
  alignas(8) unsigned char buf[4096];
  return fd_metrics_ >= 0 && pread_all(fd_metrics_, buf, sizeof buf) > 0;
}

bool SysfsGpu::read_metrics(kgm::V18* out, std::string* why) {
  alignas(8) unsigned char buf[4096];
  ssize_t n = pread_all(fd_metrics_, buf, sizeof buf);
  if (n < static_cast<ssize_t>(sizeof(kgm::Header))) {
    if (why) *why = "gpu_metrics: short read";
    return false;
  }
  kgm::Header h;
  memcpy(&h, buf, sizeof h);
  if (h.format_revision != 1 || h.content_revision != 8 || h.structure_size != sizeof(kgm::V18) ||
      n < static_cast<ssize_t>(sizeof(kgm::V18))) {
    if (why)
      *why = "gpu_metrics: unsupported table v" + std::to_string(h.format_revision) + "." +
             std::to_string(h.content_revision) + " size " + std::to_string(h.structure_size);
    return false;
  }
  memcpy(out, buf, sizeof *out);
  return true;
}

bool SysfsGpu::read_vram(double* used, double* total) {
  uint64_t u = 0, t = 0;
  if (fd_vram_used_ < 0 || !pread_u64(fd_vram_used_, &u)) return false;
  *used = static_cast<double>(u);
  if (fd_vram_total_ >= 0 && pread_u64(fd_vram_total_, &t)) *total = static_cast<double>(t);
  return true;
}

bool SysfsGpu::read_gtt(double* used) {
  uint64_t u = 0;
  if (fd_gtt_used_ < 0 || !pread_u64(fd_gtt_used_, &u)) return false;
  *used = static_cast<double>(u);
  return true;
}

DrmFdTables& DrmFdTables::get() {
  static DrmFdTables t;
  return t;
}

void DrmFdTables::scan(const std::string& pdir, std::vector<std::pair<int, std::string>>* fds) {
  fds->clear();
  DIR* d = opendir((pdir + "/fd").c_str());
  if (!d) return;
  char target[256];
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    ssize_t n = readlink((pdir + "/fd/" + e->d_name).c_str(), target, sizeof target - 1);
    if (n <= 0) continue;
    target[n] = 0;
    if (!strncmp(target, "/dev/dri/", 9)) fds->emplace_back(atoi(e->d_name), target);
  }
  closedir(d);
}

void DrmFdTables::fds_for(const std::string& pdir, const std::string& render, std::vector<int>* out) {
  out->clear();
  const int64_t now = mono_ns();
  std::unique_lock<std::mutex> lk(mu_);
  auto it = m_.find(pdir);
  if (it == m_.end()) {
    // first sight: scan now (this tick), outside the lock, once: another GPU's worker that needs
    // the same process meanwhile waits for this scan instead of repeating it
    m_[pdir].scanning = true;
    lk.unlock();
    std::vector<std::pair<int, std::string>> fds;
    scan(pdir, &fds);
    scans_++;
    lk.lock();
    Entry& e = m_[pdir];
    e.scans++;
    e.fds = std::move(fds);
    e.scanned_ns = e.used_ns = now;
    e.scanning = false;
    cv_.notify_all();
    it = m_.find(pdir);
  } else {
    cv_.wait(lk, [&] {
      it = m_.find(pdir);
      return it == m_.end() || !it->second.scanning;
    });
    if (it == m_.end()) return;
  }
  Entry& e = it->second;
  e.used_ns = now;
  if (now - e.scanned_ns > 10'000'000'000ll) e.want = true;  // refreshed off the tick
  for (const auto& [fd, target] : e.fds)
    if (target == render) out->push_back(fd);
}

void DrmFdTables::invalidate(const std::string& pdir) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(pdir);
  if (it != m_.end()) it->second.want = true;
}

int DrmFdTables::refresh_due(int max_scans) {
  const int64_t now = mono_ns();
  std::vector<std::string> due;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = m_.begin(); it != m_.end();) {
      if (!it->second.scanning && now - it->second.used_ns > 60'000'000'000ll) {  // unlisted for 60 s
        it = m_.erase(it);
        continue;
      }
      if (it->second.want && static_cast<int>(due.size()) < max_scans) {
        it->second.want = false;  // claimed: another worker's maintain() skips it
        due.push_back(it->first);
      }
      ++it;
    }
  }
  for (const auto& pdir : due) {
    std::vector<std::pair<int, std::string>> fds;
    scan(pdir, &fds);
    scans_++;
    std::lock_guard<std::mutex> g(mu_);
    auto it = m_.find(pdir);
    if (it == m_.end()) continue;
    it->second.scans++;
    it->second.fds = std::move(fds);
    it->second.scanned_ns = mono_ns();
  }
  return static_cast<int>(due.size());
}

void DrmFdTables::retain(const std::string& proc_root, const std::vector<uint32_t>& kfd_pids) {
  const std::string prefix = proc_root + "/";
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = m_.begin(); it != m_.end();) {
    const std::string& pdir = it->first;
    if (!it->second.scanning && pdir.compare(0, prefix.size(), prefix) == 0) {
      const uint32_t pid = static_cast<uint32_t>(strtoul(pdir.c_str() + prefix.size(), nullptr, 10));
      if (!std::binary_search(kfd_pids.begin(), kfd_pids.end(), pid)) {
        it = m_.erase(it);
        continue;
      }
    }
    ++it;
  }
}

uint32_t DrmFdTables::scans_of(const std::string& pdir) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(pdir);
  return it == m_.end() ? 0 : it->second.scans;
}

void DrmFdTables::clear() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = m_.begin(); it != m_.end();) {
    if (it->second.scanning) ++it;
    else it = m_.erase(it);
  }
}

size_t DrmFdTables::size() {
  std::lock_guard<std::mutex> g(mu_);
  return m_.size();
}

void SysfsGpu::maintain() { DrmFdTables::get().refresh_due(64); }

void SysfsGpu::fdinfo_usage(uint32_t pid, ProcSample* p) {
  if (render_path_.empty()) return;
  const std::string base = proc_root_ + "/" + std::to_string(pid);
  std::vector<int> fds;
  DrmFdTables::get().fds_for(base, render_path_, &fds);
  if (fds.empty()) return;
  uint64_t gfx = 0, vram = 0, gtt = 0, cpu = 0;
  bool any = false, have_vram = false;
  std::vector<uint64_t> clients;
  char text[4096];
  for (int fd : fds) {
    size_t n = 0;
    if (!read_small(base + "/fdinfo/" + std::to_string(fd), text, sizeof text, &n)) {
      DrmFdTables::get().invalidate(base);  // fd closed: rescan off the tick
      continue;
    }
    uint64_t cid = 0;
    if (fdinfo_value(text, "drm-client-id:", &cid)) {
      bool dup = false;
      for (uint64_t x : clients) dup |= (x == cid);
      if (dup) continue;  // dup()'ed fd of the same DRM file
      clients.push_back(cid);
    }
    uint64_t v = 0;
    if (fdinfo_value(text, "drm-engine-gfx:", &v)) {
      gfx += v;
      any = true;
    }
    if (fdinfo_value(text, "drm-memory-vram:", &v)) {
      vram += v;
      have_vram = true;
    }
    if (fdinfo_value(text, "drm-memory-gtt:", &v)) gtt += v;
    if (fdinfo_value(text, "drm-memory-cpu:", &v)) cpu += v;
  }
  if (any) {
    p->gfx_ns = gfx;
    p->has_gfx_ns = true;
  }
  if (have_vram) {
    p->vram_bytes = static_cast<double>(vram);
    p->gtt_bytes = static_cast<double>(gtt);
    p->cpu_bytes = static_cast<double>(cpu);
  }
}

void SysfsGpu::occupancy(const std::vector<uint32_t>& pids, std::vector<double>* out) {
  out->assign(pids.size(), kNaN);
  if (!kfd_gpu_id_) return;
  char b[64];
  for (size_t k = 0; k < pids.size(); ++k) {
    size_t n = 0;
    if (read_kfd(pids[k], KfdFile::kOccupancy, b, sizeof b, &n))
      (*out)[k] = static_cast<double>(strtoull(b, nullptr, 10));
  }
}

bool SysfsGpu::skip_not_here(uint32_t pid, int64_t now) {
  std::lock_guard<std::mutex> g(not_here_mu_);
  auto it = not_here_.find(pid);
  return it != not_here_.end() && now < it->second;
}

void SysfsGpu::note_not_here(uint32_t pid, int64_t now) {
  std::lock_guard<std::mutex> g(not_here_mu_);
  not_here_[pid] = now + kNotHereNs;
}

void SysfsGpu::prune_not_here(const std::vector<uint32_t>& listed_sorted) {
  std::lock_guard<std::mutex> g(not_here_mu_);
  for (auto it = not_here_.begin(); it != not_here_.end();) {
    if (!std::binary_search(listed_sorted.begin(), listed_sorted.end(), it->first)) it = not_here_.erase(it);
    else ++it;
  }
}

int SysfsGpu::queues_here(uint32_t pid, int64_t now) {
  // A process's user-mode queues are created when its runtime first submits work to a GPU (a
  // kernel, a copy) and live as long as its streams: a context that only allocated -- the usual
  // peer context of an RCCL rank or P2P importer -- has none there (profiles/r6_kfd_queues.md).
  return KfdQueueTables::get().count(sys_root_ + "/class/kfd/kfd/proc", pid, kfd_gpu_id_, now);
}

KfdQueueTables& KfdQueueTables::get() {
  static KfdQueueTables t;
  return t;
}

bool KfdQueueTables::scan(const std::string& qdir, std::vector<std::pair<uint64_t, int>>* per_gpu) {
  per_gpu->clear();
  DIR* d = opendir(qdir.c_str());
  if (!d) return false;
  char b[32];
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    const std::string f = qdir + "/" + e->d_name + "/gpuid";
    const int fd = ::open(f.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) continue;  // the queue went away between readdir and open
    const ssize_t n = ::read(fd, b, sizeof b - 1);
    ::close(fd);
    if (n <= 0) continue;
    b[n] = 0;
    const uint64_t gid = strtoull(b, nullptr, 10);
    auto it = std::find_if(per_gpu->begin(), per_gpu->end(), [gid](const auto& x) { return x.first == gid; });
    if (it == per_gpu->end()) per_gpu->emplace_back(gid, 1);
    else ++it->second;
  }
  closedir(d);
  return true;
}

int KfdQueueTables::count(const std::string& kfd_proc, uint32_t pid, uint64_t gpu_id, int64_t now) {
  auto answer = [gpu_id](const Entry& e) {
    if (!e.readable) return -1;
    for (const auto& x : e.per_gpu)
      if (x.first == gpu_id) return x.second;
    return 0;
  };
  {
    std::lock_guard<std::mutex> g(mu_);
    auto& byp = m_[kfd_proc];
    auto it = byp.find(pid);
    if (it != byp.end() && it->second.scans > 0 && now - it->second.scanned_ns < kRescanNs) return answer(it->second);
  }
  // scanned outside the lock (the device workers of other GPUs read their cached answers
  // meanwhile); two workers racing on one stale entry both scan, harmlessly
  Entry fresh;
  fresh.readable = scan(kfd_proc + "/" + std::to_string(pid) + "/queues", &fresh.per_gpu);
  fresh.scanned_ns = now;
  scans_.fetch_add(1, std::memory_order_relaxed);
  std::lock_guard<std::mutex> g(mu_);
  Entry& e = m_[kfd_proc][pid];
  fresh.scans = e.scans + 1;
  e = std::move(fresh);
  return answer(e);
}

void KfdQueueTables::retain(const std::string& kfd_proc, const std::vector<uint32_t>& listed_sorted) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(kfd_proc);
  if (it == m_.end()) return;
  for (auto p = it->second.begin(); p != it->second.end();)
    p = std::binary_search(listed_sorted.begin(), listed_sorted.end(), p->first) ? std::next(p) : it->second.erase(p);
}

void KfdQueueTables::clear() {
  std::lock_guard<std::mutex> g(mu_);
  m_.clear();
}

uint32_t KfdQueueTables::scans_of(const std::string& kfd_proc, uint32_t pid) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(kfd_proc);
  if (it == m_.end()) return 0;
  auto p = it->second.find(pid);
  return p == it->second.end() ? 0 : p->second.scans;
}

bool SysfsGpu::processes(std::vector<ProcSample>* out, bool read_occupancy) {
  out->clear();
  if (!kfd_gpu_id_) return false;
  const std::string kdir = sys_root_ + "/class/kfd/kfd/proc";
  DIR* d = opendir(kdir.c_str());
  if (!d) return false;
  char b[64];
  std::vector<uint32_t> listed;  // every KFD process of the node (any GPU)
  const int64_t now = mono_ns();
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    const uint32_t pid = static_cast<uint32_t>(strtoul(e->d_name, nullptr, 10));
    listed.push_back(pid);
    if (skip_not_here(pid, now)) continue;
    size_t n = 0;
    if (!read_kfd(pid, KfdFile::kVram, b, sizeof b, &n)) {  // process not on this GPU
      note_not_here(pid, now);
      continue;
    }
    ProcSample p;
    p.pid = pid;
    p.mem_bytes = static_cast<double>(strtoull(b, nullptr, 10));
    p.vram_bytes = p.mem_bytes;
    if (read_occupancy && read_kfd(pid, KfdFile::kOccupancy, b, sizeof b, &n))
      p.cu_occupancy = static_cast<double>(strtoull(b, nullptr, 10));
    p.queues = queues_here(pid, now);
    fdinfo_usage(pid, &p);
    out->push_back(std::move(p));
  }
  closedir(d);
  std::sort(listed.begin(), listed.end());
  KfdQueueTables::get().retain(kdir, listed);  // pids that left the listing
  DrmFdTables::get().retain(proc_root_, listed);
  prune_not_here(listed);
  retain_kfd(listed);  // close the kept files of processes that left
  return true;
}

bool SysfsGpu::occupancy_scan(std::vector<OccRead>* out) {
  out->clear();
  if (!kfd_gpu_id_) return false;
  const std::string kdir = sys_root_ + "/class/kfd/kfd/proc/";
  DIR* d = opendir(kdir.c_str());
  if (!d) return false;
  char b[64];
  const int64_t now = mono_ns();
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    const uint32_t pid = static_cast<uint32_t>(strtoul(e->d_name, nullptr, 10));
    if (skip_not_here(pid, now)) continue;
    size_t n = 0;
    if (!read_kfd(pid, KfdFile::kVram, b, sizeof b, &n)) {  // not on this GPU
      note_not_here(pid, now);
      continue;
    }
    OccRead r;
    r.pid = pid;
    r.vram_bytes = static_cast<double>(strtoull(b, nullptr, 10));
    if (read_kfd(pid, KfdFile::kOccupancy, b, sizeof b, &n)) r.cu_occupancy = static_cast<double>(strtoull(b, nullptr, 10));
    out->push_back(r);
  }
  closedir(d);
  return true;
}

}  // namespace gpumon

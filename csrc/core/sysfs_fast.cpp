#include "sysfs_fast.h"

#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>

#include <cstdlib>

#include "common.h"

namespace gpumon {

namespace {

int open_ro(const std::string& p) { return ::open(p.c_str(), O_RDONLY | O_CLOEXEC); }

// pread at offset 0 re-runs the attribute's show() (kernfs restarts the seq_file at pos 0).
ssize_t pread_all(int fd, void* buf, size_t cap) {
  size_t got = 0;
  while (got < cap) {
    ssize_t r = ::pread(fd, static_cast<char*>(buf) + got, cap - got, static_cast<off_t>(got));
    if (r < 0) return -1;
    if (r == 0) break;
    got += static_cast<size_t>(r);
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

void SysfsGpu::fdinfo_usage(uint32_t pid, ProcSample* p) {
  if (render_path_.empty()) return;
  const std::string base = proc_root_ + "/" + std::to_string(pid);
  const int64_t now = mono_ns();
  FdCache& c = fd_cache_[pid];
  // The set of DRM fds of a process is stable; rescan the fd table every 10 s only.
  if (c.scanned_ns == 0 || now - c.scanned_ns > 10'000'000'000ll) {
    c.fds.clear();
    c.scanned_ns = now;
    DIR* d = opendir((base + "/fd").c_str());
    if (d) {
      char target[256];
      while (dirent* e = readdir(d)) {
        if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
        ssize_t n = readlink((base + "/fd/" + e->d_name).c_str(), target, sizeof target - 1);
        if (n <= 0) continue;
        target[n] = 0;
        if (render_path_ == target) c.fds.push_back(atoi(e->d_name));
      }
      closedir(d);
    }
  }
  if (c.fds.empty()) return;
  uint64_t gfx = 0, vram = 0, gtt = 0, cpu = 0;
  bool any = false, have_vram = false;
  std::vector<uint64_t> clients;
  char text[4096];
  for (int fd : c.fds) {
    size_t n = 0;
    if (!read_small(base + "/fdinfo/" + std::to_string(fd), text, sizeof text, &n)) {
      c.scanned_ns = 0;  // fd closed: rescan next tick
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
  const std::string tail = "/stats_" + std::to_string(kfd_gpu_id_) + "/cu_occupancy";
  const std::string kdir = sys_root_ + "/class/kfd/kfd/proc/";
  char b[64];
  for (size_t k = 0; k < pids.size(); ++k) {
    size_t n = 0;
    if (read_small(kdir + std::to_string(pids[k]) + tail, b, sizeof b, &n))
      (*out)[k] = static_cast<double>(strtoull(b, nullptr, 10));
  }
}

bool SysfsGpu::processes(std::vector<ProcSample>* out) {
  out->clear();
  if (!kfd_gpu_id_) return false;
  const std::string kdir = sys_root_ + "/class/kfd/kfd/proc";
  DIR* d = opendir(kdir.c_str());
  if (!d) return false;
  const std::string vram_name = "/vram_" + std::to_string(kfd_gpu_id_);
  const std::string occ_name = "/stats_" + std::to_string(kfd_gpu_id_) + "/cu_occupancy";
  std::vector<uint32_t> seen;
  char b[64];
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    const uint32_t pid = static_cast<uint32_t>(strtoul(e->d_name, nullptr, 10));
    const std::string pdir = kdir + "/" + e->d_name;
    size_t n = 0;
    if (!read_small(pdir + vram_name, b, sizeof b, &n)) continue;  // process not on this GPU
    ProcSample p;
    p.pid = pid;
    p.mem_bytes = static_cast<double>(strtoull(b, nullptr, 10));
    p.vram_bytes = p.mem_bytes;
    if (read_small(pdir + occ_name, b, sizeof b, &n)) p.cu_occupancy = static_cast<double>(strtoull(b, nullptr, 10));
    fdinfo_usage(pid, &p);
    seen.push_back(pid);
    out->push_back(std::move(p));
  }
  closedir(d);
  // forget fd tables of processes that left this GPU
  for (auto it = fd_cache_.begin(); it != fd_cache_.end();) {
    bool alive = false;
    for (uint32_t s : seen) alive |= (s == it->first);
    it = alive ? std::next(it) : fd_cache_.erase(it);
  }
  return true;
}

}  // namespace gpumon

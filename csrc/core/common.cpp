#include <algorithm>
#include "common.h"

#include <pthread.h>
#include <signal.h>
#include <sys/utsname.h>

#include <fcntl.h>
#include <unistd.h>

#include <cstring>
#include <ctime>
#include <mutex>

namespace gpumon {

void set_thread_name(const std::string& name) { pthread_setname_np(pthread_self(), name.substr(0, 15).c_str()); }

void block_sigpipe() {
  sigset_t s;
  sigemptyset(&s);
  sigaddset(&s, SIGPIPE);
  pthread_sigmask(SIG_BLOCK, &s, nullptr);
}

std::atomic<int> g_log_level{static_cast<int>(LogLevel::kInfo)};

static std::mutex g_log_mu;

void log_line(LogLevel lvl, const char* component, const std::string& msg) {
  static const char* names[] = {"debug", "info", "warn", "error", "off"};
  int64_t ns = wall_ns();
  time_t sec = static_cast<time_t>(ns / 1000000000);
  struct tm tmv;
  gmtime_r(&sec, &tmv);
  char ts[64];
  snprintf(ts, sizeof ts, "%04d-%02d-%02dT%02d:%02d:%02d.%03dZ", tmv.tm_year + 1900, tmv.tm_mon + 1,
           tmv.tm_mday, tmv.tm_hour, tmv.tm_min, tmv.tm_sec, static_cast<int>((ns / 1000000) % 1000));
  std::lock_guard<std::mutex> g(g_log_mu);
  fprintf(stderr, "ts=%s level=%s component=%s msg=\"%s\"\n", ts, names[static_cast<int>(lvl)],
          component, msg.c_str());
}

std::vector<std::string> split(std::string_view s, char sep) {
  std::vector<std::string> out;
  size_t start = 0;
  while (true) {
    size_t p = s.find(sep, start);
    if (p == std::string_view::npos) {
      out.emplace_back(s.substr(start));
      break;
    }
    out.emplace_back(s.substr(start, p - start));
    start = p + 1;
  }
  return out;
}

std::string_view trim(std::string_view s) {
  size_t b = 0, e = s.size();
  while (b < e && (s[b] == ' ' || s[b] == '\t' || s[b] == '\n' || s[b] == '\r')) ++b;
  while (e > b && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\n' || s[e - 1] == '\r')) --e;
  return s.substr(b, e - b);
}

bool starts_with(std::string_view s, std::string_view p) {
  return s.size() >= p.size() && s.compare(0, p.size(), p) == 0;
}

bool ends_with(std::string_view s, std::string_view p) {
  return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0;
}

std::string normalize_bdf(std::string_view s) {
  s = trim(s);
  unsigned dom = 0, bus = 0, dev = 0, fn = 0;
  int used = 0;
  std::string z(s);
  if (std::count(z.begin(), z.end(), ':') == 2) {
    if (sscanf(z.c_str(), "%x:%x:%x.%x%n", &dom, &bus, &dev, &fn, &used) != 4) return "";
  } else if (std::count(z.begin(), z.end(), ':') == 1) {
    if (sscanf(z.c_str(), "%x:%x.%x%n", &bus, &dev, &fn, &used) != 3) return "";
  } else {
    return "";
  }
  if (used != static_cast<int>(z.size()) || dom > 0xffff || bus > 0xff || dev > 0x1f || fn > 7) return "";
  char b[32];
  snprintf(b, sizeof b, "%04x:%02x:%02x.%x", dom, bus, dev, fn);
  return b;
}

bool read_file(const std::string& path, std::string* out, size_t max_bytes) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  out->clear();
  char buf[8192];
  while (out->size() < max_bytes) {
    ssize_t n = ::read(fd, buf, sizeof buf);
    if (n < 0) {
      if (errno == EINTR) continue;
      ::close(fd);
      return false;
    }
    if (n == 0) break;
    out->append(buf, static_cast<size_t>(n));
  }
  ::close(fd);
  return true;
}

std::string driver_version_label(const std::string& raw_in, const std::string& module_version, std::string* source) {
  const std::string mv(trim(module_version));
  if (!mv.empty() && mv.size() <= 64 && mv.find_first_of(" \t\n") == std::string::npos) {
    *source = "module";
    return mv;
  }
  const std::string raw(trim(raw_in));
  std::string rest;
  bool proc_version = raw.empty();
  for (const char* p : {"Linux version ", "Linuxversion"})
    if (starts_with(raw, p)) {
      rest = raw.substr(strlen(p));
      proc_version = true;
      break;
    }
  if (proc_version) {
    std::string rel;
    for (char c : rest) {
      if (c == ' ' || c == '(' || c == '\t') break;
      rel.push_back(c);
    }
    if (rel.empty()) {
      struct utsname u {};
      if (uname(&u) == 0) rel = u.release;
    }
    *source = "kernel";
    return rel;
  }
  *source = "library";
  if (raw.size() <= 64) return raw;
  const size_t cut = raw.find_last_of(" ,;", 64);
  return std::string(trim(raw.substr(0, cut == std::string::npos || cut == 0 ? 64 : cut)));
}

}  // namespace gpumon

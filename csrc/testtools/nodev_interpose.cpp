// Device-node denial for bin/gpumon-exporter-nodev (tools/no_device_check.sh): linked INTO the
// exporter executable with -rdynamic, these definitions of open / open64 / openat / openat64
// interpose on every shared library's calls (libamd_smi, libdrm, hsakmt), and refuse /dev/kfd and
// /dev/dri/* with EPERM -- what a container without device access (an unprivileged DaemonSet pod:
// the device cgroup denies the hostPath device nodes) sees. Everything else is forwarded. Used to
// find out which series the default exporter keeps without device nodes.
#include <dlfcn.h>
#include <fcntl.h>
#include <stdarg.h>
#include <string.h>

#include <atomic>
#include <cerrno>
#include <cstdio>

namespace {
std::atomic<int> g_denied{0};

bool device_node(const char* p) {
  return p && (!strcmp(p, "/dev/kfd") || !strncmp(p, "/dev/dri/", 9));
}

template <typename F>
F next(const char* name) {
  return reinterpret_cast<F>(dlsym(RTLD_NEXT, name));
}

int deny(const char* path) {
  if (g_denied.fetch_add(1) < 8) fprintf(stderr, "nodev: denied open(%s)\n", path);
  errno = EPERM;
  return -1;
}
}  // namespace

extern "C" {

int open(const char* path, int flags, ...) {
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) {
    va_list ap;
    va_start(ap, flags);
    mode = static_cast<mode_t>(va_arg(ap, int));
    va_end(ap);
  }
  if (device_node(path)) return deny(path);
  static auto real = next<int (*)(const char*, int, ...)>("open");
  return real(path, flags, mode);
}

int open64(const char* path, int flags, ...) {
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) {
    va_list ap;
    va_start(ap, flags);
    mode = static_cast<mode_t>(va_arg(ap, int));
    va_end(ap);
  }
  if (device_node(path)) return deny(path);
  static auto real = next<int (*)(const char*, int, ...)>("open64");
  return real(path, flags, mode);
}

int openat(int dirfd, const char* path, int flags, ...) {
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) {
    va_list ap;
    va_start(ap, flags);
    mode = static_cast<mode_t>(va_arg(ap, int));
    va_end(ap);
  }
  if (device_node(path)) return deny(path);
  static auto real = next<int (*)(int, const char*, int, ...)>("openat");
  return real(dirfd, path, flags, mode);
}

int openat64(int dirfd, const char* path, int flags, ...) {
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) {
    va_list ap;
    va_start(ap, flags);
    mode = static_cast<mode_t>(va_arg(ap, int));
    va_end(ap);
  }
  if (device_node(path)) return deny(path);
  static auto real = next<int (*)(int, const char*, int, ...)>("openat64");
  return real(dirfd, path, flags, mode);
}

}  // extern "C"

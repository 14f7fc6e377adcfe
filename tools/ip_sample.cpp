// Where is a thread spending its CPU? Samples the user-space instruction pointer of one thread
// with a perf_event CPU-clock sampler (no ptrace, no debugger attach) and prints the hottest
// addresses as (mapping, offset) so llvm-symbolizer can name them.
//
//   g++ -O2 -o build/ip_sample tools/ip_sample.cpp
//   build/ip_sample <pid> <tid> [seconds]
#include <linux/perf_event.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

struct Map {
  uint64_t lo, hi, off;
  std::string path;
};

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: ip_sample <pid> <tid> [seconds]\n");
    return 2;
  }
  const int pid = atoi(argv[1]), tid = atoi(argv[2]);
  const double secs = argc > 3 ? atof(argv[3]) : 1.0;
  perf_event_attr a{};
  a.size = sizeof a;
  a.type = PERF_TYPE_SOFTWARE;
  a.config = PERF_COUNT_SW_CPU_CLOCK;
  a.sample_period = 50000;  // ns of CPU time between samples
  a.sample_type = PERF_SAMPLE_IP;
  a.exclude_kernel = 1;
  a.exclude_hv = 1;
  a.disabled = 1;
  const int fd = static_cast<int>(syscall(SYS_perf_event_open, &a, tid, -1, -1, 0));
  if (fd < 0) {
    fprintf(stderr, "perf_event_open: %s\n", strerror(errno));
    return 1;
  }
  const size_t page = sysconf(_SC_PAGESIZE), npages = 64;
  void* base = mmap(nullptr, page * (npages + 1), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (base == MAP_FAILED) {
    fprintf(stderr, "mmap: %s\n", strerror(errno));
    return 1;
  }
  auto* meta = static_cast<perf_event_mmap_page*>(base);
  char* data = static_cast<char*>(base) + page;
  const uint64_t size = page * npages;
  std::map<uint64_t, uint64_t> hits;
  uint64_t tail = 0, total = 0;
  ioctl(fd, PERF_EVENT_IOC_ENABLE, 0);
  const int steps = static_cast<int>(secs * 100);
  for (int s = 0; s < steps; ++s) {
    usleep(10000);
    const uint64_t head = __atomic_load_n(&meta->data_head, __ATOMIC_ACQUIRE);
    while (tail < head) {
      perf_event_header h;
      for (size_t i = 0; i < sizeof h; ++i) reinterpret_cast<char*>(&h)[i] = data[(tail + i) % size];
      if (h.type == PERF_RECORD_SAMPLE) {
        uint64_t ip = 0;
        for (size_t i = 0; i < 8; ++i) reinterpret_cast<char*>(&ip)[i] = data[(tail + sizeof h + i) % size];
        hits[ip]++;
        total++;
      }
      tail += h.size ? h.size : sizeof h;
    }
    __atomic_store_n(&meta->data_tail, tail, __ATOMIC_RELEASE);
  }
  ioctl(fd, PERF_EVENT_IOC_DISABLE, 0);
  std::vector<Map> maps;
  std::ifstream mf("/proc/" + std::to_string(pid) + "/maps");
  for (std::string line; std::getline(mf, line);) {
    std::istringstream is(line);
    std::string range, perms, off, dev, inode, path;
    is >> range >> perms >> off >> dev >> inode >> path;
    Map m;
    m.lo = std::stoull(range.substr(0, range.find('-')), nullptr, 16);
    m.hi = std::stoull(range.substr(range.find('-') + 1), nullptr, 16);
    m.off = std::stoull(off, nullptr, 16);
    m.path = path.empty() ? "[anon]" : path;
    maps.push_back(m);
  }
  std::vector<std::pair<uint64_t, uint64_t>> v(hits.begin(), hits.end());
  std::sort(v.begin(), v.end(), [](auto& x, auto& y) { return x.second > y.second; });
  printf("{\"samples\": %lu, \"top\": [", static_cast<unsigned long>(total));
  for (size_t i = 0; i < v.size() && i < 12; ++i) {
    std::string where = "?";
    uint64_t fo = 0;
    for (const auto& m : maps)
      if (v[i].first >= m.lo && v[i].first < m.hi) {
        where = m.path;
        fo = v[i].first - m.lo + m.off;
        break;
      }
    printf("%s{\"ip\": \"0x%lx\", \"n\": %lu, \"map\": \"%s\", \"file_off\": \"0x%lx\"}", i ? ", " : "",
           static_cast<unsigned long>(v[i].first), static_cast<unsigned long>(v[i].second), where.c_str(),
           static_cast<unsigned long>(fo));
  }
  printf("]}\n");
  return 0;
}

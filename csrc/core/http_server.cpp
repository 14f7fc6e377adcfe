#include "http_server.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sched.h>
#include <sys/epoll.h>
#include <sys/ioctl.h>
#include <sys/eventfd.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <strings.h>
#include <ctime>
#include <list>
#include <unordered_map>

#include "common.h"
#include "tls.h"

namespace gpumon {

namespace {

constexpr size_t kMaxHeader = 16 * 1024;
constexpr long kMaxBody = 64 * 1024;  // every route is GET/HEAD: a request body is only ever skipped
// input buffered per connection before it is parsed: above the largest acceptable request, so a
// full buffer always starts with a complete (or a refused) request
constexpr size_t kMaxInput = kMaxHeader + kMaxBody + 4096;
constexpr int64_t kIdleTimeoutNs = 60LL * 1000000000LL;
// A request whose header has not completed this long after its first byte is dropped (a client
// trickling a header must not hold a connection slot for the whole idle timeout).
constexpr int64_t kHeaderTimeoutNs = 10LL * 1000000000LL;  // GPUMON_HTTP_HEADER_TIMEOUT_S overrides
// After the last response of a "Connection: close" exchange the server half-closes and drains what
// the client still sends for at most this long before closing: closing a socket with unread input
// sends a RST, which can make the client drop the response it has not read yet (an error answer to
// a request whose body was still arriving).
constexpr int64_t kLingerNs = 2LL * 1000000000LL;
constexpr size_t kMaxConnsPerLoop = 4096;
// File descriptors left to the rest of the exporter (sysfs / procfs reads, sockets of the metadata
// pollers, the on-device helper) when the connection cap is derived from RLIMIT_NOFILE: a flood
// of scrape connections must not make the sampler's own opens fail with EMFILE.
constexpr rlim_t kFdReserve = 256;
// Connections a loop may admit over the cap while another loop closes one of its own (evict_debt_):
// a few fds out of kFdReserve.
constexpr size_t kDebtSlack = 16;
constexpr int kSndBuf = 1 << 20;  // GPUMON_HTTP_SNDBUF overrides (bytes; 0 = the kernel's autotuning)
// The connection cap also answers to the memory limit: every admitted connection may
// buffer kMaxInput of request before the header timeout closes it, plus a TLS session, so a flood
// must not push the process past its cgroup's memory.max (the DaemonSet's 256Mi, the systemd
// unit's MemoryMax) into an OOM-kill restart loop. kMemBaseline is left to the rest of the exporter
// (its steady RSS is ~10 MB; libamd_smi and the snapshots of 8 GPUs stay well under this).
constexpr uint64_t kMemBaseline = 96ull << 20;
constexpr uint64_t kTlsSessionBytes = 64ull << 10;

}  // namespace

// The smallest memory.max on the way from this process's cgroup (cgroup v2) up to the root, else
// the v1 memory controller's limit; 0 = unlimited / unknown. GPUMON_HTTP_MEMORY_BUDGET (bytes)
// overrides. `proc_cgroup` / `cgroup_root`: /proc/self/cgroup and /sys/fs/cgroup (tests: a tree).
uint64_t memory_limit_bytes(const std::string& proc_cgroup, const std::string& cgroup_root) {
  if (const char* e = getenv("GPUMON_HTTP_MEMORY_BUDGET")) return strtoull(e, nullptr, 10);
  auto num = [](const std::string& path) -> uint64_t {
    std::string t;
    if (!read_file(path, &t, 64)) return 0;
    const std::string v(trim(t));
    if (v.empty() || v == "max") return 0;
    const uint64_t x = strtoull(v.c_str(), nullptr, 10);
    return x >= (1ull << 60) ? 0 : x;  // v1 reports "unlimited" as a huge page-rounded number
  };
  std::string cg;
  uint64_t best = 0;
  if (read_file(proc_cgroup, &cg, 4096))
    for (const auto& line : split(cg, '\n')) {
      if (starts_with(line, "0::")) {  // v2: walk from this cgroup to the mount's root
        std::string path(trim(line.substr(3)));
        while (true) {
          const uint64_t v = num(cgroup_root + (path == "/" ? std::string() : path) + "/memory.max");
          if (v && (!best || v < best)) best = v;
          if (path.empty() || path == "/") break;
          const size_t slash = path.rfind('/');
          path = slash == 0 || slash == std::string::npos ? "/" : path.substr(0, slash);
        }
      }
    }
  if (!best) best = num(cgroup_root + "/memory/memory.limit_in_bytes");
  return best;
}

namespace {

const char* status_text(int s) {
  switch (s) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 413: return "Payload Too Large";
    case 431: return "Request Header Fields Too Large";
    case 503: return "Service Unavailable";
    default: return "Error";
  }
}

struct Conn {
  int fd = -1;
  std::string in;
  std::string head;                       // pending response header
  std::shared_ptr<const void> owner;      // pending body owner
  std::string inline_body;
  const char* body = nullptr;
  size_t body_len = 0;
  size_t head_off = 0, body_off = 0;
  bool writing = false;
  bool close_after = false;
  bool closing = false;  // response sent, write side shut: draining input until EOF / kLingerNs
  int64_t closing_ns = 0;
  int64_t req_start_ns = 0;  // first byte of the request still being read (0: none pending)
  int64_t last_ns = 0;
  std::list<int>::iterator lru;  // position in Loop::lru (least recently active first)
  int64_t req_ns = 0;
  std::string path;
  uint32_t served = 0;  // requests answered on this connection (a scraper's keep-alive has > 0)
  void* ssl = nullptr;  // TLS session (HttpServer::set_tls), else plain
  bool hs = false;      // TLS handshake still in progress
  bool client_cert = false;  // mutual TLS: the client's certificate verified (set after the handshake)
  // the last read stopped at the input cap: the session may hold decrypted bytes that no socket
  // event will announce (they left the socket already), so the loop reads again once there is room
  bool tls_more = false;
};

bool set_nonblock(int fd) {
  int fl = fcntl(fd, F_GETFL, 0);
  return fl >= 0 && fcntl(fd, F_SETFL, fl | O_NONBLOCK) == 0;
}

// Parses one request from c->in. Returns bytes consumed (0 = incomplete, -1 = bad, -2 = header
// too big, -3 = body too big: buffering an announced body of any size would let one client grow
// the connection's input without bound).
long parse_request(const std::string& in, HttpRequest* r) {
  size_t end = in.find("\r\n\r\n");
  if (end == std::string::npos) return in.size() > kMaxHeader ? -2 : 0;
  if (end > kMaxHeader) return -2;
  size_t le = in.find("\r\n");
  std::string_view line(in.data(), le);
  size_t s1 = line.find(' ');
  if (s1 == std::string_view::npos) return -1;
  size_t s2 = line.find(' ', s1 + 1);
  if (s2 == std::string_view::npos) return -1;
  r->method = std::string(line.substr(0, s1));
  std::string_view target = line.substr(s1 + 1, s2 - s1 - 1);
  std::string_view ver = line.substr(s2 + 1);
  size_t q = target.find('?');
  r->path = std::string(target.substr(0, q));
  r->query = q == std::string_view::npos ? "" : std::string(target.substr(q + 1));
  r->keep_alive = ver == "HTTP/1.1";
  r->accept_gzip = false;
  r->authorization.clear();
  size_t pos = le + 2;
  long content_len = 0;
  while (pos < end) {
    size_t e = in.find("\r\n", pos);
    if (e == std::string::npos || e > end) e = end;
    std::string_view h(in.data() + pos, e - pos);
    size_t colon = h.find(':');
    if (colon != std::string_view::npos) {
      std::string_view name = h.substr(0, colon);
      std::string_view val = trim(h.substr(colon + 1));
      auto ieq = [](std::string_view a, const char* b) {
        return a.size() == strlen(b) && strncasecmp(a.data(), b, a.size()) == 0;
      };
      if (ieq(name, "connection")) {
        if (val.size() >= 5 && strncasecmp(val.data(), "close", 5) == 0) r->keep_alive = false;
        if (val.size() >= 10 && strncasecmp(val.data(), "keep-alive", 10) == 0) r->keep_alive = true;
      } else if (ieq(name, "accept-encoding")) {
        std::string v(val);
        for (auto& ch : v) ch = static_cast<char>(tolower(ch));
        r->accept_gzip = v.find("gzip") != std::string::npos;
      } else if (ieq(name, "authorization")) {
        r->authorization.assign(val);
      } else if (ieq(name, "content-length")) {
        const std::string v(val);
        char* endp = nullptr;
        content_len = strtol(v.c_str(), &endp, 10);
        if (v.empty() || *endp != '\0' || content_len < 0) return -1;
        if (content_len > kMaxBody) return -3;
      }
    }
    pos = e + 2;
  }
  long consumed = static_cast<long>(end + 4);
  if (content_len > 0) {
    if (in.size() < static_cast<size_t>(consumed + content_len)) return 0;
    consumed += content_len;
  }
  return consumed;
}

}  // namespace

struct HttpServer::Loop {
  int ep = -1;
  int lfd = -1;  // the server's shared listening socket (not owned)
  int wake = -1;
  std::thread th;
  std::unordered_map<int, Conn> conns;
  std::list<int> lru;  // connection fds, least recently active first: O(1) eviction at the cap
};

bool parse_listen(const std::string& listen, std::string* host, int* port, std::string* err) {
  std::string h, p;
  const std::string l(trim(listen));
  if (l.empty()) {
    *err = "empty listen address";
    return false;
  }
  if (l[0] == '[') {
    const size_t rb = l.find(']');
    if (rb == std::string::npos || rb + 1 >= l.size() || l[rb + 1] != ':') {
      *err = "listen '" + l + "': expected [v6]:port";
      return false;
    }
    h = l.substr(1, rb - 1);
    p = l.substr(rb + 2);
    in6_addr a6{};
    if (h.empty() || inet_pton(AF_INET6, h.c_str(), &a6) != 1) {
      *err = "listen '" + l + "': '" + h + "' is not an IPv6 address";
      return false;
    }
  } else if (l.find_first_not_of("0123456789") == std::string::npos) {
    p = l;  // "9400": every address
  } else {
    const size_t colon = l.rfind(':');
    if (colon == std::string::npos) {
      *err = "listen '" + l + "': expected host:port";
      return false;
    }
    h = l.substr(0, colon);
    p = l.substr(colon + 1);
    if (h.find(':') != std::string::npos) {
      *err = "listen '" + l + "': an IPv6 address needs brackets ([v6]:port)";
      return false;
    }
    if (h == "*") h.clear();
  }
  if (p.empty() || p.size() > 5 || p.find_first_not_of("0123456789") != std::string::npos || atoi(p.c_str()) > 65535) {
    *err = "listen '" + l + "': bad port '" + p + "'";
    return false;
  }
  *host = h;
  *port = atoi(p.c_str());
  return true;
}

namespace {

// Binds the listening socket for `host` ("" = every address: dual-stack [::], else 0.0.0.0).
// Returns the fd (listening, non-blocking) or -1 with *err; *port is updated for port 0.
int open_listener(const std::string& host, int* port, std::string* bound, std::string* err) {
  struct Try {
    int family;
    std::string addr;
    bool v6only;
  };
  std::vector<Try> tries;
  in_addr a4{};
  in6_addr a6{};
  if (host.empty()) {
    tries = {{AF_INET6, "::", false}, {AF_INET, "0.0.0.0", false}};
  } else if (host == "::") {
    tries = {{AF_INET6, "::", false}};
  } else if (inet_pton(AF_INET6, host.c_str(), &a6) == 1) {
    tries = {{AF_INET6, host, true}};
  } else if (inet_pton(AF_INET, host.c_str(), &a4) == 1) {
    tries = {{AF_INET, host, false}};
  } else {  // a host name: its first passive address
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = AI_PASSIVE;
    const int rc = getaddrinfo(host.c_str(), nullptr, &hints, &res);
    if (rc != 0 || !res) {
      *err = "bad listen address " + host + ": " + gai_strerror(rc);
      return -1;
    }
    char buf[INET6_ADDRSTRLEN] = {};
    if (res->ai_family == AF_INET6)
      inet_ntop(AF_INET6, &reinterpret_cast<sockaddr_in6*>(res->ai_addr)->sin6_addr, buf, sizeof buf);
    else
      inet_ntop(AF_INET, &reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr, buf, sizeof buf);
    tries = {{res->ai_family, buf, res->ai_family == AF_INET6}};
    freeaddrinfo(res);
  }
  std::string last;
  for (size_t k = 0; k < tries.size(); ++k) {
    const Try& t = tries[k];
    const bool fallback_left = k + 1 < tries.size();
    const int fd = socket(t.family, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) {
      last = std::string("socket: ") + strerror(errno);
      if (fallback_left && (errno == EAFNOSUPPORT || errno == EPROTONOSUPPORT)) continue;  // no IPv6 here
      break;
    }
    int one = 1, v6only = t.v6only ? 1 : 0;
    // SO_REUSEADDR: a restarted exporter rebinds over its predecessor's TIME_WAIT connections. It
    // never lets two listeners share the port on Linux; SO_REUSEPORT (not set) would.
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_storage ss{};
    socklen_t sl;
    if (t.family == AF_INET6) {
      setsockopt(fd, IPPROTO_IPV6, IPV6_V6ONLY, &v6only, sizeof v6only);
      auto* sa = reinterpret_cast<sockaddr_in6*>(&ss);
      sa->sin6_family = AF_INET6;
      sa->sin6_port = htons(static_cast<uint16_t>(*port));
      inet_pton(AF_INET6, t.addr.c_str(), &sa->sin6_addr);
      sl = sizeof(sockaddr_in6);
    } else {
      auto* sa = reinterpret_cast<sockaddr_in*>(&ss);
      sa->sin_family = AF_INET;
      sa->sin_port = htons(static_cast<uint16_t>(*port));
      inet_pton(AF_INET, t.addr.c_str(), &sa->sin_addr);
      sl = sizeof(sockaddr_in);
    }
    const std::string where = (t.family == AF_INET6 ? "[" + t.addr + "]" : t.addr) + ":" + std::to_string(*port);
    if (bind(fd, reinterpret_cast<sockaddr*>(&ss), sl) != 0) {
      const int e = errno;
      last = "bind " + where + ": " + strerror(e);
      close(fd);
      // IPv6 present but unusable (disable_ipv6): the IPv4 wildcard; an address in use is final
      if (fallback_left && (e == EADDRNOTAVAIL || e == EAFNOSUPPORT)) continue;
      break;
    }
    if (listen(fd, 1024) != 0) {
      last = std::string("listen: ") + strerror(errno);
      close(fd);
      break;
    }
    if (*port == 0) {
      getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &sl);
      *port = ntohs(t.family == AF_INET6 ? reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port
                                         : reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
    }
    set_nonblock(fd);
    *bound = (t.family == AF_INET6 ? "[" + t.addr + "]" : t.addr) + ":" + std::to_string(*port) +
             (t.family == AF_INET6 && !t.v6only ? " (dual-stack)" : "");
    return fd;
  }
  *err = last;
  return -1;
}

}  // namespace

HttpServer::HttpServer(std::string addr, int port, int threads, Handler h, Observer obs)
    : addr_(std::move(addr)),
      port_(port),
      nthreads_(std::max(1, threads)),
      handler_(std::move(h)),
      observer_(std::move(obs)) {}

HttpServer::~HttpServer() { stop(); }

bool HttpServer::start(std::string* err) {
  if (running_) return true;
  auto abandon = [this]() {  // a failed start: close what was opened, start no thread
    for (auto& P : loops_) {
      close(P->ep);
      close(P->wake);
    }
    loops_.clear();
    if (lfd_ >= 0) close(lfd_);
    lfd_ = -1;
  };
  sndbuf_ = kSndBuf;
  if (const char* e = getenv("GPUMON_HTTP_SNDBUF")) sndbuf_ = std::max(0, atoi(e));
  header_timeout_ns_ = kHeaderTimeoutNs;
  if (const char* e = getenv("GPUMON_HTTP_HEADER_TIMEOUT_S"))
    header_timeout_ns_ = static_cast<int64_t>(std::max(0.1, atof(e)) * 1e9);
  max_conns_ = kMaxConnsPerLoop;
  rlimit rl{};
  if (getrlimit(RLIMIT_NOFILE, &rl) == 0 && rl.rlim_cur != RLIM_INFINITY) {
    const rlim_t usable = rl.rlim_cur > 2 * kFdReserve ? rl.rlim_cur - kFdReserve : rl.rlim_cur / 2;
    max_conns_ = std::clamp<size_t>(usable / static_cast<rlim_t>(std::max(1, nthreads_)), 8, kMaxConnsPerLoop);
  }
  if (const uint64_t mem = memory_limit_bytes("/proc/self/cgroup", "/sys/fs/cgroup"); mem > 0) {
    const uint64_t budget = mem > 2 * kMemBaseline ? mem - kMemBaseline : mem / 2;
    const uint64_t per_conn = kMaxInput + 4096 + (tls_ ? kTlsSessionBytes : 0);
    const size_t cap = std::max<size_t>(8, budget / per_conn / static_cast<uint64_t>(std::max(1, nthreads_)));
    if (cap < max_conns_) {
      GPUMON_LOG(LogLevel::kInfo, "http",
                 "connection cap " + std::to_string(cap * std::max(1, nthreads_)) + " (memory limit " +
                     std::to_string(mem >> 20) + " MiB)");
      max_conns_ = cap;
    }
  }
  lfd_ = open_listener(addr_, &port_, &bound_, err);
  if (lfd_ < 0) return false;
  exclusive_ = true;
  for (int t = 0; t < nthreads_; ++t) {
    auto L = std::make_unique<Loop>();
    L->lfd = lfd_;
    L->ep = epoll_create1(EPOLL_CLOEXEC);
    L->wake = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (L->ep < 0 || L->wake < 0) {
      *err = std::string("epoll / eventfd: ") + strerror(errno);
      if (L->ep >= 0) close(L->ep);
      if (L->wake >= 0) close(L->wake);
      abandon();
      return false;
    }
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = L->wake;
    epoll_ctl(L->ep, EPOLL_CTL_ADD, L->wake, &ev);
    loops_.push_back(std::move(L));
    watch_listener(loops_.back().get(), true);
  }
  running_ = true;
  for (auto& L : loops_) {
    Loop* p = L.get();
    p->th = std::thread([this, p] {
      set_thread_name("gpumon-http");
      block_sigpipe();  // TLS sessions write with write() (common.h)
      run(p);
    });
  }
  return true;
}

bool HttpServer::watch_listener(Loop* L, bool on) {
  if (!on) return epoll_ctl(L->ep, EPOLL_CTL_DEL, L->lfd, nullptr) == 0;
  epoll_event ev{};
  ev.data.fd = L->lfd;
  // EPOLLEXCLUSIVE: a connection wakes one loop, not every loop waiting on the shared socket.
  // EPOLL_CTL_MOD is not allowed with it, so pausing accepts (EMFILE) deletes and re-adds.
  ev.events = EPOLLIN | (exclusive_ ? static_cast<uint32_t>(EPOLLEXCLUSIVE) : 0u);
  if (epoll_ctl(L->ep, EPOLL_CTL_ADD, L->lfd, &ev) == 0) return true;
  if (errno == EINVAL && exclusive_) {  // kernel < 4.5: every loop wakes, the losers see EAGAIN
    exclusive_ = false;
    ev.events = EPOLLIN;
    return epoll_ctl(L->ep, EPOLL_CTL_ADD, L->lfd, &ev) == 0;
  }
  return errno == EEXIST;
}

void HttpServer::stop() {
  if (!running_.exchange(false)) return;
  for (auto& L : loops_) {
    uint64_t one = 1;
    ssize_t w = write(L->wake, &one, sizeof one);
    (void)w;
  }
  for (auto& L : loops_) {
    if (L->th.joinable()) L->th.join();
    for (auto& [fd, c] : L->conns) {
      if (c.ssl) tls_->free_session(c.ssl);
      close(fd);
    }
    L->conns.clear();
    L->lru.clear();
    close(L->ep);
    close(L->wake);
  }
  loops_.clear();
  if (lfd_ >= 0) close(lfd_);
  lfd_ = -1;
}

namespace {
int64_t thread_cpu_ns() {
  timespec ts{};
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}
// 0 or the error number (pthread_setschedparam returns it; errno is not set)
int set_fifo(int prio) {
  sched_param sp{};
  sp.sched_priority = prio;
  return pthread_setschedparam(pthread_self(), prio > 0 ? SCHED_FIFO : SCHED_OTHER, &sp);
}
}  // namespace

void HttpServer::run(Loop* L) {
  epoll_event evs[256];
  int64_t last_sweep = mono_ns();
  // http_rt_priority: FIFO while this loop's CPU time in the current 100 ms window stays under
  // rt_budget_ x 100 ms; demoted to SCHED_OTHER for the rest of the window otherwise.
  constexpr int64_t kRtWindowNs = 100'000'000;
  const int prio = std::clamp(rt_prio_, 0, 99);
  const int rc = prio > 0 ? set_fifo(prio) : 0;
  bool fifo = prio > 0 && rc == 0;
  if (prio > 0 && !fifo)
    GPUMON_LOG(LogLevel::kWarn, "http",
               "http_rt_priority " + std::to_string(prio) + ": " + strerror(rc) +
                   " (needs CAP_SYS_NICE); HTTP loops keep normal scheduling");
  const bool rt_on = fifo;
  if (fifo) rt_loops_.fetch_add(1);
  int64_t win_start = mono_ns(), win_cpu0 = thread_cpu_ns();
  const int64_t budget_ns = static_cast<int64_t>(std::clamp(rt_budget_, 0.01, 1.0) * kRtWindowNs);
  auto close_conn = [&](int fd) {
    epoll_ctl(L->ep, EPOLL_CTL_DEL, fd, nullptr);
    auto it = L->conns.find(fd);
    if (it != L->conns.end()) {
      if (it->second.ssl) tls_->free_session(it->second.ssl);
      L->lru.erase(it->second.lru);
      L->conns.erase(it);
    }
    close(fd);
    conns_.fetch_sub(1);
  };
  // one read of request bytes: plain read(), or decrypted bytes of a TLS session (errno EAGAIN when
  // nothing is ready, EIO on a TLS error)
  auto rd = [&](Conn& c, char* b, size_t n) -> ssize_t {
    if (!c.ssl) return read(c.fd, b, n);
    const long r = tls_->read(c.ssl, b, n);
    if (r >= 0) return r;
    errno = r == -1 ? EAGAIN : EIO;
    return -1;
  };
  auto set_events = [&](int fd, uint32_t e) {
    epoll_event ev{};
    ev.events = e;
    ev.data.fd = fd;
    epoll_ctl(L->ep, EPOLL_CTL_MOD, fd, &ev);
  };
  // Writes pending output; returns false if the connection must be closed.
  auto flush = [&](Conn& c) -> bool {
    // TLS: the body was folded into `head` (serve): records come from one buffer, resumed at
    // head_off after a full socket (partial-write mode)
    while (c.ssl && c.head_off < c.head.size()) {
      const long w = tls_->write(c.ssl, c.head.data() + c.head_off, c.head.size() - c.head_off);
      if (w == -1) return true;
      if (w < 0) return false;
      c.head_off += static_cast<size_t>(w);
    }
    while (!c.ssl && (c.head_off < c.head.size() || c.body_off < c.body_len)) {
      iovec iov[2];
      int n = 0;
      if (c.head_off < c.head.size()) {
        iov[n].iov_base = const_cast<char*>(c.head.data() + c.head_off);
        iov[n].iov_len = c.head.size() - c.head_off;
        ++n;
      }
      if (c.body_off < c.body_len) {
        iov[n].iov_base = const_cast<char*>(c.body + c.body_off);
        iov[n].iov_len = c.body_len - c.body_off;
        ++n;
      }
      // sendmsg, not writev: MSG_NOSIGNAL keeps a peer that hung up from raising SIGPIPE in a host
      // process (the Python module, an embedding service) that did not ignore it
      msghdr mh{};
      mh.msg_iov = iov;
      mh.msg_iovlen = static_cast<size_t>(n);
      ssize_t w = sendmsg(c.fd, &mh, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) return true;
        return false;
      }
      size_t ww = static_cast<size_t>(w);
      size_t hrem = c.head.size() - c.head_off;
      if (ww <= hrem) {
        c.head_off += ww;
      } else {
        c.head_off = c.head.size();
        c.body_off += ww - hrem;
      }
    }
    // complete
    if (observer_ && c.req_ns) observer_(c.path, (mono_ns() - c.req_ns) * 1e-9);
    c.writing = false;
    c.owner.reset();
    c.inline_body.clear();
    c.body = nullptr;
    c.body_len = 0;
    c.head.clear();
    c.head_off = c.body_off = 0;
    c.req_ns = 0;
    if (c.close_after) {  // lingering close (kLingerNs)
      if (c.ssl) tls_->notify_close(c.ssl);
      shutdown(c.fd, SHUT_WR);
      c.closing = true;
      c.closing_ns = mono_ns();
      c.in.clear();
    }
    return true;
  };
  // Parses and answers as many complete requests as are buffered (pipelining).
  auto serve = [&](Conn& c) -> bool {
    while (!c.writing && !c.closing) {
      HttpRequest req;
      long used = parse_request(c.in, &req);
      req.client_cert = c.client_cert;
      if (used == 0) return true;
      HttpResponse resp;
      const int64_t t_req = mono_ns();  // service time = handler + response write
      if (used < 0) {
        resp.status = used == -2 ? 431 : used == -3 ? 413 : 400;
        resp.inline_body = status_text(resp.status);
        req.keep_alive = false;
        used = static_cast<long>(c.in.size());
      } else if (req.method != "GET" && req.method != "HEAD") {
        resp.status = 405;
        resp.inline_body = "method not allowed\n";
        req.keep_alive = false;
      } else {
        handler_(req, &resp);
      }
      requests_.fetch_add(1, std::memory_order_relaxed);
      if (resp.status < 400) c.served++;
      c.req_ns = t_req;
      c.path = req.path;
      c.in.erase(0, static_cast<size_t>(used));
      c.req_start_ns = c.in.empty() ? 0 : mono_ns();  // a pipelined request already started
      const char* body = resp.data;
      size_t blen = resp.len;
      if (!body) {
        c.inline_body = std::move(resp.inline_body);
        body = c.inline_body.data();
        blen = c.inline_body.size();
      } else {
        c.owner = resp.owner;
      }
      c.head.reserve(256);
      c.head = "HTTP/1.1 ";
      c.head += std::to_string(resp.status);
      c.head += ' ';
      c.head += status_text(resp.status);
      c.head += "\r\nContent-Type: ";
      c.head += resp.content_type;
      c.head += "\r\nContent-Length: ";
      c.head += std::to_string(blen);
      c.head += "\r\n";
      c.head += resp.extra_headers;
      c.head += req.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
      c.body = req.method == "HEAD" ? nullptr : body;
      c.body_len = req.method == "HEAD" ? 0 : blen;
      if (c.ssl && c.body_len) {  // one buffer for the records (a copy is small next to encrypting it)
        c.head.append(c.body, c.body_len);
        c.body = nullptr;
        c.body_len = 0;
        c.owner.reset();
        c.inline_body.clear();
      }
      c.close_after = !req.keep_alive;
      c.writing = true;
      if (!flush(c)) return false;
      if (c.writing) {
        set_events(c.fd, EPOLLOUT | EPOLLRDHUP);
        return true;
      }
    }
    return true;
  };
  // Reads what the connection has (up to the input cap) and answers it; false = close it.
  // `readable`: the event announced input. A TLS session is always read: a record may sit in the
  // socket since the handshake's last step, or decrypted bytes in the session (tls_more).
  auto read_serve = [&](Conn& c, bool readable) -> bool {
    while (true) {
      bool peer_closed = false, capped = false;
      if (readable || c.ssl) {
        char buf[8192];
        c.tls_more = false;
        while (true) {
          ssize_t r = rd(c, buf, sizeof buf);
          if (r > 0) {
            if (c.in.empty()) c.req_start_ns = mono_ns();
            c.in.append(buf, static_cast<size_t>(r));
            if (c.in.size() > kMaxInput) {
              capped = true;
              break;
            }
            continue;
          }
          if (r == 0) peer_closed = true;
          else if (errno == EINTR) continue;
          // a read error (a reset, a TLS protocol error): the connection is done. A failed TLS
          // session reads nothing more from the socket, so level-triggered EPOLLIN would otherwise
          // keep firing.
          else if (errno != EAGAIN && errno != EWOULDBLOCK) peer_closed = true;
          break;
        }
      }
      if (!serve(c)) return false;
      if (peer_closed && !c.writing) return false;
      // A plain socket that stopped at the cap is readable again for level-triggered epoll. A TLS
      // session is not: read on now that serve() made room, or once the pending response is out.
      if (!capped || !c.ssl || c.closing) return true;
      if (c.writing) {
        c.tls_more = true;
        return true;
      }
      if (c.in.size() > kMaxInput) return false;  // serve() consumed nothing (kMaxInput says it cannot)
    }
  };

  // accept() failing with EMFILE / ENFILE leaves the listening socket readable: level-triggered
  // epoll would report it again at once and the loop would spin. Stop watching it for a moment.
  int64_t accept_resume_ns = 0, last_emfile_log_ns = INT64_MIN / 2;
  std::vector<int> closed_in_batch;
  // At the cap, the connection to close, least recently active first within each class
  // (ADVICE r4); -1 = none (every connection is mid-response):
  //   0 never answered a request, nothing pending (a connect flood's idle sockets)
  //   1 never answered, a request partly read (a trickler)
  //   2 answered before, idle now (Prometheus' keep-alive between scrapes: kept longest)
  //   3 answered before, a request partly read
  // (bytes still in the socket count as a partial request). `worst_class`: the highest class that
  // may be closed (an accept at the cap: any; paying another loop's eviction debt: 0 only).
  auto pick_victim = [&](int worst_class) {
    int victim = -1, best = worst_class + 1;
    for (int vfd : L->lru) {  // oldest first; a connection mid-response is skipped
      auto vit = L->conns.find(vfd);
      if (vit == L->conns.end() || vit->second.writing) continue;
      const Conn& vc = vit->second;
      int cls = (vc.served > 0 ? 2 : 0) + (vc.in.empty() ? 0 : 1);
      if (vc.in.empty()) {
        // bytes waiting in the socket that this loop has not read yet (a scraper accepted in this
        // batch, whose request the batch's read events have not reached, or an eviction debt paid
        // before them): not idle
        int avail = 0;
        if (ioctl(vfd, FIONREAD, &avail) == 0 && avail > 0) cls += 1;
      }
      if (cls < best) {
        best = cls;
        victim = vfd;
        if (cls == 0) break;
      }
    }
    return victim;
  };
  auto evict = [&](int victim) {
    close_conn(victim);
    evicted_.fetch_add(1, std::memory_order_relaxed);
    closed_in_batch.push_back(victim);  // its number may come back from accept() below
  };
  while (running_.load(std::memory_order_relaxed)) {
    int n = epoll_wait(L->ep, evs, 256, accept_resume_ns ? 100 : rt_on ? 100 : 1000);
    int64_t now = mono_ns();
    closed_in_batch.clear();
    // evictions another loop asked for (it admitted a newcomer at the cap with nothing to close);
    // owed only while the server is still over the cap (connections that closed by themselves
    // since have paid it)
    for (int debt = evict_debt_.load(std::memory_order_relaxed); debt > 0;) {
      if (conns_.load(std::memory_order_relaxed) <= max_conns_ * static_cast<size_t>(nthreads_)) {
        evict_debt_.compare_exchange_strong(debt, 0, std::memory_order_relaxed);
        break;
      }
      // only a connect flood's idle sockets pay a debt: never a request waiting to be read, nor a
      // scraper's keep-alive (the server stays up to kDebtSlack over the cap meanwhile)
      const int victim = pick_victim(0);
      if (victim < 0) break;  // nothing here either: the debt stays for a loop that has some
      if (!evict_debt_.compare_exchange_weak(debt, debt - 1, std::memory_order_relaxed)) continue;
      evict(victim);
      debt = evict_debt_.load(std::memory_order_relaxed);
    }
    if (accept_resume_ns && now >= accept_resume_ns) {
      accept_resume_ns = 0;
      watch_listener(L, true);
    }
    if (rt_on) {
      if (now - win_start >= kRtWindowNs) {  // new window: back to FIFO
        win_start = now;
        win_cpu0 = thread_cpu_ns();
        if (!fifo && set_fifo(prio) == 0) {
          fifo = true;
          rt_loops_.fetch_add(1);
        }
      } else if (fifo && thread_cpu_ns() - win_cpu0 > budget_ns) {  // budget spent: yield the CPU
        if (set_fifo(0) == 0) {
          fifo = false;
          rt_loops_.fetch_sub(1);
          rt_demotions_.fetch_add(1, std::memory_order_relaxed);
        }
      }
    }
    for (int i = 0; i < n; ++i) {
      // the RT budget is also checked inside a batch (every 32 events): one batch of up to 256
      // events must not run past the budget at SCHED_FIFO
      if (fifo && i > 0 && (i & 31) == 0 && thread_cpu_ns() - win_cpu0 > budget_ns && set_fifo(0) == 0) {
        fifo = false;
        rt_loops_.fetch_sub(1);
        rt_demotions_.fetch_add(1, std::memory_order_relaxed);
      }
      int fd = evs[i].data.fd;
      if (fd == L->wake) {  // stop() or an eviction request (handled above): drain the counter
        uint64_t v;
        ssize_t r = read(L->wake, &v, sizeof v);
        (void)r;
        continue;
      }
      if (fd == L->lfd) {
        while (true) {
          int cfd = accept4(L->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (cfd < 0) {
            if (errno == EMFILE || errno == ENFILE) {
              if (now - last_emfile_log_ns > 10'000'000'000) {
                last_emfile_log_ns = now;
                GPUMON_LOG(LogLevel::kWarn, "http", "accept: out of file descriptors; pausing accepts for 100 ms");
              }
              accept_resume_ns = now + 100'000'000;
              watch_listener(L, false);
            }
            break;
          }
          // the cap is the server's (loops x per-loop share): with one EPOLLEXCLUSIVE socket the first
          // idle loop takes most connections, so a per-loop count would cap it at 1/N of the fds
          const size_t cap = max_conns_ * static_cast<size_t>(nthreads_);
          if (conns_.load(std::memory_order_relaxed) >= cap) {
            // full: make room by closing a connection of this loop that is not sending a response
            const int victim = pick_victim(3);
            if (victim >= 0) {
              evict(victim);
            } else if (nthreads_ > 1 && conns_.load(std::memory_order_relaxed) < cap + kDebtSlack) {
              // nothing to close here (the other loops took the flood: with one EPOLLEXCLUSIVE
              // socket the loops' shares are uneven): admit this one and have another loop close
              // one of its connections, rather than refuse the newcomer -- a scraper arriving
              // during a flood would be the one refused
              evict_debt_.fetch_add(1, std::memory_order_relaxed);
              for (auto& O : loops_)
                if (O.get() != L) {
                  uint64_t one = 1;
                  ssize_t w = write(O->wake, &one, sizeof one);
                  (void)w;
                }
            } else {
              close(cfd);
              continue;
            }
          }
          int one = 1;
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
          // room for a whole exposition in the socket: a node's identity body is 100-200 KB
          // (8 GPUs), over the default initial send buffer, and every EAGAIN costs the
          // response an epoll round trip through the client's reads
          if (sndbuf_ > 0) setsockopt(cfd, SOL_SOCKET, SO_SNDBUF, &sndbuf_, sizeof sndbuf_);
          Conn c;
          c.fd = cfd;
          c.last_ns = now;
          if (tls_) {
            c.ssl = tls_->new_session(cfd);
            if (!c.ssl) {
              tls_failures_.fetch_add(1, std::memory_order_relaxed);
              close(cfd);
              continue;
            }
            c.hs = true;
            c.req_start_ns = now;  // the handshake is held to the header timeout
          }
          c.lru = L->lru.insert(L->lru.end(), cfd);
          L->conns.emplace(cfd, std::move(c));
          conns_.fetch_add(1);
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.fd = cfd;
          epoll_ctl(L->ep, EPOLL_CTL_ADD, cfd, &ev);
        }
        continue;
      }
      // an event of a connection evicted earlier in this batch (the number may now be a new
      // connection's: its own events come with the next epoll_wait)
      if (!closed_in_batch.empty() &&
          std::find(closed_in_batch.begin(), closed_in_batch.end(), fd) != closed_in_batch.end())
        continue;
      auto it = L->conns.find(fd);
      if (it == L->conns.end()) continue;
      Conn& c = it->second;
      c.last_ns = now;
      L->lru.splice(L->lru.end(), L->lru, c.lru);  // most recently active last
      if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
        if (c.hs) tls_failures_.fetch_add(1, std::memory_order_relaxed);  // e.g. a scraper that reset on our certificate
        close_conn(fd);
        continue;
      }
      if (c.writing) {
        if (evs[i].events & EPOLLOUT) {
          if (!flush(c)) {
            close_conn(fd);
            continue;
          }
          if (!c.writing) {
            set_events(fd, EPOLLIN | EPOLLRDHUP);
            if (c.tls_more ? !read_serve(c, false) : !serve(c)) close_conn(fd);
          }
        }
        continue;
      }
      if (c.hs) {
        const TlsServer::Step st = tls_->handshake(c.ssl);
        if (st == TlsServer::Step::kFailed) {  // a plain-HTTP client, a wrong CA, no client certificate
          tls_failures_.fetch_add(1, std::memory_order_relaxed);
          close_conn(fd);
          continue;
        }
        if (st != TlsServer::Step::kDone) {
          set_events(fd, (st == TlsServer::Step::kWantWrite ? EPOLLOUT : EPOLLIN) | EPOLLRDHUP);
          continue;
        }
        c.hs = false;
        c.client_cert = tls_->mutual() && tls_->peer_verified(c.ssl);
        c.req_start_ns = 0;
        set_events(fd, EPOLLIN | EPOLLRDHUP);
        // the request may have come with the handshake's last flight: read it now
      }
      if (c.closing) {  // discard input until the client closes too
        char buf[8192];
        ssize_t r;
        while ((r = read(fd, buf, sizeof buf)) > 0) {
        }
        if (r == 0 || (errno != EAGAIN && errno != EINTR)) close_conn(fd);
        continue;
      }
      if (!read_serve(c, (evs[i].events & (EPOLLIN | EPOLLRDHUP)) != 0)) close_conn(fd);
    }
    if (now - last_sweep > 1000000000LL) {
      last_sweep = now;
      if (tls_ && L == loops_.front().get()) tls_->maybe_reload(now);  // certificate rotation
      std::vector<int> idle;
      for (auto& [fd, c] : L->conns)
        if (now - c.last_ns > kIdleTimeoutNs || (c.closing && now - c.closing_ns > kLingerNs) ||
            (!c.writing && !c.closing && (c.hs || !c.in.empty()) && now - c.req_start_ns > header_timeout_ns_)) {
          idle.push_back(fd);
          if (c.hs) tls_failures_.fetch_add(1, std::memory_order_relaxed);  // a handshake that never finished
        }
      for (int fd : idle) close_conn(fd);
    }
  }
  if (fifo) rt_loops_.fetch_sub(1);
}

}  // namespace gpumon

// Minimal epoll HTTP/1.1 server for /metrics, /healthz, /readyz.
//
// The reference has no server (push-only). This one is built for flat scrape latency: responses
// reference immutable pre-rendered buffers (zero-copy writev), keep-alive and pipelining are
// supported, gzip is computed at most once per snapshot, and N event-loop threads share ONE
// listening socket (EPOLLEXCLUSIVE wake-ups). There is no SO_REUSEPORT: a second exporter on the
// same port fails with EADDRINUSE instead of silently taking a share of the scrapes. No Python /
// GIL on this path.
//
// Listen addresses (parse_listen): "host:port", "[v6]:port", ":port" / "port" / "*:port" (every
// address). Every address binds [::] with IPV6_V6ONLY=0, one dual-stack socket that takes IPv4
// (as ::ffff:a.b.c.d) and IPv6 scrapes, and falls back to 0.0.0.0 where the kernel has no IPv6;
// "[::]:port" is dual-stack without the fallback; "0.0.0.0:port" is IPv4 only, "[::1]:port" v6 only.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace gpumon {

class TlsServer;

struct HttpRequest {
  std::string method;
  std::string path;        // without query string
  std::string query;
  bool keep_alive = true;
  bool accept_gzip = false;
  std::string authorization;  // the Authorization header's value (http_auth_token_file)
  // mutual TLS (tls_client_ca_file): the connection's client presented a certificate that
  // verified. Handshakes without one succeed (the kubelet's probes); /metrics refuses them.
  bool client_cert = false;
};

struct HttpResponse {
  int status = 200;
  std::string content_type = "text/plain; charset=utf-8";
  std::string extra_headers;                // each "Name: value\r\n"
  std::shared_ptr<const void> owner;        // keeps `data` alive
  const char* data = nullptr;
  size_t len = 0;
  std::string inline_body;                  // used when data == nullptr
};

// "host:port" | "[v6]:port" | ":port" | "*:port" | "port" -> host ("" = every address, dual-stack)
// and port (0 = ephemeral). false with the reason in *err.
bool parse_listen(const std::string& listen, std::string* host, int* port, std::string* err);

// The memory limit the connection cap is sized against: the smallest cgroup v2 memory.max from the
// cgroup named in `proc_cgroup` (/proc/self/cgroup) up to `cgroup_root` (/sys/fs/cgroup), else the
// v1 limit; 0 = none. GPUMON_HTTP_MEMORY_BUDGET overrides.
uint64_t memory_limit_bytes(const std::string& proc_cgroup, const std::string& cgroup_root);

class HttpServer {
 public:
  using Handler = std::function<void(const HttpRequest&, HttpResponse*)>;
  using Observer = std::function<void(const std::string& path, double seconds)>;

  HttpServer(std::string addr, int port, int threads, Handler h, Observer obs);
  ~HttpServer();
  // Opt-in SCHED_FIFO for the event loops (http_rt_priority; needs CAP_SYS_NICE): a scrape is then
  // served as soon as it arrives on a CPU-saturated node. Each loop may spend at most
  // `budget` of one CPU per 100 ms window at that priority; past it the loop drops to normal
  // scheduling until the window ends, so a request flood cannot monopolise a core. Before start().
  void set_rt(int prio, double budget) {
    rt_prio_ = prio;
    rt_budget_ = budget;
  }
  // Serve HTTPS: every accepted connection handshakes first (tls.h TlsServer). Before start().
  void set_tls(std::shared_ptr<TlsServer> tls) { tls_ = std::move(tls); }
  bool tls() const { return tls_ != nullptr; }
  uint64_t tls_failures() const { return tls_failures_.load(); }  // handshakes that failed or timed out
  const TlsServer* tls_server() const { return tls_.get(); }
  TlsServer* tls_server() { return tls_.get(); }
  int rt_loops() const { return rt_loops_.load(); }           // loops running at SCHED_FIFO now
  uint64_t rt_demotions() const { return rt_demotions_.load(); }  // budget exhaustions
  uint64_t evicted() const { return evicted_.load(); }            // closed to make room at the cap
  size_t max_conns() const { return max_conns_; }                 // per loop share; the cap is x loops (start())
  bool start(std::string* err);
  void stop();
  int port() const { return port_; }
  // What was bound, for logs: "[::]:9400 (dual-stack)", "0.0.0.0:9400", "[::1]:9400", ...
  const std::string& bound() const { return bound_; }
  uint64_t connections() const { return conns_.load(); }
  uint64_t requests() const { return requests_.load(); }

 private:
  struct Loop;
  void run(Loop* L);
  bool watch_listener(Loop* L, bool on);  // add / remove the shared listening socket in L's epoll set
  std::string addr_;
  int port_;
  int lfd_ = -1;         // the one listening socket, shared by the loops
  std::atomic<bool> exclusive_{true};  // EPOLLEXCLUSIVE accepted by the kernel (>= 4.5)
  std::string bound_;
  int nthreads_;
  int sndbuf_ = 0;  // SO_SNDBUF for accepted connections (0: kernel default)
  size_t max_conns_ = 4096;        // per loop: kMaxConnsPerLoop, less when RLIMIT_NOFILE is low (start())
  int64_t header_timeout_ns_ = 0;  // a request header not complete this long after its first byte
  Handler handler_;
  Observer observer_;
  std::vector<std::unique_ptr<Loop>> loops_;
  std::atomic<bool> running_{false};
  std::atomic<uint64_t> conns_{0};
  std::atomic<uint64_t> requests_{0};
  int rt_prio_ = 0;
  double rt_budget_ = 0.2;
  std::atomic<int> rt_loops_{0};
  std::atomic<uint64_t> rt_demotions_{0};
  std::atomic<uint64_t> evicted_{0};  // connections closed to make room at the cap
  // Evictions owed by the loops: a loop at the cap with nothing of its own to evict (the other
  // loop holds the flood) admits the newcomer and asks the others to close one of theirs.
  std::atomic<int> evict_debt_{0};
  std::shared_ptr<TlsServer> tls_;
  std::atomic<uint64_t> tls_failures_{0};
};

}  // namespace gpumon

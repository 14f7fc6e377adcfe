// Tiny blocking HTTP/1.1 client: Influx compat push (keep-alive POST) and the scrape load
// generator used by bench.py (p50/p99 /metrics latency measured from the client side, the way a
// Prometheus server sees it).
//
// Reference parity: the reference opens a NEW TCP connection and blocks for every single line it
// posts (requests.post per line, /root/reference/gpu.py:145,218,252; ~35-40 ms per pod_gpu line,
// BASELINE.md). Here one batched POST per tick reuses one connection.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace gpumon {

struct Url {
  std::string host;         // IPv6 literals without the brackets
  int port = 80;
  std::string path = "/";   // including ?query
  std::string auth_header;  // "Authorization: Basic ...\r\n" from user:password@ (InfluxDB 1.x auth)
  bool tls = false;         // https://
  bool ok = false;
  std::string error;        // why ok is false
};
// http[s]://[user[:password]@]host[:port][/path?query]; host may be a [v6] literal; the port
// defaults to 80 / 443. Other schemes, a missing host or a bad port: ok = false, reason in `error`.
Url parse_url(const std::string& url);
// host[:port] for a Host header or a log line: an IPv6 literal in brackets.
std::string host_port(const std::string& host, int port);
// The URL with any password replaced by "***" (for logs and --print-config).
std::string redact_url(const std::string& url);
std::string base64_encode(const std::string& in);

class TlsContext;
class TlsConn;

class HttpClient {
 public:
  explicit HttpClient(double timeout_s = 2.0);
  ~HttpClient();
  // TLS settings for https:// URLs (created with TlsContext::create); without one, an https
  // request makes a default context (system CA bundle, verification on) on first use.
  void set_tls(std::shared_ptr<TlsContext> ctx) { tls_ctx_ = std::move(ctx); }
  // Returns HTTP status (or -1 on transport error, with *err).
  int request(const std::string& method, const Url& u, const std::string& body,
              const std::string& extra_headers, std::string* resp_body, std::string* err);
  void close_conn();

 private:
  bool connect_to(const Url& u, std::string* err);
  bool send_all(const char* p, size_t n, std::string* err);
  long recv_some(char* buf, size_t n, std::string* err);  // > 0 bytes, 0 EOF, < 0 error
  int fd_ = -1;
  std::string cur_host_;
  int cur_port_ = -1;
  bool cur_tls_ = false;
  double timeout_s_;
  std::shared_ptr<TlsContext> tls_ctx_;
  std::unique_ptr<TlsConn> tls_;
};

struct ScrapeStats {
  std::vector<double> latencies_s;   // successful requests
  uint64_t errors = 0;
  uint64_t bytes = 0;
  double wall_s = 0;
};

// `concurrency` client threads, each issuing requests back-to-back (or paced to `rate_hz`
// total when > 0) until `n_requests` total have completed or `duration_s` elapsed.
ScrapeStats scrape_load(const std::string& host, int port, const std::string& path, int n_requests,
                        double duration_s, int concurrency, double rate_hz, bool keep_alive,
                        bool gzip);

}  // namespace gpumon

// TLS for the Influx compat push: OpenSSL 3 loaded at run time (dlopen libssl.so.3 +
// libcrypto.so.3) into a typed function table, the way smi_table.h loads libamd_smi. The exporter
// keeps no link-time (or build-time header) TLS dependency: an http:// deployment never maps
// libssl, and an https:// URL on a host without it is a configuration error at startup.
//
// Reference parity: the reference posts with requests.post(INFLUXDB_URL, ...) (/root/reference/
// gpu.py:20,145,218,252), which takes https:// URLs and verifies certificates against the system
// CA bundle by default. Same defaults here: peer verification and host-name / IP checks are on;
// `influx_ca_file` replaces the bundle, `influx_tls_insecure` (off by default) disables both.
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>

namespace gpumon {

struct TlsOptions {
  std::string ca_file;      // PEM bundle; "" = the system's default verify paths / well-known bundles
  bool insecure = false;    // no peer or host-name verification (explicit opt-in only)
  std::string client_cert;  // PEM chain for mutual TLS (optional, with client_key)
  std::string client_key;
};

struct SslApi;  // the dlopen'd function table (tls.cpp)

// mtime, size and inode of a file, following symlinks (the kubelet's ..data swap of a Secret
// volume): a different stamp means the file was replaced. All zero / -1 when it cannot be read.
struct FileStamp {
  int64_t mtime_ns = 0, size = -1;
  uint64_t ino = 0;
  static FileStamp of(const std::string& path);
  bool operator==(const FileStamp& o) const { return mtime_ns == o.mtime_ns && size == o.size && ino == o.ino; }
  bool operator!=(const FileStamp& o) const { return !(*this == o); }
};

// How often TLS files are re-stamped for rotation: `dflt_ns`, or $GPUMON_TLS_RELOAD_S seconds.
int64_t tls_reload_period_ns(int64_t dflt_ns);

// Loads libssl / libcrypto once per process (thread-safe); nullptr with *err when unavailable.
// $GPUMON_LIBSSL / $GPUMON_LIBCRYPTO override the sonames.
const SslApi* ssl_api(std::string* err);

// One client context: protocol floor TLS 1.2, trust store, verification mode, client certificate.
class TlsContext {
 public:
  static std::shared_ptr<TlsContext> create(const TlsOptions& o, std::string* err);
  ~TlsContext();
  void* raw() const { return ctx_; }
  const SslApi* api() const { return api_; }
  bool verify() const { return !insecure_; }

 private:
  TlsContext() = default;
  const SslApi* api_ = nullptr;
  void* ctx_ = nullptr;  // SSL_CTX*
  bool insecure_ = false;
};

// One TLS session over a connected socket. The socket is switched to non-blocking and every call
// waits with poll() against its own deadline (timeout_s from the call's start): a peer that
// drips a handshake or a record a byte at a time cannot stretch one call past the timeout (with
// blocking I/O each of OpenSSL's recv()s would get the whole SO_RCVTIMEO again).
class TlsConn {
 public:
  TlsConn(std::shared_ptr<TlsContext> ctx, double timeout_s)
      : ctx_(std::move(ctx)), timeout_ns_(timeout_s > 0 ? static_cast<int64_t>(timeout_s * 1e9) : INT64_MAX / 4) {}
  ~TlsConn();
  // SNI + host-name (or IP literal) check + handshake. false with a named reason in *err, e.g.
  // "tls: certificate verify failed: self-signed certificate in certificate chain".
  bool handshake(int fd, const std::string& host, std::string* err);
  // Whole buffer or false (*err set).
  bool write_all(const char* p, size_t n, std::string* err);
  // > 0 bytes read, 0 = orderly close (close_notify or EOF), < 0 = error / timeout (*err set).
  long read_some(char* buf, size_t n, std::string* err);
  void shutdown();

 private:
  std::string last_error(int ret);
  // After an SSL call returned `ret`: wait for the socket in the direction OpenSSL wants, until
  // `deadline` (mono ns). true = retry the call; false = a real error or the deadline (*err set).
  bool wait_retry(int ret, int64_t deadline, std::string* err);
  std::shared_ptr<TlsContext> ctx_;
  void* ssl_ = nullptr;  // SSL*
  int fd_ = -1;
  int64_t timeout_ns_;
};

// Server side: /metrics over HTTPS (tls_cert_file / tls_key_file; tls_client_ca_file adds mutual
// TLS, a scraper without a certificate signed by that CA fails the handshake). One context per
// server, shared by the HTTP loops; one session per accepted connection, driven non-blocking by
// the loop's epoll events (http_server.cpp). No session resumption: a Prometheus keep-alive
// connection handshakes once per connection anyway.
class TlsServer {
 public:
  static std::shared_ptr<TlsServer> create(const std::string& cert_file, const std::string& key_file,
                                           const std::string& client_ca_file, std::string* err);
  ~TlsServer();
  bool mutual() const { return !ca_.empty(); }
  // Certificate rotation (cert-manager, a renewed Secret: the kubelet swaps the mounted files): at
  // most every 5 s, the files' mtime / size / inode are compared with the loaded ones; on a change a
  // new context is built and swapped in. New connections get it; sessions in flight keep theirs. A
  // change that does not load (a half-written rotation) keeps the old context and is retried on the
  // files' next change. Called by one HTTP loop.
  void maybe_reload(int64_t now_ns);
  // Re-check the files at the loop's next sweep (within a second) instead of the next period: SIGHUP.
  void request_reload() { reload_now_ = true; }
  int64_t not_after() const { return not_after_.load(); }  // the serving certificate's expiry (unix s; 0 unknown)
  uint64_t reloads_ok() const { return reloads_ok_.load(); }
  uint64_t reloads_failed() const { return reloads_failed_.load(); }
  // A session over an accepted non-blocking socket; nullptr if OpenSSL refuses one.
  void* new_session(int fd) const;
  enum class Step { kDone, kWantRead, kWantWrite, kFailed };
  Step handshake(void* ssl) const;
  // > 0 bytes read; 0 = the peer closed; -1 = nothing now (wait for EPOLLIN); -2 = a TLS error
  long read(void* ssl, char* buf, size_t n) const;
  // > 0 bytes written; -1 = the socket is full (wait for EPOLLOUT); -2 = a TLS error
  long write(void* ssl, const char* p, size_t n) const;
  void notify_close(void* ssl) const;  // one non-blocking close_notify attempt
  // Mutual TLS: the session's peer sent a certificate and it verified against the client CA.
  bool peer_verified(void* ssl) const;
  void free_session(void* ssl) const;

 private:
  TlsServer() = default;
  const SslApi* api_ = nullptr;
  std::string cert_, key_, ca_;
  mutable std::mutex mu_;
  void* ctx_ = nullptr;  // SSL_CTX*, swapped under mu_ on a reload
  FileStamp stamps_[3];
  int64_t next_check_ns_ = 0;
  std::atomic<bool> reload_now_{false};
  std::atomic<int64_t> not_after_{0};
  std::atomic<uint64_t> reloads_ok_{0}, reloads_failed_{0};
};

// Configuration-time check of the serving certificate, key and client CA: "" = usable.
std::string check_serve_tls(const std::string& cert_file, const std::string& key_file,
                            const std::string& client_ca_file);

// Configuration-time check of a push URL and its TLS settings (both entry points call it): the
// scheme, host and port parse, a token without line breaks, an https URL with libssl loadable and a
// readable CA / client certificate. "" = usable; otherwise the reason.
std::string check_push_config(const std::string& url, const std::string& token, const TlsOptions& tls);

}  // namespace gpumon

// Bearer-token authentication of /metrics (http_auth_token_file). Prometheus sends the token with
// `authorization: {credentials_file: ...}` (prometheus-operator: `bearerTokenSecret`). The token file
// is a mounted Secret: it is re-stamped every 5 s (GPUMON_TLS_RELOAD_S) and on SIGHUP, and a
// rotated token replaces the old one for the next request. The reference had no endpoint at all
// (gpu.py pushed to InfluxDB); this guards the one gpumon serves, on its own or
// next to HTTPS / mutual TLS (tls.h TlsServer).
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>

#include "tls.h"

namespace gpumon {

class TokenAuth {
 public:
  // nullptr with *err when the file cannot be read or holds no usable token
  static std::shared_ptr<TokenAuth> create(const std::string& path, std::string* err);

  // true when `authorization` (the request's header value) is "Bearer <the current token>".
  // Compares in time independent of where the values differ. Re-stamps the file when due.
  bool allow(std::string_view authorization);
  void request_reload() { reload_now_ = true; }
  uint64_t reloads_ok() const { return reloads_ok_.load(); }
  uint64_t reloads_failed() const { return reloads_failed_.load(); }

 private:
  TokenAuth() = default;
  void maybe_reload(int64_t now_ns);
  std::string path_;
  mutable std::mutex mu_;                   // token_ swap; the reload check itself is claimed by CAS
  std::shared_ptr<const std::string> token_;
  FileStamp stamp_;                         // written by the thread holding checking_
  std::atomic<int64_t> next_check_ns_{0};
  std::atomic<bool> checking_{false}, reload_now_{false};
  std::atomic<uint64_t> reloads_ok_{0}, reloads_failed_{0};
};

// Reads a token file: the first line, surrounding whitespace trimmed; visible ASCII only, at most
// 4 KiB. "" with *token set, else the reason.
std::string read_token_file(const std::string& path, std::string* token);
// "" when `path` is empty or holds a usable token, else the reason (startup checks of both entry points)
std::string check_auth_token_file(const std::string& path);

}  // namespace gpumon

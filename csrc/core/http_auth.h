// Bearer-token authentication of /metrics (http_auth_token_file). Prometheus sends the token with
// `authorization: {credentials_file: ...}` (prometheus-operator: `bearerTokenSecret`). The token file
// is a mounted Secret: it is re-stamped every 5 s (GPUMON_TLS_RELOAD_S) and on SIGHUP, and a
// rotated file replaces the old tokens for the next request. Each line holds one accepted token, so a
// rotation needs no window of refused scrapes: add the new token as a second line, move the scrapers
// to it, then drop the old line. The reference had no endpoint at all
// (gpu.py pushed to InfluxDB); this guards the one gpumon serves, on its own or
// next to HTTPS / mutual TLS (tls.h TlsServer).
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <vector>

#include "tls.h"

namespace gpumon {

class TokenAuth {
 public:
  // nullptr with *err when the file cannot be read or holds no usable token
  static std::shared_ptr<TokenAuth> create(const std::string& path, std::string* err);

  // kOk when `authorization` (the request's header value) is "Bearer <one of the file's tokens>".
  // Compares every token, each in time independent of where the values differ. Re-stamps the file
  // when due.
  enum class Verdict { kOk, kMissing, kScheme, kToken };  // kScheme: not "Bearer ..."
  Verdict check(std::string_view authorization);
  void request_reload() { reload_now_ = true; }
  uint64_t reloads_ok() const { return reloads_ok_.load(); }
  uint64_t reloads_failed() const { return reloads_failed_.load(); }

 private:
  TokenAuth() = default;
  void maybe_reload(int64_t now_ns);
  std::string path_;
  mutable std::mutex mu_;                   // tokens_ swap; the reload check itself is claimed by CAS
  std::shared_ptr<const std::vector<std::string>> tokens_;
  FileStamp stamp_;                         // written by the thread holding checking_
  std::atomic<int64_t> next_check_ns_{0};
  std::atomic<bool> checking_{false}, reload_now_{false};
  std::atomic<uint64_t> reloads_ok_{0}, reloads_failed_{0};
};

// Reads a token file: one token per line (surrounding whitespace trimmed, blank lines skipped),
// visible ASCII only, at most 4 KiB each and kMaxTokens of them. "" with *tokens set, else the reason.
constexpr size_t kMaxTokens = 16;
std::string read_token_file(const std::string& path, std::vector<std::string>* tokens);
// "" when `path` is empty or holds a usable token, else the reason (startup checks of both entry points)
std::string check_auth_token_file(const std::string& path);

}  // namespace gpumon

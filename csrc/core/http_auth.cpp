#include "http_auth.h"

#include <fcntl.h>
#include <strings.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

#include "common.h"

namespace gpumon {

namespace {
constexpr size_t kMaxToken = 4096;
constexpr int64_t kCheckPeriodNs = 5'000'000'000LL;  // as the /metrics certificate (tls.cpp)
}  // namespace

std::string read_token_file(const std::string& path, std::vector<std::string>* tokens) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return "cannot read " + path + ": " + strerror(errno);
  // room for kMaxTokens of the longest token and their line ends, plus one byte to see "too big"
  constexpr size_t kCap = kMaxTokens * (kMaxToken + 2) + 1;
  std::string buf(kCap, '\0');
  size_t n = 0;
  while (n < kCap) {
    const ssize_t r = ::read(fd, &buf[n], kCap - n);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    n += static_cast<size_t>(r);
  }
  ::close(fd);
  if (n == kCap) return path + ": larger than " + std::to_string(kCap - 1) + " bytes";
  buf.resize(n);
  std::vector<std::string> out;
  size_t pos = 0;
  while (pos <= buf.size()) {
    size_t nl = buf.find('\n', pos);
    if (nl == std::string::npos) nl = buf.size();
    const std::string_view v = trim(std::string_view(buf).substr(pos, nl - pos));
    pos = nl + 1;
    if (v.empty()) continue;
    if (v.size() > kMaxToken) return path + ": a token longer than " + std::to_string(kMaxToken) + " bytes";
    for (const char ch : v)
      if (ch < 0x21 || ch > 0x7e) return path + ": a token has a character that is not visible ASCII";
    if (out.size() == kMaxTokens) return path + ": more than " + std::to_string(kMaxTokens) + " tokens";
    out.emplace_back(v);
  }
  if (out.empty()) return path + ": no token in the file";
  *tokens = std::move(out);
  return "";
}

std::string check_auth_token_file(const std::string& path) {
  if (path.empty()) return "";
  std::vector<std::string> t;
  return read_token_file(path, &t);
}

std::shared_ptr<TokenAuth> TokenAuth::create(const std::string& path, std::string* err) {
  std::shared_ptr<TokenAuth> a(new TokenAuth);
  a->path_ = path;
  a->stamp_ = FileStamp::of(path);  // before the read: a rotation during it is seen next time
  std::vector<std::string> t;
  if (std::string e = read_token_file(path, &t); !e.empty()) {
    *err = "http_auth_token_file: " + e;
    return nullptr;
  }
  a->tokens_ = std::make_shared<const std::vector<std::string>>(std::move(t));
  a->next_check_ns_ = mono_ns() + tls_reload_period_ns(kCheckPeriodNs);
  return a;
}

void TokenAuth::maybe_reload(int64_t now_ns) {
  if (now_ns < next_check_ns_.load(std::memory_order_relaxed) && !reload_now_.load(std::memory_order_relaxed)) return;
  // one HTTP loop re-stamps; the others go on with the current token
  if (checking_.exchange(true, std::memory_order_acquire)) return;
  reload_now_ = false;
  next_check_ns_ = now_ns + tls_reload_period_ns(kCheckPeriodNs);
  const FileStamp now = FileStamp::of(path_);
  if (now != stamp_) {
    stamp_ = now;
    std::vector<std::string> t;
    if (std::string e = read_token_file(path_, &t); e.empty()) {
      const size_t k = t.size();
      auto fresh = std::make_shared<const std::vector<std::string>>(std::move(t));
      {
        std::lock_guard<std::mutex> g(mu_);
        tokens_ = std::move(fresh);
      }
      reloads_ok_.fetch_add(1);
      GPUMON_LOG(LogLevel::kInfo, "http",
                 "reloaded the /metrics bearer tokens from " + path_ + " (" + std::to_string(k) + " accepted)");
    } else {
      reloads_failed_.fetch_add(1);
      GPUMON_LOG(LogLevel::kWarn, "http", "the bearer token file changed but is not usable (keeping the previous tokens): " + e);
    }
  }
  checking_.store(false, std::memory_order_release);
}

TokenAuth::Verdict TokenAuth::check(std::string_view authorization) {
  maybe_reload(mono_ns());
  std::shared_ptr<const std::vector<std::string>> toks;
  {
    std::lock_guard<std::mutex> g(mu_);
    toks = tokens_;
  }
  // "Bearer" is case-insensitive (RFC 7235 auth-scheme), followed by one or more spaces
  const std::string_view a = trim(authorization);
  if (a.empty()) return Verdict::kMissing;
  if (a.size() < 7 || strncasecmp(a.data(), "bearer ", 7) != 0) return Verdict::kScheme;
  const std::string_view got = trim(a.substr(7));
  // every token, and every byte of each, is compared whatever the first difference
  bool ok = false;
  for (const std::string& want : *toks) {
    unsigned diff = got.size() != want.size();
    for (size_t i = 0; i < want.size(); ++i)
      diff |= static_cast<unsigned char>(want[i]) ^ static_cast<unsigned char>(i < got.size() ? got[i] : 0);
    ok |= diff == 0;
  }
  return ok ? Verdict::kOk : Verdict::kToken;
}

}  // namespace gpumon

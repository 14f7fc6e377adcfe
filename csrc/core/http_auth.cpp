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

std::string read_token_file(const std::string& path, std::string* token) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return "cannot read " + path + ": " + strerror(errno);
  char buf[kMaxToken + 2];
  size_t n = 0;
  while (n < sizeof buf) {
    const ssize_t r = ::read(fd, buf + n, sizeof buf - n);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    n += static_cast<size_t>(r);
  }
  ::close(fd);
  std::string_view v(buf, n);
  if (const size_t nl = v.find('\n'); nl != std::string_view::npos) v = v.substr(0, nl);  // the first line
  v = trim(v);
  if (v.size() > kMaxToken) return path + ": token longer than " + std::to_string(kMaxToken) + " bytes";
  if (v.empty()) return path + ": no token in the file";
  for (const char ch : v)
    if (ch < 0x21 || ch > 0x7e) return path + ": the token has a character that is not visible ASCII";
  token->assign(v);
  return "";
}

std::string check_auth_token_file(const std::string& path) {
  if (path.empty()) return "";
  std::string t;
  return read_token_file(path, &t);
}

std::shared_ptr<TokenAuth> TokenAuth::create(const std::string& path, std::string* err) {
  std::shared_ptr<TokenAuth> a(new TokenAuth);
  a->path_ = path;
  a->stamp_ = FileStamp::of(path);  // before the read: a rotation during it is seen next time
  std::string t;
  if (std::string e = read_token_file(path, &t); !e.empty()) {
    *err = "http_auth_token_file: " + e;
    return nullptr;
  }
  a->token_ = std::make_shared<const std::string>(std::move(t));
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
    std::string t;
    if (std::string e = read_token_file(path_, &t); e.empty()) {
      auto fresh = std::make_shared<const std::string>(std::move(t));
      {
        std::lock_guard<std::mutex> g(mu_);
        token_ = std::move(fresh);
      }
      reloads_ok_.fetch_add(1);
      GPUMON_LOG(LogLevel::kInfo, "http", "reloaded the /metrics bearer token from " + path_);
    } else {
      reloads_failed_.fetch_add(1);
      GPUMON_LOG(LogLevel::kWarn, "http", "the bearer token file changed but is not usable (keeping the previous token): " + e);
    }
  }
  checking_.store(false, std::memory_order_release);
}

bool TokenAuth::allow(std::string_view authorization) {
  maybe_reload(mono_ns());
  std::shared_ptr<const std::string> tok;
  {
    std::lock_guard<std::mutex> g(mu_);
    tok = token_;
  }
  // "Bearer" is case-insensitive (RFC 7235 auth-scheme), followed by one or more spaces
  const std::string_view a = trim(authorization);
  if (a.size() < 7 || strncasecmp(a.data(), "bearer ", 7) != 0) return false;
  const std::string_view got = trim(a.substr(7));
  const std::string& want = *tok;
  // every byte of the expected token is compared whatever the first difference
  unsigned diff = got.size() != want.size();
  for (size_t i = 0; i < want.size(); ++i)
    diff |= static_cast<unsigned char>(want[i]) ^ static_cast<unsigned char>(i < got.size() ? got[i] : 0);
  return diff == 0;
}

}  // namespace gpumon

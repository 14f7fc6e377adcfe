// Docker Engine API listing (docker_lite.h).
#include "docker_lite.h"

#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "common.h"

namespace gpumon {

namespace {

constexpr int kMaxDepth = 64;                  // JSON nesting the reader follows
constexpr size_t kMaxResponse = 64u << 20;     // bytes read from the daemon at most

// Bounded recursive-descent JSON reader: extracts strings, string arrays and string maps, skips
// anything else (numbers, literals, nested objects) after validating it.
class JsonReader {
 public:
  explicit JsonReader(const std::string& s) : b_(s.data()), p_(s.data()), e_(s.data() + s.size()) {}

  bool ok() const { return err_.empty(); }
  const std::string& error() const { return err_; }
  void fail(const std::string& m) {
    if (err_.empty()) err_ = m + " at byte " + std::to_string(off());
  }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  bool peek(char c) {
    ws();
    return p_ < e_ && *p_ == c;
  }
  bool eat(char c) {
    if (!peek(c)) {
      fail(std::string("expected '") + c + "'");
      return false;
    }
    ++p_;
    return true;
  }
  bool at_end() {
    ws();
    return p_ == e_;
  }

  bool string(std::string* out) {
    if (!eat('"')) return false;
    out->clear();
    while (p_ < e_) {
      const unsigned char c = static_cast<unsigned char>(*p_++);
      if (c == '"') return true;
      if (c < 0x20) return fail("control character in string"), false;
      if (c != '\\') {
        out->push_back(static_cast<char>(c));
        continue;
      }
      if (p_ >= e_) break;
      const char x = *p_++;
      switch (x) {
        case '"': out->push_back('"'); break;
        case '\\': out->push_back('\\'); break;
        case '/': out->push_back('/'); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return false;
          if (cp >= 0xD800 && cp <= 0xDBFF) {  // high surrogate: a low one must follow
            uint32_t lo;
            if (e_ - p_ < 2 || p_[0] != '\\' || p_[1] != 'u') return fail("lone high surrogate"), false;
            p_ += 2;
            if (!hex4(&lo)) return false;
            if (lo < 0xDC00 || lo > 0xDFFF) return fail("bad low surrogate"), false;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
            return fail("lone low surrogate"), false;
          }
          utf8(cp, out);
          break;
        }
        default:
          return fail("bad escape"), false;
      }
    }
    return fail("unterminated string"), false;
  }

  // any value, discarded
  bool skip(int depth = 0) {
    if (depth > kMaxDepth) return fail("nesting too deep"), false;
    ws();
    if (p_ >= e_) return fail("unexpected end"), false;
    const char c = *p_;
    if (c == '"') {
      std::string tmp;
      return string(&tmp);
    }
    if (c == '{') {
      ++p_;
      if (peek('}')) return ++p_, true;
      for (;;) {
        std::string k;
        if (!string(&k) || !eat(':') || !skip(depth + 1)) return false;
        if (peek(',')) {
          ++p_;
          continue;
        }
        return eat('}');
      }
    }
    if (c == '[') {
      ++p_;
      if (peek(']')) return ++p_, true;
      for (;;) {
        if (!skip(depth + 1)) return false;
        if (peek(',')) {
          ++p_;
          continue;
        }
        return eat(']');
      }
    }
    if (c == '-' || (c >= '0' && c <= '9')) return number();
    for (const char* lit : {"true", "false", "null"}) {
      const size_t n = strlen(lit);
      if (static_cast<size_t>(e_ - p_) >= n && memcmp(p_, lit, n) == 0) {
        p_ += n;
        return true;
      }
    }
    return fail("unexpected character"), false;
  }

  // ["a", "b"] (null -> empty); non-string elements are skipped
  bool string_array(std::vector<std::string>* out) {
    out->clear();
    if (null()) return true;
    if (!eat('[')) return false;
    if (peek(']')) return ++p_, true;
    for (;;) {
      if (peek('"')) {
        std::string s;
        if (!string(&s)) return false;
        out->push_back(std::move(s));
      } else if (!skip(1)) {
        return false;
      }
      if (peek(',')) {
        ++p_;
        continue;
      }
      return eat(']');
    }
  }

  // {"k": "v"} (null -> empty); non-string values are skipped
  bool string_map(std::map<std::string, std::string>* out) {
    out->clear();
    if (null()) return true;
    if (!eat('{')) return false;
    if (peek('}')) return ++p_, true;
    for (;;) {
      std::string k, v;
      if (!string(&k) || !eat(':')) return false;
      if (peek('"')) {
        if (!string(&v)) return false;
        (*out)[k] = std::move(v);
      } else if (!skip(1)) {
        return false;
      }
      if (peek(',')) {
        ++p_;
        continue;
      }
      return eat('}');
    }
  }

  // {"k": v, ...}: on_member(key) must consume the value (null -> no members)
  template <typename F>
  bool members(F on_member) {
    if (null()) return true;
    if (!eat('{')) return false;
    if (peek('}')) return ++p_, true;
    for (;;) {
      std::string k;
      if (!string(&k) || !eat(':') || !on_member(k)) return false;
      if (peek(',')) {
        ++p_;
        continue;
      }
      return eat('}');
    }
  }

  // [v, ...]: on_elem() must consume each element (null -> none)
  template <typename F>
  bool elements(F on_elem) {
    if (null()) return true;
    if (!eat('[')) return false;
    if (peek(']')) return ++p_, true;
    for (;;) {
      if (!on_elem()) return false;
      if (peek(',')) {
        ++p_;
        continue;
      }
      return eat(']');
    }
  }

  bool null() {
    ws();
    if (e_ - p_ >= 4 && memcmp(p_, "null", 4) == 0) {
      p_ += 4;
      return true;
    }
    return false;
  }

 private:
  size_t off() const { return static_cast<size_t>(p_ - b_); }

  bool hex4(uint32_t* v) {
    if (e_ - p_ < 4) return fail("short \\u escape"), false;
    *v = 0;
    for (int i = 0; i < 4; ++i) {
      const char c = *p_++;
      *v <<= 4;
      if (c >= '0' && c <= '9') *v |= static_cast<uint32_t>(c - '0');
      else if (c >= 'a' && c <= 'f') *v |= static_cast<uint32_t>(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') *v |= static_cast<uint32_t>(c - 'A' + 10);
      else return fail("bad \\u escape"), false;
    }
    return true;
  }

  static void utf8(uint32_t cp, std::string* out) {
    if (cp < 0x80) {
      out->push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out->push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out->push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out->push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }

  bool number() {
    const char* s = p_;
    if (p_ < e_ && *p_ == '-') ++p_;
    const char* d = p_;
    while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    if (p_ == d) return fail("bad number"), false;
    if (p_ < e_ && *p_ == '.') {
      const char* f = ++p_;
      while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
      if (p_ == f) return fail("bad fraction"), false;
    }
    if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
      ++p_;
      if (p_ < e_ && (*p_ == '+' || *p_ == '-')) ++p_;
      const char* x = p_;
      while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
      if (p_ == x) return fail("bad exponent"), false;
    }
    return p_ > s;
  }

  const char* b_;
  const char* p_;
  const char* e_;
  std::string err_;
};

std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
  return s;
}

}  // namespace

bool docker_parse_containers(const std::string& json, std::vector<DockerContainer>* out, std::string* err) {
  out->clear();
  JsonReader r(json);
  auto bad = [&]() {
    *err = r.ok() ? "malformed container list" : r.error();
    out->clear();
    return false;
  };
  if (!r.eat('[')) return bad();
  if (r.peek(']')) {
    r.eat(']');
    return r.at_end() ? true : bad();
  }
  for (;;) {
    DockerContainer c;
    if (!r.eat('{')) return bad();
    if (!r.peek('}')) {
      for (;;) {
        std::string key;
        if (!r.string(&key) || !r.eat(':')) return bad();
        bool got;
        if (key == "Id" && r.peek('"')) {
          got = r.string(&c.id);
        } else if (key == "State" && r.peek('"')) {
          got = r.string(&c.state);
        } else if (key == "Names") {
          std::vector<std::string> names;
          got = r.string_array(&names);
          if (got && !names.empty()) c.name = names[0].size() > 1 && names[0][0] == '/' ? names[0].substr(1) : names[0];
        } else if (key == "Labels") {
          got = r.string_map(&c.labels);
        } else {
          got = r.skip(1);
        }
        if (!got) return bad();
        if (r.peek(',')) {
          r.eat(',');
          continue;
        }
        break;
      }
    }
    if (!r.eat('}')) return bad();
    if (!c.id.empty()) out->push_back(std::move(c));
    if (r.peek(',')) {
      r.eat(',');
      continue;
    }
    if (!r.eat(']') || !r.at_end()) return bad();
    return true;
  }
}

bool docker_parse_inspect(const std::string& json, DockerInspect* out, std::string* err) {
  *out = DockerInspect{};
  JsonReader r(json);
  const bool ok = r.members([&](const std::string& k) {
    if (k == "Id" && r.peek('"')) return r.string(&out->id);
    if (k == "Config")
      return r.members([&](const std::string& ck) { return ck == "Env" ? r.string_array(&out->env) : r.skip(2); });
    if (k == "HostConfig")
      return r.members([&](const std::string& hk) {
        if (hk != "Devices") return r.skip(2);
        return r.elements([&]() {
          return r.members([&](const std::string& dk) {
            if (dk == "PathOnHost" && r.peek('"')) {
              std::string path;
              if (!r.string(&path)) return false;
              out->devices.push_back(std::move(path));
              return true;
            }
            return r.skip(4);
          });
        });
      });
    return r.skip(1);
  });
  if (!ok || !r.at_end()) {
    *err = r.ok() ? "malformed container inspect" : r.error();
    return false;
  }
  return true;
}

bool http1_parse_response(const std::string& raw, int* status, std::string* body, std::string* err, bool eof) {
  const size_t hdr_end = raw.find("\r\n\r\n");
  if (hdr_end == std::string::npos) {
    *err = "truncated HTTP response header";
    return false;
  }
  const size_t line_end = raw.find("\r\n");
  const std::string line = raw.substr(0, line_end);
  if (line.compare(0, 5, "HTTP/") != 0 || line.size() < 12 || line[8] != ' ') {
    *err = "bad HTTP status line";
    return false;
  }
  *status = atoi(line.c_str() + 9);
  long long content_length = -1;
  bool chunked = false;
  for (size_t p = line_end + 2; p < hdr_end;) {
    size_t e = raw.find("\r\n", p);
    if (e == std::string::npos || e > hdr_end) e = hdr_end;
    const std::string h = raw.substr(p, e - p);
    const size_t colon = h.find(':');
    if (colon != std::string::npos) {
      const std::string name = lower(h.substr(0, colon));
      size_t v = colon + 1;
      while (v < h.size() && (h[v] == ' ' || h[v] == '\t')) ++v;
      const std::string value = lower(h.substr(v));
      if (name == "content-length") {
        char* endp = nullptr;
        content_length = strtoll(value.c_str(), &endp, 10);
        if (endp == value.c_str() || content_length < 0) {
          *err = "bad Content-Length";
          return false;
        }
      } else if (name == "transfer-encoding" && value.find("chunked") != std::string::npos) {
        chunked = true;
      }
    }
    p = e + 2;
  }
  const size_t b = hdr_end + 4;
  body->clear();
  if (chunked) {
    size_t p = b;
    for (;;) {
      const size_t e = raw.find("\r\n", p);
      if (e == std::string::npos) {
        *err = "truncated chunk size";
        return false;
      }
      char* endp = nullptr;
      const std::string sz = raw.substr(p, e - p);
      const unsigned long long n = strtoull(sz.c_str(), &endp, 16);
      if (endp == sz.c_str() || n > kMaxResponse) {
        *err = "bad chunk size";
        return false;
      }
      p = e + 2;
      if (n == 0) return true;  // trailers (if any) ignored
      if (raw.size() - p < n + 2) {
        *err = "truncated chunk";
        return false;
      }
      body->append(raw, p, n);
      p += n + 2;
    }
  }
  if (content_length >= 0) {
    if (raw.size() - b < static_cast<unsigned long long>(content_length)) {
      *err = "truncated body";
      return false;
    }
    body->assign(raw, b, static_cast<size_t>(content_length));
    return true;
  }
  if (!eof) {
    *err = "body delimited by connection close: incomplete until EOF";
    return false;
  }
  body->assign(raw, b, std::string::npos);
  return true;
}

namespace {

// One HTTP/1.0 GET on the daemon's unix socket: *status (-1 transport failure) and the body.
bool docker_get(const std::string& socket_path, const std::string& target, std::string* body_out, int* status_out,
                std::string* err, int timeout_ms) {
  int& status = *status_out;
  status = -1;
  const int64_t deadline = mono_ns() + static_cast<int64_t>(timeout_ms) * 1000000;
  std::string path = socket_path;
  if (path.rfind("unix://", 0) == 0) path = path.substr(7);
  sockaddr_un sa{};
  sa.sun_family = AF_UNIX;
  if (path.size() >= sizeof sa.sun_path) {
    *err = "socket path too long";
    return false;
  }
  memcpy(sa.sun_path, path.c_str(), path.size() + 1);
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  if (fd < 0) {
    *err = std::string("socket: ") + strerror(errno);
    return false;
  }
  struct Closer {
    int fd;
    ~Closer() { ::close(fd); }
  } closer{fd};
  auto wait_for = [&](short ev) {
    for (;;) {
      const int64_t left_ms = (deadline - mono_ns()) / 1000000;
      if (left_ms <= 0) return false;
      pollfd p{fd, ev, 0};
      const int r = ::poll(&p, 1, static_cast<int>(left_ms));
      if (r > 0) return true;
      if (r == 0 || errno != EINTR) return false;
    }
  };
  if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) {
    if (errno != EINPROGRESS && errno != EAGAIN) {
      *err = "connect " + path + ": " + strerror(errno);
      return false;
    }
    int so = 0;
    socklen_t sl = sizeof so;
    if (!wait_for(POLLOUT) || getsockopt(fd, SOL_SOCKET, SO_ERROR, &so, &sl) != 0 || so != 0) {
      *err = "connect " + path + ": " + (so ? strerror(so) : "timed out");
      return false;
    }
  }
  // HTTP/1.0: the daemon answers with Content-Length or closes the connection (no chunking)
  const std::string req = "GET " + target + " HTTP/1.0\r\nHost: docker\r\nUser-Agent: gpumon\r\n\r\n";
  for (size_t off = 0; off < req.size();) {
    const ssize_t w = ::send(fd, req.data() + off, req.size() - off, MSG_NOSIGNAL);
    if (w > 0) {
      off += static_cast<size_t>(w);
    } else if (w < 0 && (errno == EAGAIN || errno == EINTR)) {
      if (!wait_for(POLLOUT)) {
        *err = "write timed out";
        return false;
      }
    } else {
      *err = std::string("write: ") + strerror(errno);
      return false;
    }
  }
  std::string raw, body;
  int st = -1;
  bool framed = false;  // a complete Content-Length / chunked response arrived before EOF
  size_t hdr_end = std::string::npos, want = 0;
  bool chunked = false;
  char buf[65536];
  for (;;) {
    const ssize_t r = ::recv(fd, buf, sizeof buf, 0);
    if (r > 0) {
      raw.append(buf, static_cast<size_t>(r));
      if (raw.size() > kMaxResponse) {
        *err = "response too large";
        return false;
      }
      // a daemon that keeps the connection open despite HTTP/1.0 still ends the read here. The full
      // parse runs only once the bytes could hold a complete framed response (Content-Length
      // reached, or the chunked terminator just arrived), so a large listing is not re-parsed per read.
      if (hdr_end == std::string::npos && (hdr_end = raw.find("\r\n\r\n")) != std::string::npos) {
        std::string h = raw.substr(0, hdr_end);
        for (auto& c : h) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
        const size_t cl = h.find("\r\ncontent-length:");
        if (cl != std::string::npos) want = hdr_end + 4 + strtoull(h.c_str() + cl + 17, nullptr, 10);
        chunked = h.find("\r\ntransfer-encoding:") != std::string::npos && h.find("chunked") != std::string::npos;
      }
      const bool maybe_complete = hdr_end != std::string::npos &&
                                  ((want && raw.size() >= want) ||
                                   (chunked && raw.size() >= 5 && raw.compare(raw.size() - 5, 5, "0\r\n\r\n") == 0));
      std::string e;
      if (maybe_complete && http1_parse_response(raw, &st, &body, &e, false)) {
        framed = true;
        break;
      }
      continue;
    }
    if (r == 0) break;
    if (errno == EINTR) continue;
    if (errno == EAGAIN) {
      if (!wait_for(POLLIN)) {
        *err = "read timed out";
        return false;
      }
      continue;
    }
    *err = std::string("read: ") + strerror(errno);
    return false;
  }
  if (!framed && !http1_parse_response(raw, &st, &body, err, true)) return false;
  status = st;
  if (st != 200) {
    *err = "GET " + target + ": HTTP " + std::to_string(st) + (body.empty() ? "" : ": " + body.substr(0, 200));
    return false;
  }
  *body_out = std::move(body);
  return true;
}

}  // namespace

bool docker_list(const std::string& socket_path, std::vector<DockerContainer>* out, std::string* err, int timeout_ms,
                 int* http_status) {
  int local_status;
  out->clear();
  std::string body;
  return docker_get(socket_path, "/containers/json", &body, http_status ? http_status : &local_status, err,
                    timeout_ms) &&
         docker_parse_containers(body, out, err);
}

bool docker_inspect(const std::string& socket_path, const std::string& id, DockerInspect* out, std::string* err,
                    int timeout_ms, int* http_status) {
  int local_status;
  int& status = http_status ? *http_status : local_status;
  status = -1;
  if (id.empty() || id.size() > 128 || id.find_first_not_of("0123456789abcdef") != std::string::npos) {
    *err = "container id must be hex";
    return false;
  }
  std::string body;
  return docker_get(socket_path, "/containers/" + id + "/json", &body, &status, err, timeout_ms) &&
         docker_parse_inspect(body, out, err);
}

}  // namespace gpumon

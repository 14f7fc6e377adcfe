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
#include "json_lite.h"

namespace gpumon {

namespace {

constexpr size_t kMaxResponse = 64u << 20;     // bytes read from the daemon at most

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
    // EAGAIN on a non-blocking unix-socket connect means the listener's backlog is full and no
    // connection was made (unlike TCP's EINPROGRESS): report it rather than wait for it
    if (errno != EINPROGRESS) {
      *err = "connect " + path + ": " + (errno == EAGAIN ? std::string("listener backlog full") : strerror(errno));
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

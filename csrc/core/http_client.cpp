#include "http_client.h"

#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cctype>
#include <cerrno>
#include <cstring>
#include <strings.h>
#include <thread>

#include "common.h"
#include "tls.h"

namespace gpumon {

std::string base64_encode(const std::string& in) {
  static const char* k = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  out.reserve((in.size() + 2) / 3 * 4);
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    const uint32_t v = (static_cast<uint8_t>(in[i]) << 16) | (static_cast<uint8_t>(in[i + 1]) << 8) |
                       static_cast<uint8_t>(in[i + 2]);
    out += k[v >> 18];
    out += k[(v >> 12) & 63];
    out += k[(v >> 6) & 63];
    out += k[v & 63];
  }
  if (i < in.size()) {
    const uint32_t v = (static_cast<uint8_t>(in[i]) << 16) |
                       (i + 1 < in.size() ? static_cast<uint8_t>(in[i + 1]) << 8 : 0);
    out += k[v >> 18];
    out += k[(v >> 12) & 63];
    out += i + 1 < in.size() ? k[(v >> 6) & 63] : '=';
    out += '=';
  }
  return out;
}

namespace {

std::string pct_decode(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && isxdigit(static_cast<unsigned char>(s[i + 1])) &&
        isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      out += static_cast<char>(strtol(s.substr(i + 1, 2).c_str(), nullptr, 16));
      i += 2;
    } else {
      out += s[i];
    }
  }
  return out;
}

}  // namespace

Url parse_url(const std::string& url) {
  Url u;
  auto bad = [&](const std::string& why) {
    u.ok = false;
    u.error = why;
    return u;
  };
  std::string s = url;
  if (starts_with(s, "http://")) {
    s = s.substr(7);
  } else if (starts_with(s, "https://")) {
    s = s.substr(8);
    u.tls = true;
    u.port = 443;
  } else {
    const size_t sc = s.find("://");
    return bad(sc == std::string::npos ? "no http:// or https:// scheme"
                                       : "unsupported scheme '" + s.substr(0, sc) + "' (http or https)");
  }
  size_t slash = s.find_first_of("/?#");
  std::string hp = slash == std::string::npos ? s : s.substr(0, slash);
  u.path = slash == std::string::npos ? "/" : s.substr(slash);
  const size_t frag = u.path.find('#');  // never sent (RFC 9110 4.2.4)
  if (frag != std::string::npos) u.path.resize(frag);
  if (u.path.empty() || u.path[0] != '/') u.path = "/" + u.path;
  if (u.path.find_first_of(" \r\n\t") != std::string::npos) return bad("whitespace in the path");
  const size_t at = hp.rfind('@');
  if (at != std::string::npos) {
    u.auth_header = "Authorization: Basic " + base64_encode(pct_decode(hp.substr(0, at))) + "\r\n";
    hp = hp.substr(at + 1);
  }
  std::string port;
  if (!hp.empty() && hp[0] == '[') {  // [v6]:port
    const size_t rb = hp.find(']');
    if (rb == std::string::npos) return bad("unterminated [IPv6] literal");
    u.host = hp.substr(1, rb - 1);
    if (rb + 1 < hp.size()) {
      if (hp[rb + 1] != ':') return bad("junk after the [IPv6] literal");
      port = hp.substr(rb + 2);
      if (port.empty()) return bad("empty port");
    }
  } else {
    const size_t colon = hp.rfind(':');
    u.host = colon == std::string::npos ? hp : hp.substr(0, colon);
    if (colon != std::string::npos) {
      port = hp.substr(colon + 1);
      if (port.empty()) return bad("empty port");
    }
    if (u.host.find(':') != std::string::npos) return bad("an IPv6 host needs brackets ([v6]:port)");
  }
  if (u.host.empty()) return bad("no host");
  if (u.host.find_first_of(" \r\n\t/") != std::string::npos) return bad("bad character in the host");
  if (!port.empty()) {
    if (port.find_first_not_of("0123456789") != std::string::npos || port.size() > 5) return bad("bad port '" + port + "'");
    u.port = atoi(port.c_str());
  }
  if (u.port <= 0 || u.port >= 65536) return bad("port out of range");
  u.ok = true;
  return u;
}

std::string host_port(const std::string& host, int port) {
  const bool v6 = host.find(':') != std::string::npos;
  return (v6 ? "[" + host + "]" : host) + ":" + std::to_string(port);
}

std::string redact_url(const std::string& url) {
  const size_t scheme = url.find("://");
  const size_t start = scheme == std::string::npos ? 0 : scheme + 3;
  const size_t end = url.find_first_of("/?", start);
  const size_t at = url.rfind('@', end == std::string::npos ? std::string::npos : end);
  if (at == std::string::npos || at < start) return url;
  const size_t colon = url.find(':', start);
  if (colon == std::string::npos || colon > at) return url;  // user without a password
  return url.substr(0, colon + 1) + "***" + url.substr(at);
}

HttpClient::HttpClient(double timeout_s) : timeout_s_(timeout_s) {}

HttpClient::~HttpClient() { close_conn(); }

void HttpClient::close_conn() {
  if (tls_) tls_->shutdown();
  tls_.reset();
  if (fd_ >= 0) close(fd_);
  fd_ = -1;
}

bool HttpClient::send_all(const char* p, size_t n, std::string* err) {
  if (tls_) return tls_->write_all(p, n, err);
  while (n) {
    ssize_t w = send(fd_, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      *err = std::string("send: ") + strerror(errno);
      return false;
    }
    p += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

long HttpClient::recv_some(char* buf, size_t n, std::string* err) {
  if (tls_) return tls_->read_some(buf, n, err);
  ssize_t r;
  do r = recv(fd_, buf, n, 0);
  while (r < 0 && errno == EINTR);
  if (r < 0) *err = errno == EAGAIN || errno == EWOULDBLOCK ? "timed out" : std::string("recv: ") + strerror(errno);
  return r;
}

bool HttpClient::connect_to(const Url& u, std::string* err) {
  if (fd_ >= 0 && u.host == cur_host_ && u.port == cur_port_ && u.tls == cur_tls_) return true;
  close_conn();
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  std::string port = std::to_string(u.port);
  int rc = getaddrinfo(u.host.c_str(), port.c_str(), &hints, &res);
  if (rc != 0 || !res) {
    *err = std::string("resolve ") + u.host + ": " + gai_strerror(rc);
    return false;
  }
  for (addrinfo* p = res; p; p = p->ai_next) {
    int fd = socket(p->ai_family, p->ai_socktype | SOCK_CLOEXEC, p->ai_protocol);
    if (fd < 0) continue;
    timeval tv;
    tv.tv_sec = static_cast<long>(timeout_s_);
    tv.tv_usec = static_cast<long>((timeout_s_ - tv.tv_sec) * 1e6);
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    if (connect(fd, p->ai_addr, p->ai_addrlen) == 0) {
      fd_ = fd;
      break;
    }
    close(fd);
  }
  freeaddrinfo(res);
  if (fd_ < 0) {
    *err = "connect " + host_port(u.host, u.port) + ": " + strerror(errno);
    return false;
  }
  if (u.tls) {
    if (!tls_ctx_) {
      tls_ctx_ = TlsContext::create(TlsOptions{}, err);
      if (!tls_ctx_) {
        close_conn();
        return false;
      }
    }
    tls_ = std::make_unique<TlsConn>(tls_ctx_, timeout_s_);
    if (!tls_->handshake(fd_, u.host, err)) {
      tls_.reset();  // no close_notify after a failed handshake
      close_conn();
      return false;
    }
  }
  cur_host_ = u.host;
  cur_port_ = u.port;
  cur_tls_ = u.tls;
  return true;
}

// Largest Content-Length accepted: the client sizes its buffer from it before reading. A body
// without a length (read to EOF) is held to the same bound, and the header to kMaxHeaderBytes.
constexpr long kMaxBodyBytes = 256L << 20;
constexpr size_t kMaxHeaderBytes = 64u << 10;

int HttpClient::request(const std::string& method, const Url& u, const std::string& body,
                        const std::string& extra_headers, std::string* resp_body,
                        std::string* err) {
  for (int attempt = 0; attempt < 2; ++attempt) {
    bool reused = fd_ >= 0;
    if (!connect_to(u, err)) return -1;
    std::string req = method + " " + u.path + " HTTP/1.1\r\nHost: " + host_port(u.host, u.port) +
                      "\r\nConnection: keep-alive\r\n" + extra_headers;
    if (!body.empty() || method == "POST")
      req += "Content-Length: " + std::to_string(body.size()) + "\r\n";
    req += "\r\n";
    // a tick's push (a few KB of lines) leaves in one write: one TCP segment, or one TLS record,
    // instead of a header segment and a body segment
    const bool one_write = body.size() <= (64u << 10);
    if (one_write) req += body;
    std::string serr;
    if (!send_all(req.data(), req.size(), &serr) || (!one_write && !send_all(body.data(), body.size(), &serr))) {
      close_conn();
      if (reused) continue;  // stale keep-alive connection: retry once on a fresh one
      *err = serr;
      return -1;
    }
    std::string in;
    char buf[16384];
    size_t hdr_end = std::string::npos;
    // SO_RCVTIMEO bounds each recv(); this bounds the whole response, so a server that drips a
    // byte at a time cannot hold the caller (the Influx pusher, which stop() joins) indefinitely.
    const int64_t deadline =
        timeout_s_ > 0 ? mono_ns() + static_cast<int64_t>(2 * timeout_s_ * 1e9) : INT64_MAX;
    auto expired = [&] {
      if (mono_ns() <= deadline) return false;
      close_conn();
      *err = "response timed out";
      return true;
    };
    std::string rerr;
    while (hdr_end == std::string::npos) {
      const long r = recv_some(buf, sizeof buf, &rerr);
      if (r <= 0) break;
      in.append(buf, static_cast<size_t>(r));
      hdr_end = in.find("\r\n\r\n");
      if (hdr_end == std::string::npos && in.size() > kMaxHeaderBytes) {
        close_conn();
        *err = "response header too large";
        return -1;
      }
      if (hdr_end == std::string::npos && expired()) return -1;
    }
    if (hdr_end == std::string::npos) {
      close_conn();
      if (reused && in.empty()) continue;
      *err = "no response header" + (rerr.empty() ? std::string() : " (" + rerr + ")");
      return -1;
    }
    int status = 0;
    if (in.size() > 12) status = atoi(in.c_str() + 9);
    long clen = -1;
    bool close_after = false, chunked = false;
    size_t pos = in.find("\r\n") + 2;
    while (pos < hdr_end) {
      size_t e = in.find("\r\n", pos);
      std::string_view h(in.data() + pos, e - pos);
      if (h.size() > 15 && strncasecmp(h.data(), "content-length:", 15) == 0)
        clen = strtol(std::string(h.substr(15)).c_str(), nullptr, 10);
      if (h.size() > 18 && strncasecmp(h.data(), "transfer-encoding:", 18) == 0) {
        std::string v(h.substr(18));
        for (auto& ch : v) ch = static_cast<char>(tolower(static_cast<unsigned char>(ch)));
        chunked = v.find("chunked") != std::string::npos;
      }
      if (h.size() > 11 && strncasecmp(h.data(), "connection:", 11) == 0 &&
          h.find("close") != std::string_view::npos)
        close_after = true;
      pos = e + 2;
    }
    std::string rb = in.substr(hdr_end + 4);
    if (clen > kMaxBodyBytes) {
      close_conn();
      *err = "response body of " + std::to_string(clen) + " bytes refused";
      return -1;
    }
    if (chunked && status != 204 && status != 304) {
      // RFC 9112 7.1 (a proxy in front of InfluxDB answers errors this way): size line, data,
      // CRLF ... a 0-size chunk, optional trailers, CRLF. Keeps the connection reusable.
      std::string raw = std::move(rb), out;
      size_t at = 0;
      auto need = [&](size_t upto) -> bool {  // raw holds at least `upto` bytes, or fail
        while (raw.size() < upto) {
          const long r = recv_some(buf, sizeof buf, &rerr);
          if (r <= 0) return false;
          raw.append(buf, static_cast<size_t>(r));
          if (raw.size() > static_cast<size_t>(kMaxBodyBytes) + 4096 || expired()) return false;
        }
        return true;
      };
      auto line = [&](std::string* l) -> bool {  // next CRLF-terminated line from `at`
        size_t e;
        while ((e = raw.find("\r\n", at)) == std::string::npos) {
          if (raw.size() - at > 4096 || !need(raw.size() + 1)) return false;
        }
        *l = raw.substr(at, e - at);
        at = e + 2;
        return true;
      };
      bool ok = true;
      for (;;) {
        std::string l;
        if (!line(&l)) {
          ok = false;
          break;
        }
        char* endp = nullptr;
        const unsigned long long n = strtoull(l.c_str(), &endp, 16);  // chunk extensions after ';' ignored
        if (endp == l.c_str() || n > static_cast<unsigned long long>(kMaxBodyBytes) ||
            out.size() + n > static_cast<size_t>(kMaxBodyBytes)) {
          ok = false;
          break;
        }
        if (n == 0) {  // trailers until an empty line
          do {
            if (!line(&l)) {
              ok = false;
              break;
            }
          } while (!l.empty());
          break;
        }
        if (!need(at + n + 2) || raw.compare(at + n, 2, "\r\n") != 0) {
          ok = false;
          break;
        }
        out.append(raw, at, n);
        at += n + 2;
      }
      if (!ok) {
        const bool timed_out = !err->empty() && *err == "response timed out";
        close_conn();
        if (!timed_out) *err = "bad chunked body" + (rerr.empty() ? std::string() : " (" + rerr + ")");
        return -1;
      }
      rb = std::move(out);
    } else if (clen >= 0) {
      // the body lands in place: one buffer of the announced length, no 16 KB staging copies
      size_t got = std::min(rb.size(), static_cast<size_t>(clen));
      rb.resize(static_cast<size_t>(clen));
      while (got < static_cast<size_t>(clen)) {
        const long r = recv_some(&rb[got], static_cast<size_t>(clen) - got, &rerr);
        if (r <= 0) {
          close_conn();
          *err = "short body" + (rerr.empty() ? std::string() : " (" + rerr + ")");
          return -1;
        }
        got += static_cast<size_t>(r);
        if (got < static_cast<size_t>(clen) && expired()) return -1;
      }
    } else if (status != 204 && status != 304) {
      // no length: read to EOF
      while (true) {
        const long r = recv_some(buf, sizeof buf, &rerr);
        if (r <= 0) break;
        rb.append(buf, static_cast<size_t>(r));
        if (rb.size() > static_cast<size_t>(kMaxBodyBytes)) {
          close_conn();
          *err = "response body too large";
          return -1;
        }
        if (expired()) return -1;
      }
      close_after = true;
    }
    if (resp_body) *resp_body = std::move(rb);
    if (close_after) close_conn();
    return status;
  }
  *err = "request failed";
  return -1;
}

ScrapeStats scrape_load(const std::string& host, int port, const std::string& path, int n_requests,
                        double duration_s, int concurrency, double rate_hz, bool keep_alive,
                        bool gzip) {
  ScrapeStats total;
  concurrency = std::max(1, concurrency);
  std::atomic<int> issued{0};
  std::vector<ScrapeStats> per(concurrency);
  int64_t t0 = mono_ns();
  int64_t deadline = duration_s > 0 ? t0 + static_cast<int64_t>(duration_s * 1e9) : INT64_MAX;
  double per_thread_period = rate_hz > 0 ? concurrency / rate_hz : 0.0;
  std::vector<std::thread> th;
  Url u;
  u.host = host;
  u.port = port;
  u.path = path;
  u.ok = true;
  std::string hdr = gzip ? "Accept-Encoding: gzip\r\n" : "";
  for (int t = 0; t < concurrency; ++t) {
    th.emplace_back([&, t] {
      HttpClient c(5.0);
      int64_t next = t0 + static_cast<int64_t>(per_thread_period * 1e9 * t / concurrency);
      while (true) {
        if (n_requests > 0 && issued.fetch_add(1) >= n_requests) break;
        if (mono_ns() >= deadline) break;
        if (per_thread_period > 0) {
          int64_t now = mono_ns();
          if (next > now) std::this_thread::sleep_for(std::chrono::nanoseconds(next - now));
          next += static_cast<int64_t>(per_thread_period * 1e9);
        }
        std::string body, err;
        int64_t a = mono_ns();
        int st = c.request("GET", u, "", hdr, &body, &err);
        int64_t b = mono_ns();
        if (st == 200) {
          per[t].latencies_s.push_back((b - a) * 1e-9);
          per[t].bytes += body.size();
        } else {
          per[t].errors++;
        }
        if (!keep_alive) c.close_conn();
      }
    });
  }
  for (auto& x : th) x.join();
  total.wall_s = (mono_ns() - t0) * 1e-9;
  for (auto& p : per) {
    total.latencies_s.insert(total.latencies_s.end(), p.latencies_s.begin(), p.latencies_s.end());
    total.errors += p.errors;
    total.bytes += p.bytes;
  }
  return total;
}

}  // namespace gpumon

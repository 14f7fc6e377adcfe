#include "grpc_lite.h"

#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <mutex>

#include "common.h"
#include "hpack.h"

namespace gpumon {

namespace {

enum : uint8_t {
  kData = 0, kHeaders = 1, kRstStream = 3, kSettings = 4, kPing = 6, kGoaway = 7, kWindowUpdate = 8, kContinuation = 9
};
enum : uint8_t { kEndStream = 0x1, kAck = 0x1, kEndHeaders = 0x4, kPadded = 0x8, kPriority = 0x20 };
constexpr uint32_t kWindow = 16u << 20;
constexpr size_t kMaxResponse = 64u << 20;  // buffered frames, and the reassembled body

void frame(std::string* o, uint8_t type, uint8_t flags, uint32_t stream, std::string_view payload) {
  const uint32_t n = static_cast<uint32_t>(payload.size());
  o->push_back(static_cast<char>((n >> 16) & 0xFF));
  o->push_back(static_cast<char>((n >> 8) & 0xFF));
  o->push_back(static_cast<char>(n & 0xFF));
  o->push_back(static_cast<char>(type));
  o->push_back(static_cast<char>(flags));
  o->push_back(static_cast<char>((stream >> 24) & 0x7F));
  o->push_back(static_cast<char>((stream >> 16) & 0xFF));
  o->push_back(static_cast<char>((stream >> 8) & 0xFF));
  o->push_back(static_cast<char>(stream & 0xFF));
  o->append(payload);
}

void be32(std::string* o, uint32_t v) {
  for (int s = 24; s >= 0; s -= 8) o->push_back(static_cast<char>((v >> s) & 0xFF));
}

// HPACK integer with an N-bit prefix (RFC 7541 §5.1).
void hpack_int(std::string* o, uint8_t first, int prefix_bits, uint64_t v) {
  const uint64_t max = (1u << prefix_bits) - 1;
  if (v < max) {
    o->push_back(static_cast<char>(first | v));
    return;
  }
  o->push_back(static_cast<char>(first | max));
  v -= max;
  while (v >= 128) {
    o->push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  o->push_back(static_cast<char>(v));
}

// "Literal header field never indexed -- new name", plain (non-Huffman) strings (§6.2.3).
void hpack_literal(std::string* o, std::string_view name, std::string_view value) {
  o->push_back(0x10);
  hpack_int(o, 0x00, 7, name.size());
  o->append(name);
  hpack_int(o, 0x00, 7, value.size());
  o->append(value);
}

bool write_all(int fd, const std::string& b, int64_t deadline_ns) {
  size_t off = 0;
  while (off < b.size()) {
    ssize_t n = ::send(fd, b.data() + off, b.size() - off, MSG_NOSIGNAL);
    if (n > 0) {
      off += static_cast<size_t>(n);
      continue;
    }
    if (n < 0 && (errno == EAGAIN || errno == EINTR)) {
      pollfd p{fd, POLLOUT, 0};
      const int64_t left = (deadline_ns - mono_ns()) / 1000000;
      if (left <= 0 || ::poll(&p, 1, static_cast<int>(left)) <= 0) return false;
      continue;
    }
    return false;
  }
  return true;
}

}  // namespace

const char* grpc_code_name(int code) {
  static const char* const n[] = {"OK", "CANCELLED", "UNKNOWN", "INVALID_ARGUMENT", "DEADLINE_EXCEEDED",
                                  "NOT_FOUND", "ALREADY_EXISTS", "PERMISSION_DENIED", "RESOURCE_EXHAUSTED",
                                  "FAILED_PRECONDITION", "ABORTED", "OUT_OF_RANGE", "UNIMPLEMENTED", "INTERNAL",
                                  "UNAVAILABLE", "DATA_LOSS", "UNAUTHENTICATED"};
  return code >= 0 && code <= 16 ? n[code] : "UNKNOWN_CODE";
}

std::string grpc_percent_decode(std::string_view s) {
  auto hex = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && hex(s[i + 1]) >= 0 && hex(s[i + 2]) >= 0) {
      o.push_back(static_cast<char>(hex(s[i + 1]) * 16 + hex(s[i + 2])));
      i += 2;
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

bool grpc_unary_unix(const std::string& socket_path, const std::string& path, const std::string& request,
                     std::string* response, std::string* err, int timeout_ms, GrpcStatus* status_out) {
  GrpcStatus local;
  GrpcStatus& st = status_out ? *status_out : local;
  st = GrpcStatus{};
  const int64_t deadline = mono_ns() + static_cast<int64_t>(timeout_ms) * 1000000;
  std::string path_only = socket_path;
  if (path_only.rfind("unix://", 0) == 0) path_only = path_only.substr(7);
  int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    *err = std::string("socket: ") + strerror(errno);
    return false;
  }
  struct Closer {
    int fd;
    ~Closer() { ::close(fd); }
  } closer{fd};
  sockaddr_un sa{};
  sa.sun_family = AF_UNIX;
  if (path_only.size() >= sizeof sa.sun_path) {
    *err = "socket path too long";
    return false;
  }
  memcpy(sa.sun_path, path_only.c_str(), path_only.size() + 1);
  // The deadline covers every step: a unix-socket connect() blocks while the listener's backlog is
  // full, and is bounded by SO_SNDTIMEO; after it the socket is non-blocking, so a server that
  // accepts and never reads cannot stall write_all() past the deadline.
  const int sndto_ms = std::max(timeout_ms, 1);  // a zero SO_SNDTIMEO would mean "block forever"
  timeval tv{sndto_ms / 1000, (sndto_ms % 1000) * 1000};
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) {
    *err = "connect " + path_only + ": " + strerror(errno);
    return false;
  }
  ::fcntl(fd, F_SETFL, ::fcntl(fd, F_GETFL) | O_NONBLOCK);
  std::string out = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
  std::string settings;
  auto setting = [&](uint16_t id, uint32_t v) {
    settings.push_back(static_cast<char>(id >> 8));
    settings.push_back(static_cast<char>(id & 0xFF));
    be32(&settings, v);
  };
  setting(0x2, 0);        // ENABLE_PUSH off
  setting(0x4, kWindow);  // INITIAL_WINDOW_SIZE (stream)
  frame(&out, kSettings, 0, 0, settings);
  std::string wu;
  be32(&wu, kWindow - 65535);  // connection window up to 16 MiB too
  frame(&out, kWindowUpdate, 0, 0, wu);
  std::string hb;
  hpack_literal(&hb, ":method", "POST");
  hpack_literal(&hb, ":scheme", "http");
  hpack_literal(&hb, ":path", path);
  hpack_literal(&hb, ":authority", "localhost");
  hpack_literal(&hb, "content-type", "application/grpc");
  hpack_literal(&hb, "te", "trailers");
  frame(&out, kHeaders, kEndHeaders, 1, hb);
  std::string msg;
  msg.push_back(0);  // not compressed
  be32(&msg, static_cast<uint32_t>(request.size()));
  msg.append(request);
  frame(&out, kData, kEndStream, 1, msg);
  if (!write_all(fd, out, deadline)) {
    *err = "write failed";
    return false;
  }

  std::string in, body;
  bool ended = false;
  HpackDecoder hpack;      // one per connection: the dynamic table spans header blocks
  std::string hblock;      // header block being assembled (HEADERS + CONTINUATION)
  bool in_block = false, block_ends_stream = false;
  auto finish_block = [&]() -> bool {
    HeaderList fields;
    std::string herr;
    if (!hpack.decode(hblock, &fields, &herr)) {
      *err = herr;
      return false;
    }
    for (const auto& [k, v] : fields) {
      if (k == ":status") st.http_status = atoi(v.c_str());
      else if (k == "grpc-status") st.code = atoi(v.c_str());
      else if (k == "grpc-message") st.message = grpc_percent_decode(v);
    }
    hblock.clear();
    in_block = false;
    if (block_ends_stream) ended = true;
    return true;
  };
  while (!ended) {
    // parse complete frames
    while (in.size() >= 9) {
      const uint32_t len = (static_cast<uint8_t>(in[0]) << 16) | (static_cast<uint8_t>(in[1]) << 8) |
                           static_cast<uint8_t>(in[2]);
      if (in.size() < 9 + len) break;
      const uint8_t type = static_cast<uint8_t>(in[3]), flags = static_cast<uint8_t>(in[4]);
      const uint32_t stream = ((static_cast<uint8_t>(in[5]) & 0x7F) << 24) | (static_cast<uint8_t>(in[6]) << 16) |
                              (static_cast<uint8_t>(in[7]) << 8) | static_cast<uint8_t>(in[8]);
      std::string_view pl(in.data() + 9, len);
      std::string reply;
      if (type == kSettings && !(flags & kAck)) {
        frame(&reply, kSettings, kAck, 0, {});
      } else if (type == kPing && !(flags & kAck)) {
        frame(&reply, kPing, kAck, 0, pl);
      } else if (type == kGoaway) {
        *err = "GOAWAY from server";
        return false;
      } else if (type == kRstStream && stream == 1) {
        *err = "stream reset by server";
        return false;
      } else if (type == kData && stream == 1) {
        size_t pad = 0, start = 0;
        if (flags & kPadded) {
          if (pl.empty()) {
            *err = "bad padded DATA";
            return false;
          }
          pad = static_cast<uint8_t>(pl[0]);
          start = 1;
        }
        if (start + pad > pl.size()) {
          *err = "bad DATA padding";
          return false;
        }
        body.append(pl.substr(start, pl.size() - start - pad));
        if (body.size() > kMaxResponse) {
          *err = "response too large";
          return false;
        }
        if (flags & kEndStream) ended = true;
      } else if ((type == kHeaders || type == kContinuation) && stream == 1) {
        // response headers, trailers, or a Trailers-Only error response
        if ((type == kHeaders) == in_block) {
          *err = "malformed header block sequence";
          return false;
        }
        std::string_view frag = pl;
        if (type == kHeaders) {
          size_t pad = 0, start = 0;
          if (flags & kPadded) {
            if (frag.empty()) {
              *err = "bad padded HEADERS";
              return false;
            }
            pad = static_cast<uint8_t>(frag[0]);
            start = 1;
          }
          if (flags & kPriority) start += 5;
          if (start + pad > frag.size()) {
            *err = "bad HEADERS padding";
            return false;
          }
          frag = frag.substr(start, frag.size() - start - pad);
          in_block = true;
          block_ends_stream = flags & kEndStream;
        }
        hblock.append(frag);
        if ((flags & kEndHeaders) && !finish_block()) return false;
      }
      if (!reply.empty() && !write_all(fd, reply, deadline)) {
        *err = "write failed";
        return false;
      }
      in.erase(0, 9 + len);
      if (ended) break;
    }
    if (ended) break;
    const int64_t left = (deadline - mono_ns()) / 1000000;
    if (left <= 0) {
      *err = "timeout";
      return false;
    }
    pollfd p{fd, POLLIN, 0};
    if (::poll(&p, 1, static_cast<int>(left)) <= 0) {
      *err = "timeout";
      return false;
    }
    char buf[65536];
    ssize_t n = ::recv(fd, buf, sizeof buf, 0);
    if (n < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    if (n <= 0) {
      *err = "connection closed";
      return false;
    }
    in.append(buf, static_cast<size_t>(n));
    if (in.size() > kMaxResponse + 9) {
      *err = "response too large";
      return false;
    }
  }
  if (st.http_status != 0 && st.http_status != 200) {
    *err = "HTTP :status " + std::to_string(st.http_status) + (st.code >= 0 ? std::string(", grpc-status ") +
           std::to_string(st.code) + " " + grpc_code_name(st.code) : std::string());
    return false;
  }
  if (st.code > 0) {
    *err = "grpc-status " + std::to_string(st.code) + " " + grpc_code_name(st.code) +
           (st.message.empty() ? std::string() : ": " + st.message);
    return false;
  }
  if (body.size() < 5) {
    *err = st.code == 0 ? "grpc-status 0 OK without a response message"
                        : "no gRPC message and no grpc-status in the response";
    return false;
  }
  const uint32_t mlen = (static_cast<uint8_t>(body[1]) << 24) | (static_cast<uint8_t>(body[2]) << 16) |
                        (static_cast<uint8_t>(body[3]) << 8) | static_cast<uint8_t>(body[4]);
  if (body[0] != 0 || body.size() < 5 + static_cast<size_t>(mlen)) {
    *err = body[0] != 0 ? "compressed gRPC message not supported" : "truncated gRPC message";
    return false;
  }
  response->assign(body, 5, mlen);
  return true;
}

// ---------------------------------------------------------------------------------------------
bool PbReader::varint(uint64_t* v) {
  uint64_t x = 0;
  for (int s = 0; s < 64; s += 7) {
    if (p_ >= b_.size()) return ok_ = false;
    const uint8_t c = static_cast<uint8_t>(b_[p_++]);
    x |= static_cast<uint64_t>(c & 0x7F) << s;
    if (!(c & 0x80)) {
      *v = x;
      return true;
    }
  }
  return ok_ = false;
}

bool PbReader::next(uint32_t* field, uint32_t* wire) {
  if (p_ >= b_.size() || !ok_) return false;
  uint64_t key = 0;
  if (!varint(&key)) return false;
  *field = static_cast<uint32_t>(key >> 3);
  *wire = static_cast<uint32_t>(key & 7);
  return *field != 0 || (ok_ = false);
}

bool PbReader::bytes(std::string_view* v) {
  uint64_t n = 0;
  if (!varint(&n) || n > b_.size() - p_) return ok_ = false;
  *v = b_.substr(p_, n);
  p_ += n;
  return true;
}

bool PbReader::skip(uint32_t wire) {
  uint64_t tmp;
  std::string_view sv;
  switch (wire) {
    case 0: return varint(&tmp);
    case 1:
      if (b_.size() - p_ < 8) return ok_ = false;
      p_ += 8;
      return true;
    case 2: return bytes(&sv);
    case 5:
      if (b_.size() - p_ < 4) return ok_ = false;
      p_ += 4;
      return true;
    default: return ok_ = false;
  }
}

namespace {

// DynamicResource{2 claim_name, 3 claim_namespace, 4 ClaimResource{1 CDIDevice{1 name}, 2 driver_name,
// 4 device_name}} -> one row per claimed device of a wanted DRA driver.
bool parse_dynamic_resource(std::string_view b, const std::vector<std::string>& drivers, const std::string& ns,
                            const std::string& pod, const std::string& cname, std::vector<PodDeviceRow>* out) {
  PbReader dr(b);
  uint32_t f, w;
  std::vector<std::string_view> claims;
  while (dr.next(&f, &w)) {
    std::string_view v;
    if (w == 2 && f == 4) {
      if (!dr.bytes(&v)) return false;
      claims.push_back(v);
    } else if (!dr.skip(w)) {
      return false;
    }
  }
  if (!dr.ok()) return false;
  for (std::string_view cb : claims) {
    PbReader c(cb);
    std::string driver, device, cdi;
    while (c.next(&f, &w)) {
      std::string_view v;
      if (w == 2 && (f == 1 || f == 2 || f == 4)) {
        if (!c.bytes(&v)) return false;
        if (f == 2) driver.assign(v);
        else if (f == 4) device.assign(v);
        else if (cdi.empty()) {  // CDIDevice{1 name}
          PbReader cd(v);
          uint32_t f2, w2;
          while (cd.next(&f2, &w2)) {
            std::string_view n;
            if (w2 == 2 && f2 == 1) {
              if (!cd.bytes(&n)) return false;
              cdi.assign(n);
            } else if (!cd.skip(w2)) {
              return false;
            }
          }
        }
      } else if (!c.skip(w)) {
        return false;
      }
    }
    if (!c.ok()) return false;
    if (std::find(drivers.begin(), drivers.end(), driver) == drivers.end()) continue;
    const std::string& id = device.empty() ? cdi : device;
    if (!id.empty()) out->push_back({ns, pod, cname, driver, id});
  }
  return true;
}

}  // namespace

// ListPodResourcesResponse{1: PodResources{1 name, 2 namespace, 3 ContainerResources{1 name,
// 2 ContainerDevices{1 resource_name, 2 device_ids}, 5 DynamicResource}}}  (k8s.io/kubelet
// podresources/v1 api.proto)
bool parse_list_pod_resources(std::string_view msg, const std::string& resource_prefix,
                              std::vector<PodDeviceRow>* out, const std::vector<std::string>& dra_drivers) {
  PbReader top(msg);
  uint32_t f, w;
  while (top.next(&f, &w)) {
    if (f != 1 || w != 2) {
      if (!top.skip(w)) return false;
      continue;
    }
    std::string_view pod_b;
    if (!top.bytes(&pod_b)) return false;
    std::string name, ns;
    std::vector<std::string_view> containers;
    PbReader pod(pod_b);
    while (pod.next(&f, &w)) {
      std::string_view v;
      if (w == 2 && (f == 1 || f == 2 || f == 3)) {
        if (!pod.bytes(&v)) return false;
        if (f == 1) name.assign(v);
        else if (f == 2) ns.assign(v);
        else containers.push_back(v);
      } else if (!pod.skip(w)) {
        return false;
      }
    }
    if (!pod.ok()) return false;
    for (std::string_view cb : containers) {
      PbReader c(cb);
      std::string cname;
      std::vector<std::string_view> devs, dyn;
      while (c.next(&f, &w)) {
        std::string_view v;
        if (w == 2 && (f == 1 || f == 2 || f == 5)) {
          if (!c.bytes(&v)) return false;
          if (f == 1) cname.assign(v);
          else if (f == 2) devs.push_back(v);
          else dyn.push_back(v);
        } else if (!c.skip(w)) {
          return false;
        }
      }
      if (!c.ok()) return false;
      for (std::string_view db : dyn)
        if (!dra_drivers.empty() && !parse_dynamic_resource(db, dra_drivers, ns, name, cname, out)) return false;
      for (std::string_view db : devs) {
        PbReader d(db);
        std::string res;
        std::vector<std::string> ids;
        while (d.next(&f, &w)) {
          std::string_view v;
          if (w == 2 && (f == 1 || f == 2)) {
            if (!d.bytes(&v)) return false;
            if (f == 1) res.assign(v);
            else ids.emplace_back(v);
          } else if (!d.skip(w)) {
            return false;
          }
        }
        if (!d.ok()) return false;
        if (!resource_prefix.empty() && res.rfind(resource_prefix, 0) != 0) continue;
        for (auto& id : ids) out->push_back({ns, name, cname, res, id});
      }
    }
  }
  return top.ok();
}

bool podresources_list(const std::string& socket_path, const std::string& resource_prefix,
                       std::vector<PodDeviceRow>* out, std::string* err, int timeout_ms,
                       const std::vector<std::string>& dra_drivers, GrpcStatus* status) {
  std::string resp;
  out->clear();
  if (!grpc_unary_unix(socket_path, "/v1.PodResourcesLister/List", "", &resp, err, timeout_ms, status)) return false;
  if (!parse_list_pod_resources(resp, resource_prefix, out, dra_drivers)) {
    *err = "malformed ListPodResourcesResponse";
    return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
namespace {

bool parse_map_entry(std::string_view b, std::map<std::string, std::string>* m) {
  PbReader r(b);
  uint32_t f, w;
  std::string k, v;
  while (r.next(&f, &w)) {
    std::string_view x;
    if (w == 2 && (f == 1 || f == 2)) {
      if (!r.bytes(&x)) return false;
      (f == 1 ? k : v).assign(x);
    } else if (!r.skip(w)) {
      return false;
    }
  }
  if (!r.ok()) return false;
  (*m)[k] = v;
  return true;
}

// name = field 1 of a nested metadata message (ContainerMetadata / PodSandboxMetadata); the
// sandbox metadata also carries uid (2) and namespace (3).
bool parse_metadata(std::string_view b, std::string* name, std::string* uid, std::string* ns) {
  PbReader r(b);
  uint32_t f, w;
  while (r.next(&f, &w)) {
    std::string_view x;
    if (w == 2 && f >= 1 && f <= 3) {
      if (!r.bytes(&x)) return false;
      if (f == 1) name->assign(x);
      else if (f == 2 && uid) uid->assign(x);
      else if (f == 3 && ns) ns->assign(x);
    } else if (!r.skip(w)) {
      return false;
    }
  }
  return r.ok();
}

}  // namespace

bool parse_cri_containers(std::string_view msg, std::vector<CriContainer>* out) {
  PbReader top(msg);
  uint32_t f, w;
  while (top.next(&f, &w)) {
    if (f != 1 || w != 2) {
      if (!top.skip(w)) return false;
      continue;
    }
    std::string_view cb;
    if (!top.bytes(&cb)) return false;
    CriContainer c;
    PbReader r(cb);
    while (r.next(&f, &w)) {
      std::string_view x;
      if (w != 2 || (f != 1 && f != 2 && f != 3 && f != 8 && f != 9)) {
        if (!r.skip(w)) return false;
        continue;
      }
      if (!r.bytes(&x)) return false;
      if (f == 1) c.id.assign(x);
      else if (f == 2) c.sandbox_id.assign(x);
      else if (f == 3 && !parse_metadata(x, &c.name, nullptr, nullptr)) return false;
      else if (f == 8 && !parse_map_entry(x, &c.labels)) return false;
      else if (f == 9 && !parse_map_entry(x, &c.annotations)) return false;
    }
    if (!r.ok()) return false;
    out->push_back(std::move(c));
  }
  return top.ok();
}

bool parse_cri_sandboxes(std::string_view msg, std::vector<CriSandbox>* out) {
  PbReader top(msg);
  uint32_t f, w;
  while (top.next(&f, &w)) {
    if (f != 1 || w != 2) {
      if (!top.skip(w)) return false;
      continue;
    }
    std::string_view sb;
    if (!top.bytes(&sb)) return false;
    CriSandbox s;
    PbReader r(sb);
    while (r.next(&f, &w)) {
      std::string_view x;
      if (w != 2 || (f != 1 && f != 2 && f != 5 && f != 6)) {
        if (!r.skip(w)) return false;
        continue;
      }
      if (!r.bytes(&x)) return false;
      if (f == 1) s.id.assign(x);
      else if (f == 2 && !parse_metadata(x, &s.name, &s.uid, &s.pod_namespace)) return false;
      else if (f == 5 && !parse_map_entry(x, &s.labels)) return false;
      else if (f == 6 && !parse_map_entry(x, &s.annotations)) return false;
    }
    if (!r.ok()) return false;
    out->push_back(std::move(s));
  }
  return top.ok();
}

bool cri_list(const std::string& socket_path, std::vector<CriContainer>* containers, std::vector<CriSandbox>* sandboxes,
              std::string* err, int timeout_ms, GrpcStatus* status) {
  containers->clear();
  sandboxes->clear();
  // runtime.v1 first; a runtime that answers UNIMPLEMENTED (containerd < 1.7, older cri-o) speaks
  // runtime.v1alpha2, whose List* messages are wire-identical. The version that worked is remembered
  // per socket.
  static std::mutex mu;
  static std::map<std::string, std::string> api_of;
  std::string api;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = api_of.find(socket_path);
    api = it == api_of.end() ? "runtime.v1" : it->second;
  }
  GrpcStatus local;
  GrpcStatus& st = status ? *status : local;
  std::string resp;
  if (!grpc_unary_unix(socket_path, "/" + api + ".RuntimeService/ListContainers", "", &resp, err, timeout_ms, &st)) {
    if (st.code != 12 || api != "runtime.v1") return false;
    api = "runtime.v1alpha2";
    if (!grpc_unary_unix(socket_path, "/" + api + ".RuntimeService/ListContainers", "", &resp, err, timeout_ms, &st))
      return false;
  }
  {
    std::lock_guard<std::mutex> g(mu);
    api_of[socket_path] = api;
  }
  if (!parse_cri_containers(resp, containers)) {
    *err = "malformed ListContainersResponse";
    return false;
  }
  if (!grpc_unary_unix(socket_path, "/" + api + ".RuntimeService/ListPodSandbox", "", &resp, err, timeout_ms, &st))
    return false;
  if (!parse_cri_sandboxes(resp, sandboxes)) {
    *err = "malformed ListPodSandboxResponse";
    return false;
  }
  return true;
}

}  // namespace gpumon

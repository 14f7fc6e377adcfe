#include "tls.h"

#include <arpa/inet.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/stat.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <initializer_list>
#include <mutex>

#include "common.h"
#include "http_client.h"

namespace gpumon {

// OpenSSL 3 ABI pieces used here (stable since 1.1.0; declared locally so no openssl headers are
// needed to build): opaque handles as void*, and the constant values of ssl.h / prov_ssl.h.
namespace ossl {
constexpr int kVerifyNone = 0, kVerifyPeer = 1;
constexpr int kCtrlSetTlsextHostname = 55, kTlsextNametypeHostName = 0;
constexpr int kCtrlSetMinProtoVersion = 123, kTls12Version = 0x0303;
constexpr int kFiletypePem = 1;
constexpr int kVerifyFailIfNoPeerCert = 2;
constexpr int kCtrlMode = 33, kCtrlSetSessCacheMode = 44;
constexpr long kModeEnablePartialWrite = 0x1, kModeAcceptMovingWriteBuffer = 0x2, kSessCacheOff = 0;
constexpr uint64_t kOpNoRenegotiation = 0x40000000U;
constexpr int kErrorNone = 0, kErrorSsl = 1, kErrorWantRead = 2, kErrorWantWrite = 3, kErrorSyscall = 5,
              kErrorZeroReturn = 6;
constexpr long kVerifyOk = 0;
constexpr uint64_t kInitLoadSslStrings = 0x00200000L, kInitLoadCryptoStrings = 0x00000002L;
}  // namespace ossl

struct SslApi {
  void* ssl_dl = nullptr;
  void* crypto_dl = nullptr;
  // libssl
  int (*OPENSSL_init_ssl)(uint64_t, const void*) = nullptr;
  const void* (*TLS_client_method)() = nullptr;
  const void* (*TLS_server_method)() = nullptr;
  int (*SSL_CTX_set_session_id_context)(void*, const unsigned char*, unsigned int) = nullptr;
  int (*SSL_CTX_set_num_tickets)(void*, size_t) = nullptr;
  uint64_t (*SSL_CTX_set_options)(void*, uint64_t) = nullptr;
  void (*SSL_set_accept_state)(void*) = nullptr;
  int (*SSL_do_handshake)(void*) = nullptr;
  void* (*SSL_CTX_get0_certificate)(const void*) = nullptr;
  const void* (*X509_get0_notAfter)(const void*) = nullptr;
  int (*ASN1_TIME_to_tm)(const void*, struct tm*) = nullptr;
  void* (*SSL_CTX_new)(const void*) = nullptr;
  void (*SSL_CTX_free)(void*) = nullptr;
  long (*SSL_CTX_ctrl)(void*, int, long, void*) = nullptr;
  void (*SSL_CTX_set_verify)(void*, int, void*) = nullptr;
  int (*SSL_CTX_set_default_verify_paths)(void*) = nullptr;
  int (*SSL_CTX_load_verify_locations)(void*, const char*, const char*) = nullptr;
  int (*SSL_CTX_use_certificate_chain_file)(void*, const char*) = nullptr;
  int (*SSL_CTX_use_PrivateKey_file)(void*, const char*, int) = nullptr;
  int (*SSL_CTX_check_private_key)(const void*) = nullptr;
  void* (*SSL_CTX_get_cert_store)(const void*) = nullptr;
  void* (*SSL_new)(void*) = nullptr;
  void (*SSL_free)(void*) = nullptr;
  int (*SSL_set_fd)(void*, int) = nullptr;
  long (*SSL_ctrl)(void*, int, long, void*) = nullptr;
  int (*SSL_set1_host)(void*, const char*) = nullptr;
  void* (*SSL_get0_param)(void*) = nullptr;
  int (*SSL_connect)(void*) = nullptr;
  int (*SSL_read)(void*, void*, int) = nullptr;
  int (*SSL_write)(void*, const void*, int) = nullptr;
  int (*SSL_shutdown)(void*) = nullptr;
  int (*SSL_get_error)(const void*, int) = nullptr;
  long (*SSL_get_verify_result)(const void*) = nullptr;
  void* (*SSL_get0_peer_certificate)(const void*) = nullptr;
  // libcrypto
  int (*X509_VERIFY_PARAM_set1_ip_asc)(void*, const char*) = nullptr;
  const char* (*X509_verify_cert_error_string)(long) = nullptr;
  void* (*X509_STORE_get0_objects)(const void*) = nullptr;
  int (*OPENSSL_sk_num)(const void*) = nullptr;
  unsigned long (*ERR_get_error)() = nullptr;
  void (*ERR_error_string_n)(unsigned long, char*, size_t) = nullptr;
  void (*ERR_clear_error)() = nullptr;
};

namespace {

std::once_flag g_once;
SslApi* g_api = nullptr;
std::string g_err;

template <class T>
bool sym(void* dl, const char* name, T* out, std::string* missing) {
  *out = reinterpret_cast<T>(dlsym(dl, name));
  if (!*out) *missing += std::string(missing->empty() ? "" : ", ") + name;
  return *out != nullptr;
}

void load_api() {
  const char* ssl_env = getenv("GPUMON_LIBSSL");
  const char* crypto_env = getenv("GPUMON_LIBCRYPTO");
  auto* a = new SslApi;
  // An override is the only name tried: a wrong path must fail, not quietly load the default.
  // libcrypto first, RTLD_GLOBAL: libssl resolves its own libcrypto dependency to the same object.
  auto open_first = [](const char* env, std::initializer_list<const char*> names, int flags) -> void* {
    if (env && *env) return dlopen(env, flags);
    for (const char* n : names)
      if (void* h = dlopen(n, flags)) return h;
    return nullptr;
  };
  a->crypto_dl = open_first(crypto_env, {"libcrypto.so.3", "libcrypto.so"}, RTLD_NOW | RTLD_GLOBAL);
  const char* why = a->crypto_dl ? nullptr : dlerror();
  if (a->crypto_dl) {
    a->ssl_dl = open_first(ssl_env, {"libssl.so.3", "libssl.so"}, RTLD_NOW | RTLD_LOCAL);
    if (!a->ssl_dl) why = dlerror();
  }
  if (!a->ssl_dl || !a->crypto_dl) {
    g_err = std::string("https needs OpenSSL 3 (libssl.so.3 / libcrypto.so.3): ") + (why ? why : "not found");
    if (a->ssl_dl) dlclose(a->ssl_dl);
    if (a->crypto_dl) dlclose(a->crypto_dl);
    delete a;
    return;
  }
  std::string missing;
  void* s = a->ssl_dl;
  void* c = a->crypto_dl;
  sym(s, "OPENSSL_init_ssl", &a->OPENSSL_init_ssl, &missing);
  sym(s, "TLS_client_method", &a->TLS_client_method, &missing);
  sym(s, "TLS_server_method", &a->TLS_server_method, &missing);
  sym(s, "SSL_CTX_set_session_id_context", &a->SSL_CTX_set_session_id_context, &missing);
  sym(s, "SSL_CTX_set_num_tickets", &a->SSL_CTX_set_num_tickets, &missing);
  sym(s, "SSL_CTX_set_options", &a->SSL_CTX_set_options, &missing);
  sym(s, "SSL_set_accept_state", &a->SSL_set_accept_state, &missing);
  sym(s, "SSL_do_handshake", &a->SSL_do_handshake, &missing);
  sym(s, "SSL_CTX_get0_certificate", &a->SSL_CTX_get0_certificate, &missing);
  sym(c, "X509_get0_notAfter", &a->X509_get0_notAfter, &missing);
  sym(c, "ASN1_TIME_to_tm", &a->ASN1_TIME_to_tm, &missing);
  sym(s, "SSL_CTX_new", &a->SSL_CTX_new, &missing);
  sym(s, "SSL_CTX_free", &a->SSL_CTX_free, &missing);
  sym(s, "SSL_CTX_ctrl", &a->SSL_CTX_ctrl, &missing);
  sym(s, "SSL_CTX_set_verify", &a->SSL_CTX_set_verify, &missing);
  sym(s, "SSL_CTX_set_default_verify_paths", &a->SSL_CTX_set_default_verify_paths, &missing);
  sym(s, "SSL_CTX_load_verify_locations", &a->SSL_CTX_load_verify_locations, &missing);
  sym(s, "SSL_CTX_use_certificate_chain_file", &a->SSL_CTX_use_certificate_chain_file, &missing);
  sym(s, "SSL_CTX_use_PrivateKey_file", &a->SSL_CTX_use_PrivateKey_file, &missing);
  sym(s, "SSL_CTX_check_private_key", &a->SSL_CTX_check_private_key, &missing);
  sym(s, "SSL_CTX_get_cert_store", &a->SSL_CTX_get_cert_store, &missing);
  sym(s, "SSL_new", &a->SSL_new, &missing);
  sym(s, "SSL_free", &a->SSL_free, &missing);
  sym(s, "SSL_set_fd", &a->SSL_set_fd, &missing);
  sym(s, "SSL_ctrl", &a->SSL_ctrl, &missing);
  sym(s, "SSL_set1_host", &a->SSL_set1_host, &missing);
  sym(s, "SSL_get0_param", &a->SSL_get0_param, &missing);
  sym(s, "SSL_connect", &a->SSL_connect, &missing);
  sym(s, "SSL_read", &a->SSL_read, &missing);
  sym(s, "SSL_write", &a->SSL_write, &missing);
  sym(s, "SSL_shutdown", &a->SSL_shutdown, &missing);
  sym(s, "SSL_get_error", &a->SSL_get_error, &missing);
  sym(s, "SSL_get_verify_result", &a->SSL_get_verify_result, &missing);
  sym(s, "SSL_get0_peer_certificate", &a->SSL_get0_peer_certificate, &missing);
  sym(c, "X509_VERIFY_PARAM_set1_ip_asc", &a->X509_VERIFY_PARAM_set1_ip_asc, &missing);
  sym(c, "X509_verify_cert_error_string", &a->X509_verify_cert_error_string, &missing);
  sym(c, "X509_STORE_get0_objects", &a->X509_STORE_get0_objects, &missing);
  sym(c, "OPENSSL_sk_num", &a->OPENSSL_sk_num, &missing);
  sym(c, "ERR_get_error", &a->ERR_get_error, &missing);
  sym(c, "ERR_error_string_n", &a->ERR_error_string_n, &missing);
  sym(c, "ERR_clear_error", &a->ERR_clear_error, &missing);
  if (!missing.empty()) {
    g_err = "libssl / libcrypto lack " + missing + " (OpenSSL >= 3 required)";
    dlclose(a->ssl_dl);
    dlclose(a->crypto_dl);
    delete a;
    return;
  }
  a->OPENSSL_init_ssl(ossl::kInitLoadSslStrings | ossl::kInitLoadCryptoStrings, nullptr);
  g_api = a;  // never unloaded: OpenSSL keeps process-wide state
}

std::string err_queue(const SslApi* a) {
  std::string out;
  for (unsigned long e; (e = a->ERR_get_error()) != 0;) {
    char buf[256];
    a->ERR_error_string_n(e, buf, sizeof buf);
    out = buf;  // the last (outermost) entry names the failing operation best
  }
  return out;
}

bool is_ip_literal(const std::string& h) {
  unsigned char b[16];
  return inet_pton(AF_INET, h.c_str(), b) == 1 || inet_pton(AF_INET6, h.c_str(), b) == 1;
}

// Bundles where distributions keep the CA set, for when libssl's compiled-in OPENSSLDIR holds none
// (a slim image that copies the bundle but not the hashed certs/ directory).
const char* const kBundles[] = {"/etc/ssl/certs/ca-certificates.crt", "/etc/pki/tls/certs/ca-bundle.crt",
                                "/etc/ssl/ca-bundle.pem", "/etc/ssl/cert.pem"};

}  // namespace

const SslApi* ssl_api(std::string* err) {
  std::call_once(g_once, load_api);
  if (!g_api && err) *err = g_err;
  return g_api;
}

std::shared_ptr<TlsContext> TlsContext::create(const TlsOptions& o, std::string* err) {
  const SslApi* a = ssl_api(err);
  if (!a) return nullptr;
  std::shared_ptr<TlsContext> t(new TlsContext);
  t->api_ = a;
  t->insecure_ = o.insecure;
  a->ERR_clear_error();
  t->ctx_ = a->SSL_CTX_new(a->TLS_client_method());
  if (!t->ctx_) {
    *err = "tls: SSL_CTX_new: " + err_queue(a);
    return nullptr;
  }
  a->SSL_CTX_ctrl(t->ctx_, ossl::kCtrlSetMinProtoVersion, ossl::kTls12Version, nullptr);
  if (!o.insecure) {
    if (!o.ca_file.empty()) {
      if (a->SSL_CTX_load_verify_locations(t->ctx_, o.ca_file.c_str(), nullptr) != 1) {
        *err = "tls: cannot load CA file " + o.ca_file + ": " + err_queue(a);
        return nullptr;
      }
    } else {
      a->SSL_CTX_set_default_verify_paths(t->ctx_);
      a->ERR_clear_error();  // a missing default directory is not an error by itself
      const void* objs = a->X509_STORE_get0_objects(a->SSL_CTX_get_cert_store(t->ctx_));
      if (!objs || a->OPENSSL_sk_num(objs) <= 0) {
        // the default file held nothing (SSL_CERT_FILE unset, OPENSSLDIR empty): the usual bundles
        for (const char* b : kBundles)
          if (access(b, R_OK) == 0 && a->SSL_CTX_load_verify_locations(t->ctx_, b, nullptr) == 1) break;
        a->ERR_clear_error();
        const void* again = a->X509_STORE_get0_objects(a->SSL_CTX_get_cert_store(t->ctx_));
        // a hashed certs/ directory (SSL_CERT_DIR / OPENSSLDIR) is only read on demand and counts 0
        // here: refuse only when no bundle file and no such directory can be found either
        const char* dir_env = getenv("SSL_CERT_DIR");
        const bool have_dir = (dir_env && *dir_env && access(dir_env, R_OK) == 0) || access("/etc/ssl/certs", R_OK) == 0;
        if ((!again || a->OPENSSL_sk_num(again) <= 0) && !have_dir) {
          *err = "tls: no CA certificates found (no system bundle): set influx_ca_file";
          return nullptr;
        }
      }
    }
  }
  a->SSL_CTX_set_verify(t->ctx_, o.insecure ? ossl::kVerifyNone : ossl::kVerifyPeer, nullptr);
  if (!o.client_cert.empty() || !o.client_key.empty()) {
    const std::string& key = o.client_key.empty() ? o.client_cert : o.client_key;
    if (a->SSL_CTX_use_certificate_chain_file(t->ctx_, o.client_cert.c_str()) != 1) {
      *err = "tls: cannot load client certificate " + o.client_cert + ": " + err_queue(a);
      return nullptr;
    }
    if (a->SSL_CTX_use_PrivateKey_file(t->ctx_, key.c_str(), ossl::kFiletypePem) != 1 ||
        a->SSL_CTX_check_private_key(t->ctx_) != 1) {
      *err = "tls: cannot load client key " + key + ": " + err_queue(a);
      return nullptr;
    }
  }
  return t;
}

TlsContext::~TlsContext() {
  if (ctx_) api_->SSL_CTX_free(ctx_);
}

TlsConn::~TlsConn() {
  if (ssl_) ctx_->api()->SSL_free(ssl_);
}

std::string TlsConn::last_error(int ret) {
  const SslApi* a = ctx_->api();
  const int e = a->SSL_get_error(ssl_, ret);
  const int saved_errno = errno;
  std::string q = err_queue(a);
  switch (e) {
    case ossl::kErrorZeroReturn:
      return "tls: connection closed by peer";
    case ossl::kErrorWantRead:
    case ossl::kErrorWantWrite:
      return "tls: timed out";
    case ossl::kErrorSyscall:
      if (!q.empty()) return "tls: " + q;
      if (saved_errno == EAGAIN || saved_errno == EWOULDBLOCK) return "tls: timed out";
      return saved_errno ? std::string("tls: ") + strerror(saved_errno) : "tls: unexpected EOF";
    default:
      return "tls: " + (q.empty() ? "error " + std::to_string(e) : q);
  }
}

bool TlsConn::wait_retry(int ret, int64_t deadline, std::string* err) {
  const SslApi* a = ctx_->api();
  const int e = a->SSL_get_error(ssl_, ret);
  short ev;
  if (e == ossl::kErrorWantRead) ev = POLLIN;
  else if (e == ossl::kErrorWantWrite) ev = POLLOUT;
  else {
    *err = last_error(ret);
    return false;
  }
  for (;;) {
    const int64_t left = deadline - mono_ns();
    if (left <= 0) {
      *err = "tls: timed out";
      return false;
    }
    pollfd p{fd_, ev, 0};
    const int r = poll(&p, 1, static_cast<int>(std::min<int64_t>(left / 1000000 + 1, 60000)));
    if (r > 0) return true;  // ready (or an error condition the retried call will report)
    if (r < 0 && errno != EINTR) {
      *err = std::string("tls: poll: ") + strerror(errno);
      return false;
    }
  }
}

bool TlsConn::handshake(int fd, const std::string& host, std::string* err) {
  const SslApi* a = ctx_->api();
  a->ERR_clear_error();
  fd_ = fd;
  const int fl = fcntl(fd, F_GETFL, 0);
  if (fl < 0 || fcntl(fd, F_SETFL, fl | O_NONBLOCK) != 0) {
    *err = std::string("tls: fcntl: ") + strerror(errno);
    return false;
  }
  ssl_ = a->SSL_new(ctx_->raw());
  if (!ssl_ || a->SSL_set_fd(ssl_, fd) != 1) {
    *err = "tls: SSL_new: " + err_queue(a);
    return false;
  }
  const bool ip = is_ip_literal(host);
  // RFC 6066: no SNI for IP literals
  if (!ip) a->SSL_ctrl(ssl_, ossl::kCtrlSetTlsextHostname, ossl::kTlsextNametypeHostName, const_cast<char*>(host.c_str()));
  if (ctx_->verify()) {
    const int ok = ip ? a->X509_VERIFY_PARAM_set1_ip_asc(a->SSL_get0_param(ssl_), host.c_str())
                      : a->SSL_set1_host(ssl_, host.c_str());
    if (ok != 1) {
      *err = "tls: cannot set the expected peer name " + host;
      return false;
    }
  }
  const int64_t deadline = mono_ns() + timeout_ns_;
  int r;
  std::string werr;
  while ((r = a->SSL_connect(ssl_)) != 1) {
    const int e = a->SSL_get_error(ssl_, r);
    if ((e == ossl::kErrorWantRead || e == ossl::kErrorWantWrite) && wait_retry(r, deadline, &werr)) continue;
    break;
  }
  if (r != 1) {
    if (werr == "tls: timed out") {
      *err = "tls: handshake with " + host + " timed out";
      return false;
    }
    const long v = a->SSL_get_verify_result(ssl_);
    if (ctx_->verify() && v != ossl::kVerifyOk) {
      a->ERR_clear_error();
      *err = std::string("tls: certificate verify failed: ") + a->X509_verify_cert_error_string(v);
    } else {
      *err = last_error(r);
      if (err->find("handshake") == std::string::npos) *err += " (handshake with " + host + ")";
    }
    return false;
  }
  return true;
}

bool TlsConn::write_all(const char* p, size_t n, std::string* err) {
  const SslApi* a = ctx_->api();
  const int64_t deadline = mono_ns() + timeout_ns_;
  while (n) {
    const int chunk = static_cast<int>(std::min<size_t>(n, 1 << 30));
    a->ERR_clear_error();
    const int w = a->SSL_write(ssl_, p, chunk);
    if (w <= 0) {
      if (wait_retry(w, deadline, err)) continue;
      return false;
    }
    p += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

long TlsConn::read_some(char* buf, size_t n, std::string* err) {
  const SslApi* a = ctx_->api();
  const int64_t deadline = mono_ns() + timeout_ns_;
  for (;;) {
    a->ERR_clear_error();
    errno = 0;
    const int r = a->SSL_read(ssl_, buf, static_cast<int>(std::min<size_t>(n, 1 << 30)));
    if (r > 0) return r;
    const int e = a->SSL_get_error(ssl_, r);
    if (e == ossl::kErrorZeroReturn) return 0;
    // EOF without close_notify: many servers (and proxies) just close; the HTTP framing decides
    if (e == ossl::kErrorSyscall && errno == 0 && a->ERR_get_error() == 0) return 0;
    std::string werr;
    if ((e == ossl::kErrorWantRead || e == ossl::kErrorWantWrite) && wait_retry(r, deadline, &werr)) continue;
    *err = werr.empty() ? last_error(r) : werr;
    return -1;
  }
}

void TlsConn::shutdown() {
  if (ssl_) {
    ctx_->api()->SSL_shutdown(ssl_);  // non-blocking: one attempt to send close_notify
    ctx_->api()->ERR_clear_error();
  }
}

namespace {

// One server context from the files (nullptr with *err); *not_after = the leaf certificate's expiry.
void* build_server_ctx(const SslApi* a, const std::string& cert_file, const std::string& key_file,
                       const std::string& client_ca_file, int64_t* not_after, std::string* err) {
  for (const std::string* f : {&cert_file, &key_file, &client_ca_file})
    if (!f->empty() && access(f->c_str(), R_OK) != 0) {
      *err = "cannot read " + *f + ": " + strerror(errno);
      return nullptr;
    }
  a->ERR_clear_error();
  void* ctx = a->SSL_CTX_new(a->TLS_server_method());
  if (!ctx) {
    *err = "tls: SSL_CTX_new: " + err_queue(a);
    return nullptr;
  }
  auto fail = [&](std::string why) -> void* {
    *err = std::move(why);
    a->SSL_CTX_free(ctx);
    return nullptr;
  };
  a->SSL_CTX_ctrl(ctx, ossl::kCtrlSetMinProtoVersion, ossl::kTls12Version, nullptr);
  // partial writes: a response larger than the socket buffer goes out record by record, resumed
  // from the loop's offset on the next EPOLLOUT
  a->SSL_CTX_ctrl(ctx, ossl::kCtrlMode, ossl::kModeEnablePartialWrite | ossl::kModeAcceptMovingWriteBuffer, nullptr);
  a->SSL_CTX_ctrl(ctx, ossl::kCtrlSetSessCacheMode, ossl::kSessCacheOff, nullptr);
  a->SSL_CTX_set_num_tickets(ctx, 0);
  // no TLS 1.2 renegotiation: a write would then wait for the peer's records (WANT_READ) while the
  // loop waits for EPOLLOUT -- a scraper has no reason to renegotiate
  a->SSL_CTX_set_options(ctx, ossl::kOpNoRenegotiation);
  static const unsigned char kSid[] = "gpumon";
  a->SSL_CTX_set_session_id_context(ctx, kSid, sizeof kSid - 1);
  if (a->SSL_CTX_use_certificate_chain_file(ctx, cert_file.c_str()) != 1)
    return fail("tls: cannot load certificate " + cert_file + ": " + err_queue(a));
  if (a->SSL_CTX_use_PrivateKey_file(ctx, key_file.c_str(), ossl::kFiletypePem) != 1 ||
      a->SSL_CTX_check_private_key(ctx) != 1)
    return fail("tls: cannot load key " + key_file + " (or it does not match the certificate): " + err_queue(a));
  if (!client_ca_file.empty()) {
    if (a->SSL_CTX_load_verify_locations(ctx, client_ca_file.c_str(), nullptr) != 1)
      return fail("tls: cannot load client CA " + client_ca_file + ": " + err_queue(a));
    // REQUEST a client certificate and verify one that is sent (a wrong CA still fails the
    // handshake), but do not REQUIRE one: the kubelet's HTTPS probes present none, and /healthz /
    // /readyz must answer them. /metrics itself needs a verified certificate (peer_verified(),
    // checked per request in Exporter::handle_http: 403 without one). ADVICE r5: with
    // FAIL_IF_NO_PEER_CERT every probe failed at the handshake and restarted the pod.
    a->SSL_CTX_set_verify(ctx, ossl::kVerifyPeer, nullptr);
  }
  *not_after = 0;
  if (const void* x = a->SSL_CTX_get0_certificate(ctx)) {
    struct tm t {};
    if (const void* na = a->X509_get0_notAfter(x); na && a->ASN1_TIME_to_tm(na, &t) == 1) *not_after = timegm(&t);
  }
  a->ERR_clear_error();
  return ctx;
}

}  // namespace

int64_t tls_reload_period_ns(int64_t dflt_ns) {
  const char* e = getenv("GPUMON_TLS_RELOAD_S");
  return e && *e ? static_cast<int64_t>(std::max(0.1, atof(e)) * 1e9) : dflt_ns;
}

FileStamp FileStamp::of(const std::string& path) {
  FileStamp s;
  struct stat st {};
  if (path.empty() || ::stat(path.c_str(), &st) != 0) return s;  // follows the kubelet's ..data symlink
  s.mtime_ns = static_cast<int64_t>(st.st_mtim.tv_sec) * 1000000000LL + st.st_mtim.tv_nsec;
  s.size = static_cast<int64_t>(st.st_size);
  s.ino = static_cast<uint64_t>(st.st_ino);
  return s;
}

std::shared_ptr<TlsServer> TlsServer::create(const std::string& cert_file, const std::string& key_file,
                                             const std::string& client_ca_file, std::string* err) {
  if (cert_file.empty() && key_file.empty() && !client_ca_file.empty()) {
    *err = "tls_client_ca_file needs tls_cert_file and tls_key_file";
    return nullptr;
  }
  if (cert_file.empty() || key_file.empty()) {
    *err = "tls_cert_file and tls_key_file go together";
    return nullptr;
  }
  const SslApi* a = ssl_api(err);
  if (!a) return nullptr;
  std::shared_ptr<TlsServer> t(new TlsServer);
  t->api_ = a;
  t->cert_ = cert_file;
  t->key_ = key_file;
  t->ca_ = client_ca_file;
  // stamped before the load: a rotation while it loads is seen as a change next time
  t->stamps_[0] = FileStamp::of(cert_file);
  t->stamps_[1] = FileStamp::of(key_file);
  t->stamps_[2] = FileStamp::of(client_ca_file);
  int64_t na = 0;
  t->ctx_ = build_server_ctx(a, cert_file, key_file, client_ca_file, &na, err);
  if (!t->ctx_) return nullptr;
  t->not_after_ = na;
  t->next_check_ns_ = mono_ns() + tls_reload_period_ns(5'000'000'000LL);  // just loaded
  return t;
}

void TlsServer::maybe_reload(int64_t now_ns) {
  if (now_ns < next_check_ns_ && !reload_now_.exchange(false)) return;
  next_check_ns_ = now_ns + tls_reload_period_ns(5'000'000'000LL);
  const FileStamp now[3] = {FileStamp::of(cert_), FileStamp::of(key_), FileStamp::of(ca_)};
  if (now[0] == stamps_[0] && now[1] == stamps_[1] && now[2] == stamps_[2]) return;
  for (int i = 0; i < 3; ++i) stamps_[i] = now[i];  // a broken change is retried on the next change only
  std::string err;
  int64_t na = 0;
  void* fresh = build_server_ctx(api_, cert_, key_, ca_, &na, &err);
  if (!fresh) {
    reloads_failed_.fetch_add(1);
    GPUMON_LOG(LogLevel::kWarn, "http", "TLS files changed but do not load (keeping the previous certificate): " + err);
    return;
  }
  void* old;
  {
    std::lock_guard<std::mutex> g(mu_);
    old = ctx_;
    ctx_ = fresh;
  }
  api_->SSL_CTX_free(old);  // sessions made from it hold their own reference
  not_after_ = na;
  reloads_ok_.fetch_add(1);
  GPUMON_LOG(LogLevel::kInfo, "http", "reloaded the TLS certificate " + cert_);
}

TlsServer::~TlsServer() {
  if (ctx_) api_->SSL_CTX_free(ctx_);
}

bool TlsServer::peer_verified(void* ssl) const {
  return ssl && api_->SSL_get0_peer_certificate(ssl) != nullptr && api_->SSL_get_verify_result(ssl) == ossl::kVerifyOk;
}

void* TlsServer::new_session(int fd) const {
  void* ssl;
  {
    std::lock_guard<std::mutex> g(mu_);
    ssl = api_->SSL_new(ctx_);
  }
  if (!ssl) return nullptr;
  if (api_->SSL_set_fd(ssl, fd) != 1) {
    api_->SSL_free(ssl);
    return nullptr;
  }
  api_->SSL_set_accept_state(ssl);
  return ssl;
}

TlsServer::Step TlsServer::handshake(void* ssl) const {
  api_->ERR_clear_error();
  const int r = api_->SSL_do_handshake(ssl);
  if (r == 1) return Step::kDone;
  const int e = api_->SSL_get_error(ssl, r);
  if (e == ossl::kErrorWantRead) return Step::kWantRead;
  if (e == ossl::kErrorWantWrite) return Step::kWantWrite;
  api_->ERR_clear_error();
  return Step::kFailed;
}

long TlsServer::read(void* ssl, char* buf, size_t n) const {
  api_->ERR_clear_error();
  const int r = api_->SSL_read(ssl, buf, static_cast<int>(std::min<size_t>(n, 1 << 30)));
  if (r > 0) return r;
  const int e = api_->SSL_get_error(ssl, r);
  if (e == ossl::kErrorWantRead || e == ossl::kErrorWantWrite) return -1;
  api_->ERR_clear_error();
  // close_notify, or a peer that just closed the TCP connection: both end the connection
  return e == ossl::kErrorZeroReturn || e == ossl::kErrorSyscall ? 0 : -2;
}

long TlsServer::write(void* ssl, const char* p, size_t n) const {
  api_->ERR_clear_error();
  const int w = api_->SSL_write(ssl, p, static_cast<int>(std::min<size_t>(n, 1 << 30)));
  if (w > 0) return w;
  const int e = api_->SSL_get_error(ssl, w);
  if (e == ossl::kErrorWantWrite || e == ossl::kErrorWantRead) return -1;
  api_->ERR_clear_error();
  return -2;
}

void TlsServer::notify_close(void* ssl) const {
  api_->SSL_shutdown(ssl);
  api_->ERR_clear_error();
}

void TlsServer::free_session(void* ssl) const { api_->SSL_free(ssl); }

std::string check_serve_tls(const std::string& cert_file, const std::string& key_file,
                            const std::string& client_ca_file) {
  if (cert_file.empty() && key_file.empty() && client_ca_file.empty()) return "";
  std::string err;
  return TlsServer::create(cert_file, key_file, client_ca_file, &err) ? "" : err;
}

std::string check_push_config(const std::string& url, const std::string& token, const TlsOptions& tls) {
  if (url.empty()) return "";
  const Url u = parse_url(url);
  if (!u.ok) return "influx_url " + redact_url(url) + ": " + (u.error.empty() ? "not a usable URL" : u.error);
  if (token.find_first_of("\r\n") != std::string::npos) return "influx_token contains a line break";
  if (!u.tls) {
    if (!tls.ca_file.empty() || !tls.client_cert.empty() || tls.insecure)
      GPUMON_LOG(LogLevel::kWarn, "influx", "TLS settings given for an http:// INFLUXDB_URL: ignored");
    return "";
  }
  for (const std::string* f : {&tls.ca_file, &tls.client_cert, &tls.client_key})
    if (!f->empty() && access(f->c_str(), R_OK) != 0) return "cannot read " + *f + ": " + strerror(errno);
  std::string err;
  if (!TlsContext::create(tls, &err)) return err;
  return "";
}

}  // namespace gpumon

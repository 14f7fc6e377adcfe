// The exporter's HTTP endpoints: /metrics (snapshot, gzip, per-request family filters), /healthz,
// /livez, /readyz and the index page. Runs on the HTTP loop threads (http_server.cpp).
#include "exporter_internal.h"

#include <cctype>
#include <cstdlib>

#include "common.h"

namespace gpumon {

namespace {

std::string url_decode(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '+') {
      o.push_back(' ');
    } else if (s[i] == '%' && i + 2 < s.size() && isxdigit(static_cast<unsigned char>(s[i + 1])) &&
               isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      o.push_back(static_cast<char>(std::stoi(s.substr(i + 1, 2), nullptr, 16)));
      i += 2;
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

// Bounds on a per-request filter: the globs come from any client that can reach the port, and a
// filter runs on an HTTP loop thread. Matching is O(glob x name) (glob_match), so these keep one
// request's work to ~32 globs x 128 chars x ~150 family names.
constexpr size_t kMaxFilterQuery = 8192, kMaxFilterGlobs = 32, kMaxGlobLen = 128;

// include=a,b&exclude=c (each repeatable): the family globs of a per-request filter.
// 1 = a filter, 0 = no filter keys, -1 = over the bounds above (*err says which).
int parse_filter_query(const std::string& q, std::vector<std::string>* inc, std::vector<std::string>* exc,
                       std::string* err) {
  if (q.size() > kMaxFilterQuery) {
    *err = "query longer than " + std::to_string(kMaxFilterQuery) + " bytes";
    return -1;
  }
  bool any = false;
  for (const auto& kv : split(q, '&')) {
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    const std::string k = url_decode(kv.substr(0, eq));
    std::vector<std::string>* dst = k == "include" ? inc : k == "exclude" ? exc : nullptr;
    if (!dst) continue;
    any = true;
    for (const auto& g : split(url_decode(kv.substr(eq + 1)), ',')) {
      if (g.empty()) continue;
      if (g.size() > kMaxGlobLen) {
        *err = "glob longer than " + std::to_string(kMaxGlobLen) + " bytes";
        return -1;
      }
      dst->push_back(g);
      if (inc->size() + exc->size() > kMaxFilterGlobs) {
        *err = "more than " + std::to_string(kMaxFilterGlobs) + " globs";
        return -1;
      }
    }
  }
  return any ? 1 : 0;
}

}  // namespace

std::shared_ptr<const Exporter::Filtered> Exporter::filtered(const Snapshot& s, const std::string& query, bool gzip) {
  {
    std::lock_guard<std::mutex> g(filter_mu_);
    if (filter_seq_ != s.seq) {
      filter_cache_.clear();
      filter_seq_ = s.seq;
    }
    auto it = filter_cache_.find(query);
    if (it != filter_cache_.end() && (!gzip || !it->second->body_gz.empty())) return it->second;
  }
  std::vector<std::string> inc, exc;
  std::string err;
  parse_filter_query(query, &inc, &exc, &err);  // handle_http validated it
  auto f = std::make_shared<Filtered>();
  filter_exposition(s.body, inc, exc, &f->body);
  if (gzip) gzip_compress(f->body, &f->body_gz, 1);
  std::lock_guard<std::mutex> g(filter_mu_);
  if (filter_seq_ == s.seq && (filter_cache_.size() < kFilterCache || filter_cache_.count(query)))
    filter_cache_[query] = f;
  return f;
}

void Exporter::handle_http(const HttpRequest& req, HttpResponse* resp) {
  if (req.path == "/metrics") {
    if (!req.client_cert && server_ && server_->tls_server() && server_->tls_server()->mutual()) {
      // mutual TLS: the handshake asks for a client certificate without requiring one (so the
      // kubelet's HTTPS probes reach /healthz and /readyz); the metrics need one that verified
      mtls_refused_.fetch_add(1, std::memory_order_relaxed);
      resp->status = 403;
      resp->inline_body = "client certificate required\n";
      return;
    }
    if (const auto v = auth_ ? auth_->check(req.authorization) : TokenAuth::Verdict::kOk; v != TokenAuth::Verdict::kOk) {
      auth_failures_[static_cast<int>(v) - 1].fetch_add(1, std::memory_order_relaxed);
      resp->status = 401;
      resp->extra_headers = "WWW-Authenticate: Bearer realm=\"gpumon\"\r\n";
      resp->inline_body = "unauthorized\n";
      return;
    }
    auto s = store_.get();
    if (!s) {
      resp->status = 503;
      resp->inline_body = "no sample yet\n";
      return;
    }
    resp->content_type = "text/plain; version=0.0.4; charset=utf-8";
    std::vector<std::string> inc, exc;
    std::string err;
    const int fq = req.query.empty() ? 0 : parse_filter_query(req.query, &inc, &exc, &err);
    if (fq < 0) {
      resp->status = 400;
      resp->inline_body = "bad family filter: " + err + "\n";
      return;
    }
    if (fq > 0) {
      // per-request family filter (e.g. a fast Prometheus job for node_gpu_* only)
      auto f = filtered(*s, req.query, req.accept_gzip && cfg_.gzip);
      if (req.accept_gzip && !f->body_gz.empty()) {
        resp->extra_headers = "Content-Encoding: gzip\r\n";
        resp->data = f->body_gz.data();
        resp->len = f->body_gz.size();
      } else {
        resp->data = f->body.data();
        resp->len = f->body.size();
      }
      resp->owner = f;
      return;
    }
    const bool fresh_gz = req.accept_gzip && s->gzip && !s->compressed();
    const std::string* gz = req.accept_gzip ? s->gzipped(true) : nullptr;
    if (fresh_gz && gz) gz_lazy_.fetch_add(1, std::memory_order_relaxed);
    if (req.accept_gzip && s->gzip) {
      // the gzip scrapers' cadence (EWMA of the spacing; bursts under 50 ms ignored) for the tick
      // thread's prediction above
      const int64_t now = mono_ns();
      const int64_t prev = gz_last_scrape_ns_.exchange(now, std::memory_order_relaxed);
      const int64_t d = prev > 0 ? now - prev : 0;
      if (d > 50'000'000) {
        const int64_t p = gz_period_ns_.load(std::memory_order_relaxed);
        const bool same_scraper = p > 0 && d < 8 * p;
        gz_period_ns_.store(same_scraper ? (3 * p + d) / 4 : d, std::memory_order_relaxed);
        const int64_t dev = same_scraper ? std::abs(d - p) : 0, j = gz_jitter_ns_.load(std::memory_order_relaxed);
        gz_jitter_ns_.store(same_scraper ? (3 * j + dev) / 4 : 0, std::memory_order_relaxed);
      }
    }
    if (gz) {
      resp->extra_headers = "Content-Encoding: gzip\r\n";
      resp->data = gz->data();
      resp->len = gz->size();
    } else {
      resp->data = s->body.data();
      resp->len = s->body.size();
    }
    resp->owner = s;
    return;
  }
  if (req.path == "/healthz" || req.path == "/livez") {
    bool ok = healthy();
    resp->status = ok ? 200 : 503;
    resp->inline_body = ok ? "ok\n" : "sampler stalled\n";
    return;
  }
  if (req.path == "/readyz") {
    bool ok = ready() && backend_up_;
    resp->status = ok ? 200 : 503;
    resp->inline_body = ok ? "ready\n" : ("not ready: " + backend_error() + "\n");
    return;
  }
  if (req.path == "/" || req.path.empty()) {
    resp->content_type = "text/html; charset=utf-8";
    resp->inline_body =
        "<html><head><title>gpumon MI355X exporter</title></head><body><h1>gpumon</h1>"
        "<p><a href=\"/metrics\">/metrics</a> &middot; <a href=\"/healthz\">/healthz</a> &middot; "
        "<a href=\"/readyz\">/readyz</a></p></body></html>\n";
    return;
  }
  resp->status = 404;
  resp->inline_body = "not found\n";
}

}  // namespace gpumon

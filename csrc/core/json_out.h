// Minimal JSON writer for the exporter's loopback introspection endpoints (exporter_debug.cpp) and
// the configuration dump (options.cpp). NaN / inf numbers are written as null.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace gpumon {

class JsonOut {
 public:
  JsonOut& obj() { return open('{'); }
  JsonOut& end_obj() { return close('}'); }
  JsonOut& arr() { return open('['); }
  JsonOut& end_arr() { return close(']'); }
  JsonOut& key(const char* k) {
    sep();
    quote(k);
    s_ += ':';
    after_key_ = true;
    return *this;
  }
  JsonOut& str(const std::string& v) {
    sep();
    quote(v);
    return *this;
  }
  JsonOut& num(double v) {
    sep();
    if (!std::isfinite(v)) {
      s_ += "null";
    } else {
      // the shortest of 15 / 17 significant digits that reads back as the same double (0.1, not
      // 0.10000000000000001)
      char b[40];
      snprintf(b, sizeof b, "%.15g", v);
      if (strtod(b, nullptr) != v) snprintf(b, sizeof b, "%.17g", v);
      s_ += b;
    }
    return *this;
  }
  JsonOut& i64(int64_t v) {
    sep();
    s_ += std::to_string(v);
    return *this;
  }
  JsonOut& u64(uint64_t v) {
    sep();
    s_ += std::to_string(v);
    return *this;
  }
  JsonOut& boolean(bool v) {
    sep();
    s_ += v ? "true" : "false";
    return *this;
  }
  JsonOut& null() {
    sep();
    s_ += "null";
    return *this;
  }
  // key + value shorthands
  JsonOut& kv(const char* k, const std::string& v) { return key(k).str(v); }
  JsonOut& kv(const char* k, const char* v) { return key(k).str(v); }
  JsonOut& kv(const char* k, double v) { return key(k).num(v); }
  JsonOut& kv(const char* k, bool v) { return key(k).boolean(v); }
  JsonOut& kv(const char* k, int v) { return key(k).i64(v); }
  JsonOut& kv(const char* k, int64_t v) { return key(k).i64(v); }
  JsonOut& kv(const char* k, uint64_t v) { return key(k).u64(v); }
  JsonOut& kv(const char* k, const std::vector<std::string>& v) {
    key(k).arr();
    for (const auto& x : v) str(x);
    return end_arr();
  }
  const std::string& text() const { return s_; }
  std::string take() { return std::move(s_); }

  static void quote_to(const std::string& v, std::string* o) {
    o->push_back('"');
    for (unsigned char c : v) {
      if (c == '"' || c == '\\') {
        o->push_back('\\');
        o->push_back(static_cast<char>(c));
      } else if (c == '\n') {
        o->append("\\n");
      } else if (c == '\t') {
        o->append("\\t");
      } else if (c < 0x20) {
        char b[8];
        snprintf(b, sizeof b, "\\u%04x", c);
        o->append(b);
      } else {
        o->push_back(static_cast<char>(c));
      }
    }
    o->push_back('"');
  }

 private:
  void quote(const std::string& v) { quote_to(v, &s_); }
  void sep() {
    if (after_key_) {
      after_key_ = false;
      return;
    }
    if (!first_.empty()) {
      if (!first_.back()) s_ += ',';
      first_.back() = false;
    }
  }
  JsonOut& open(char c) {
    sep();
    s_ += c;
    first_.push_back(true);
    return *this;
  }
  JsonOut& close(char c) {
    s_ += c;
    if (!first_.empty()) first_.pop_back();
    return *this;
  }
  std::string s_;
  std::vector<bool> first_;
  bool after_key_ = false;
};

}  // namespace gpumon

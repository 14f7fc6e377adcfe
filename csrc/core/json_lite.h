// Bounded recursive-descent JSON reader shared by the JSON sources (docker_lite.cpp: Docker Engine
// API; kubelet_files.cpp: the kubelet's device-plugin checkpoint). Extracts strings, string arrays
// and string maps, validates and skips everything else; nesting depth and escapes are bounded.
#pragma once

#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace gpumon {

constexpr int kJsonMaxDepth = 64;  // JSON nesting the reader follows

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
    if (depth > kJsonMaxDepth) return fail("nesting too deep"), false;
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

}  // namespace gpumon

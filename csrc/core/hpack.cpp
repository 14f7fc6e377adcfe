#include "hpack.h"

#include <algorithm>
#include <array>

namespace gpumon {

namespace {

// RFC 7541 Appendix A: the static table (index 1..61).
constexpr std::pair<const char*, const char*> kStatic[] = {
    {":authority", ""}, {":method", "GET"}, {":method", "POST"}, {":path", "/"}, {":path", "/index.html"},
    {":scheme", "http"}, {":scheme", "https"}, {":status", "200"}, {":status", "204"}, {":status", "206"},
    {":status", "304"}, {":status", "400"}, {":status", "404"}, {":status", "500"}, {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"}, {"accept-language", ""}, {"accept-ranges", ""}, {"accept", ""},
    {"access-control-allow-origin", ""}, {"age", ""}, {"allow", ""}, {"authorization", ""},
    {"cache-control", ""}, {"content-disposition", ""}, {"content-encoding", ""}, {"content-language", ""},
    {"content-length", ""}, {"content-location", ""}, {"content-range", ""}, {"content-type", ""},
    {"cookie", ""}, {"date", ""}, {"etag", ""}, {"expect", ""}, {"expires", ""}, {"from", ""}, {"host", ""},
    {"if-match", ""}, {"if-modified-since", ""}, {"if-none-match", ""}, {"if-range", ""},
    {"if-unmodified-since", ""}, {"last-modified", ""}, {"link", ""}, {"location", ""}, {"max-forwards", ""},
    {"proxy-authenticate", ""}, {"proxy-authorization", ""}, {"range", ""}, {"referer", ""}, {"refresh", ""},
    {"retry-after", ""}, {"server", ""}, {"set-cookie", ""}, {"strict-transport-security", ""},
    {"transfer-encoding", ""}, {"user-agent", ""}, {"vary", ""}, {"via", ""}, {"www-authenticate", ""}};
constexpr size_t kStaticN = sizeof(kStatic) / sizeof(kStatic[0]);
static_assert(kStaticN == 61, "HPACK static table has 61 entries");

// Appendix B is a canonical Huffman code: codes are assigned in (length, symbol) order, so the
// code LENGTH of every symbol defines it. Symbols grouped by length (257 = EOS); the assignment
// reproduces every Appendix C example (tests/test_hpack.py).
struct Group {
  int len;
  std::vector<int> syms;
};
std::vector<Group> groups() {
  auto chars = [](const char* s) {
    std::vector<int> v;
    for (; *s; ++s) v.push_back(static_cast<unsigned char>(*s));
    return v;
  };
  std::vector<Group> g = {
      {5, chars("012aceiost")},
      {6, chars(" %-./3456789=A_bdfghlmnpru")},
      {7, chars(":BCDEFGHIJKLMNOPQRSTUVWYjkqvwxyz")},
      {8, chars("&*,;XZ")},
      {10, chars("!\"()?")},
      {11, chars("'+|")},
      {12, chars("#>")},
      {13, {0, '$', '@', '[', ']', '~'}},
      {14, chars("^}")},
      {15, chars("<`{")},
      {19, {92, 195, 208}},
      {20, {128, 130, 131, 162, 184, 194, 224, 226}},
      {21, {153, 161, 167, 172, 176, 177, 179, 209, 216, 217, 227, 229, 230}},
      {22, {129, 132, 133, 134, 136, 146, 154, 156, 160, 163, 164, 169, 170,
            173, 178, 181, 185, 186, 187, 189, 190, 196, 198, 228, 232, 233}},
      {23, {1,   135, 137, 138, 139, 140, 141, 143, 147, 149, 150, 151, 152, 155, 157,
            158, 165, 166, 168, 174, 175, 180, 182, 183, 188, 191, 197, 231, 239}},
      {24, {9, 142, 144, 145, 148, 159, 171, 206, 215, 225, 236, 237}},
      {25, {199, 207, 234, 235}},
      {26, {192, 193, 200, 201, 202, 205, 210, 213, 218, 219, 238, 240, 242, 243, 255}},
      {27, {203, 204, 211, 212, 214, 221, 222, 223, 241, 244, 245, 246, 247, 248, 250, 251, 252, 253, 254}},
      {28, {2,  3,  4,  5,  6,  7,  8,  11, 12, 14, 15, 16, 17, 18,  19,  20,  21, 23,
            24, 25, 26, 27, 28, 29, 30, 31, 127, 220, 249}},
      {30, {10, 13, 22, 256}},
  };
  for (auto& x : g) std::sort(x.syms.begin(), x.syms.end());
  return g;
}

struct Huff {
  // canonical decoding tables per code length 1..30
  std::array<uint32_t, 31> first{};   // first code of this length
  std::array<uint32_t, 31> count{};   // symbols of this length
  std::array<uint32_t, 31> offset{};  // index of the first of them in `order`
  std::vector<int> order;             // symbols in code order
  std::array<uint32_t, 257> code{};
  std::array<uint8_t, 257> len{};
  Huff() {
    uint32_t c = 0;
    int prev = 0;
    for (const auto& g : groups()) {
      for (size_t k = 0; k < g.syms.size(); ++k) {
        if (prev) c = (c + 1) << (g.len - prev);
        prev = g.len;
        if (k == 0) {
          first[g.len] = c;
          offset[g.len] = static_cast<uint32_t>(order.size());
        }
        count[g.len]++;
        order.push_back(g.syms[k]);
        code[g.syms[k]] = c;
        len[g.syms[k]] = static_cast<uint8_t>(g.len);
      }
    }
  }
};

const Huff& huff() {
  static const Huff h;
  return h;
}

}  // namespace

bool hpack_huffman_decode(std::string_view in, std::string* out) {
  const Huff& h = huff();
  out->clear();
  uint32_t code = 0;
  int len = 0;
  for (unsigned char byte : in) {
    for (int b = 7; b >= 0; --b) {
      code = (code << 1) | ((byte >> b) & 1u);
      ++len;
      if (len > 30) return false;
      if (h.count[len] && code >= h.first[len] && code - h.first[len] < h.count[len]) {
        const int sym = h.order[h.offset[len] + (code - h.first[len])];
        if (sym == 256) return false;  // EOS inside a string is an error (§5.2)
        out->push_back(static_cast<char>(sym));
        code = 0;
        len = 0;
      }
    }
  }
  // padding: fewer than 8 bits, all ones (a prefix of EOS)
  return len < 8 && code == ((1u << len) - 1);
}

std::string hpack_huffman_encode(std::string_view in) {
  const Huff& h = huff();
  std::string out;
  uint64_t acc = 0;
  int bits = 0;
  for (unsigned char c : in) {
    acc = (acc << h.len[c]) | h.code[c];
    bits += h.len[c];
    while (bits >= 8) {
      out.push_back(static_cast<char>((acc >> (bits - 8)) & 0xFF));
      bits -= 8;
    }
  }
  if (bits > 0) out.push_back(static_cast<char>(((acc << (8 - bits)) | ((1u << (8 - bits)) - 1)) & 0xFF));
  return out;
}

namespace {

// Integer with an N-bit prefix (§5.1). `p` advances past it.
bool read_int(std::string_view b, size_t* p, int prefix, uint64_t* v) {
  if (*p >= b.size()) return false;
  const uint64_t max = (1u << prefix) - 1;
  uint64_t x = static_cast<unsigned char>(b[(*p)++]) & max;
  if (x < max) {
    *v = x;
    return true;
  }
  for (int shift = 0; shift <= 56; shift += 7) {
    if (*p >= b.size()) return false;
    const unsigned char c = static_cast<unsigned char>(b[(*p)++]);
    x += static_cast<uint64_t>(c & 0x7F) << shift;
    if (!(c & 0x80)) {
      *v = x;
      return true;
    }
  }
  return false;
}

bool read_str(std::string_view b, size_t* p, std::string* out) {
  if (*p >= b.size()) return false;
  const bool huffman = static_cast<unsigned char>(b[*p]) & 0x80;
  uint64_t n = 0;
  if (!read_int(b, p, 7, &n) || n > b.size() - *p) return false;
  std::string_view raw = b.substr(*p, n);
  *p += n;
  if (huffman) return hpack_huffman_decode(raw, out);
  out->assign(raw);
  return true;
}

}  // namespace

bool HpackDecoder::lookup(uint64_t index, std::pair<std::string, std::string>* out) const {
  if (index == 0) return false;
  if (index <= kStaticN) {
    *out = {kStatic[index - 1].first, kStatic[index - 1].second};
    return true;
  }
  const uint64_t d = index - kStaticN - 1;
  if (d >= table_.size()) return false;
  *out = table_[d];
  return true;
}

void HpackDecoder::evict_to(size_t max) {
  while (size_ > max && !table_.empty()) {
    size_ -= 32 + table_.back().first.size() + table_.back().second.size();
    table_.pop_back();
  }
}

void HpackDecoder::insert(std::string name, std::string value) {
  const size_t sz = 32 + name.size() + value.size();
  if (sz > max_) {  // larger than the table: empties it (§4.4)
    table_.clear();
    size_ = 0;
    return;
  }
  evict_to(max_ - sz);
  size_ += sz;
  table_.emplace_front(std::move(name), std::move(value));
}

bool HpackDecoder::decode(std::string_view b, HeaderList* out, std::string* err) {
  size_t p = 0;
  bool fields_seen = false;
  while (p < b.size()) {
    const unsigned char c = static_cast<unsigned char>(b[p]);
    uint64_t idx = 0;
    if (c & 0x80) {  // indexed field (§6.1)
      std::pair<std::string, std::string> f;
      if (!read_int(b, &p, 7, &idx) || !lookup(idx, &f)) {
        *err = "hpack: bad index " + std::to_string(idx);
        return false;
      }
      out->push_back(std::move(f));
      fields_seen = true;
    } else if ((c & 0xE0) == 0x20) {  // dynamic table size update (§6.3), only before fields
      uint64_t sz = 0;
      if (!read_int(b, &p, 5, &sz) || sz > limit_ || fields_seen) {
        *err = "hpack: bad table size update";
        return false;
      }
      max_ = static_cast<size_t>(sz);
      evict_to(max_);
    } else {
      // literal: with incremental indexing (01, 6-bit index), without (0000) / never indexed
      // (0001) (4-bit index); index 0 = the name follows as a string
      const bool indexing = (c & 0xC0) == 0x40;
      std::string name, value;
      if (!read_int(b, &p, indexing ? 6 : 4, &idx)) {
        *err = "hpack: truncated literal";
        return false;
      }
      if (idx) {
        std::pair<std::string, std::string> f;
        if (!lookup(idx, &f)) {
          *err = "hpack: bad name index " + std::to_string(idx);
          return false;
        }
        name = std::move(f.first);
      } else if (!read_str(b, &p, &name)) {
        *err = "hpack: bad name string";
        return false;
      }
      if (!read_str(b, &p, &value)) {
        *err = "hpack: bad value string";
        return false;
      }
      if (indexing) insert(name, value);
      out->emplace_back(std::move(name), std::move(value));
      fields_seen = true;
    }
  }
  return true;
}

}  // namespace gpumon

// HPACK (RFC 7541) header-block decoder for the native gRPC client (grpc_lite.cpp).
//
// Why: a gRPC status travels in HTTP/2 headers -- the trailers (grpc-status / grpc-message) after
// the response message, or a "Trailers-Only" HEADERS frame when the call fails outright
// (Unimplemented, PermissionDenied, version skew). kubelet and containerd (Go http2) encode them
// with HPACK: static / dynamic table indices and Huffman-coded strings. Without a decoder every
// failure collapses into "no gRPC message". This is the replacement for the error reporting of
// `docker inspect` the reference relied on (/root/reference/gpu.py:86-88).
//
// Scope: full decoding (indexed fields, the three literal forms, dynamic-table size updates,
// eviction, Huffman strings with EOS-padding checks); no encoder beyond the test helper.
#pragma once

#include <cstdint>
#include <deque>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace gpumon {

using HeaderList = std::vector<std::pair<std::string, std::string>>;

// Huffman-decodes an HPACK string literal (Appendix B code); false on an invalid code, a
// padding longer than 7 bits or not all-ones, or an EOS symbol inside the string.
bool hpack_huffman_decode(std::string_view in, std::string* out);
// Huffman-encodes (tests, and the fake servers that need Go-like header blocks).
std::string hpack_huffman_encode(std::string_view in);

class HpackDecoder {
 public:
  // `max_table`: the SETTINGS_HEADER_TABLE_SIZE this endpoint advertised (default 4096).
  explicit HpackDecoder(size_t max_table = 4096) : limit_(max_table), max_(max_table) {}
  // Decodes one complete header block (HEADERS + CONTINUATION payloads concatenated, padding and
  // priority removed) and appends its fields to `out`. The dynamic table carries over to the next
  // block of the same connection. False with `err` set on malformed input (a connection error).
  bool decode(std::string_view block, HeaderList* out, std::string* err);
  size_t table_size() const { return size_; }
  size_t table_entries() const { return table_.size(); }

 private:
  bool lookup(uint64_t index, std::pair<std::string, std::string>* out) const;
  void insert(std::string name, std::string value);
  void evict_to(size_t max);
  std::deque<std::pair<std::string, std::string>> table_;  // newest first (dynamic index 62 = front)
  size_t size_ = 0;
  size_t limit_;  // what we advertised: a size update above it is an error
  size_t max_;    // current max (after size updates)
};

}  // namespace gpumon

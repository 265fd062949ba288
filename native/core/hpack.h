// HPACK (RFC 7541) header compression for the HTTP/2 transport under gRPC.
//
// Decoder: full RFC 7541 — static + dynamic table, size updates, Huffman strings —
// since the kubelet's grpc-go peer Huffman-codes and indexes freely.
// Encoder: stateless (never adds to the peer's dynamic table): static-table hits are
// emitted indexed, everything else as "literal without indexing", Huffman-coded when
// that is shorter.  The header sets gRPC exchanges are a handful of short fields, so
// the dynamic table would buy nothing and statelessness keeps encode() thread-safe.
#pragma once

#include <cstdint>
#include <deque>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace bgc::hpack {

using Header = std::pair<std::string, std::string>;
using HeaderList = std::vector<Header>;

size_t huffman_encoded_length(std::string_view s);
std::string huffman_encode(std::string_view s);
// False on invalid codes, an embedded EOS, or padding that is not an EOS prefix ≤ 7 bits.
bool huffman_decode(std::string_view in, std::string* out);

// Integer with an N-bit prefix (RFC 7541 §5.1); `first` holds the bits above the prefix.
void encode_int(std::string& out, uint64_t v, int prefix_bits, uint8_t first);

std::string encode(const HeaderList& headers);

class Decoder {
 public:
  explicit Decoder(size_t max_table_size = 4096) : max_size_(max_table_size), limit_(max_table_size) {}
  // Decodes one complete header block; false (with *err) on a compression error, which
  // is a connection error in HTTP/2.
  bool decode(std::string_view block, HeaderList* out, std::string* err);
  size_t table_size() const { return size_; }
  size_t table_entries() const { return table_.size(); }

 private:
  bool lookup(uint64_t index, Header* h) const;
  void insert(Header h);
  void evict();
  std::deque<Header> table_;  // front = most recent (index 62)
  size_t size_ = 0;
  size_t max_size_;
  size_t limit_;  // SETTINGS_HEADER_TABLE_SIZE we advertised
};

}  // namespace bgc::hpack

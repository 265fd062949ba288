#include "core/hpack.h"

#include <array>
#include <mutex>

namespace bgc::hpack {
namespace {

// RFC 7541 Appendix B.  The code is canonical (codes assigned in (length, symbol)
// order); tests/unit/test_http2.py re-derives it from the lengths and cross-checks the
// encoder against libnghttp2's decoder for every byte value.
const uint32_t kHuffCode[257] = {
    0x1ff8, 0x7fffd8, 0xfffffe2, 0xfffffe3, 0xfffffe4, 0xfffffe5, 0xfffffe6, 0xfffffe7,
    0xfffffe8, 0xffffea, 0x3ffffffc, 0xfffffe9, 0xfffffea, 0x3ffffffd, 0xfffffeb, 0xfffffec,
    0xfffffed, 0xfffffee, 0xfffffef, 0xffffff0, 0xffffff1, 0xffffff2, 0x3ffffffe, 0xffffff3,
    0xffffff4, 0xffffff5, 0xffffff6, 0xffffff7, 0xffffff8, 0xffffff9, 0xffffffa, 0xffffffb,
    0x14, 0x3f8, 0x3f9, 0xffa, 0x1ff9, 0x15, 0xf8, 0x7fa,
    0x3fa, 0x3fb, 0xf9, 0x7fb, 0xfa, 0x16, 0x17, 0x18,
    0x0, 0x1, 0x2, 0x19, 0x1a, 0x1b, 0x1c, 0x1d,
    0x1e, 0x1f, 0x5c, 0xfb, 0x7ffc, 0x20, 0xffb, 0x3fc,
    0x1ffa, 0x21, 0x5d, 0x5e, 0x5f, 0x60, 0x61, 0x62,
    0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a,
    0x6b, 0x6c, 0x6d, 0x6e, 0x6f, 0x70, 0x71, 0x72,
    0xfc, 0x73, 0xfd, 0x1ffb, 0x7fff0, 0x1ffc, 0x3ffc, 0x22,
    0x7ffd, 0x3, 0x23, 0x4, 0x24, 0x5, 0x25, 0x26,
    0x27, 0x6, 0x74, 0x75, 0x28, 0x29, 0x2a, 0x7,
    0x2b, 0x76, 0x2c, 0x8, 0x9, 0x2d, 0x77, 0x78,
    0x79, 0x7a, 0x7b, 0x7ffe, 0x7fc, 0x3ffd, 0x1ffd, 0xffffffc,
    0xfffe6, 0x3fffd2, 0xfffe7, 0xfffe8, 0x3fffd3, 0x3fffd4, 0x3fffd5, 0x7fffd9,
    0x3fffd6, 0x7fffda, 0x7fffdb, 0x7fffdc, 0x7fffdd, 0x7fffde, 0xffffeb, 0x7fffdf,
    0xffffec, 0xffffed, 0x3fffd7, 0x7fffe0, 0xffffee, 0x7fffe1, 0x7fffe2, 0x7fffe3,
    0x7fffe4, 0x1fffdc, 0x3fffd8, 0x7fffe5, 0x3fffd9, 0x7fffe6, 0x7fffe7, 0xffffef,
    0x3fffda, 0x1fffdd, 0xfffe9, 0x3fffdb, 0x3fffdc, 0x7fffe8, 0x7fffe9, 0x1fffde,
    0x7fffea, 0x3fffdd, 0x3fffde, 0xfffff0, 0x1fffdf, 0x3fffdf, 0x7fffeb, 0x7fffec,
    0x1fffe0, 0x1fffe1, 0x3fffe0, 0x1fffe2, 0x7fffed, 0x3fffe1, 0x7fffee, 0x7fffef,
    0xfffea, 0x3fffe2, 0x3fffe3, 0x3fffe4, 0x7ffff0, 0x3fffe5, 0x3fffe6, 0x7ffff1,
    0x3ffffe0, 0x3ffffe1, 0xfffeb, 0x7fff1, 0x3fffe7, 0x7ffff2, 0x3fffe8, 0x1ffffec,
    0x3ffffe2, 0x3ffffe3, 0x3ffffe4, 0x7ffffde, 0x7ffffdf, 0x3ffffe5, 0xfffff1, 0x1ffffed,
    0x7fff2, 0x1fffe3, 0x3ffffe6, 0x7ffffe0, 0x7ffffe1, 0x3ffffe7, 0x7ffffe2, 0xfffff2,
    0x1fffe4, 0x1fffe5, 0x3ffffe8, 0x3ffffe9, 0xffffffd, 0x7ffffe3, 0x7ffffe4, 0x7ffffe5,
    0xfffec, 0xfffff3, 0xfffed, 0x1fffe6, 0x3fffe9, 0x1fffe7, 0x1fffe8, 0x7ffff3,
    0x3fffea, 0x3fffeb, 0x1ffffee, 0x1ffffef, 0xfffff4, 0xfffff5, 0x3ffffea, 0x7ffff4,
    0x3ffffeb, 0x7ffffe6, 0x3ffffec, 0x3ffffed, 0x7ffffe7, 0x7ffffe8, 0x7ffffe9, 0x7ffffea,
    0x7ffffeb, 0xffffffe, 0x7ffffec, 0x7ffffed, 0x7ffffee, 0x7ffffef, 0x7fffff0, 0x3ffffee,
    0x3fffffff,
};
const uint8_t kHuffLen[257] = {
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28,
    28, 28, 28, 28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28,
    6, 10, 10, 12, 13, 6, 8, 11, 10, 10, 8, 11, 8, 6, 6, 6,
    5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 7, 8, 15, 6, 12, 10,
    13, 6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7,
    7, 7, 7, 7, 7, 7, 7, 7, 8, 7, 8, 13, 19, 13, 14, 6,
    15, 5, 6, 5, 6, 5, 6, 6, 6, 5, 7, 7, 6, 6, 6, 5,
    6, 7, 6, 5, 5, 6, 7, 7, 7, 7, 7, 15, 11, 14, 13, 28,
    20, 22, 20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23,
    24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23, 22, 23, 23, 24,
    22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23,
    21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22, 22, 23,
    26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25,
    19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27,
    20, 24, 20, 21, 22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23,
    26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26,
    30,
};

struct HuffNode {
  int16_t child[2] = {-1, -1};
  int16_t sym = -1;
};

class HuffTree {
 public:
  HuffTree() {
    nodes_.emplace_back();
    for (int s = 0; s < 257; ++s) {
      int n = 0;
      for (int b = kHuffLen[s] - 1; b >= 0; --b) {
        int bit = (kHuffCode[s] >> b) & 1;
        if (nodes_[n].child[bit] < 0) {
          nodes_[n].child[bit] = static_cast<int16_t>(nodes_.size());
          nodes_.emplace_back();
        }
        n = nodes_[n].child[bit];
      }
      nodes_[n].sym = static_cast<int16_t>(s);
    }
  }
  const std::vector<HuffNode>& nodes() const { return nodes_; }

 private:
  std::vector<HuffNode> nodes_;
};

const HuffTree& tree() {
  static const HuffTree t;
  return t;
}

struct StaticEntry {
  const char* name;
  const char* value;
};

// RFC 7541 Appendix A (index 1..61).
constexpr std::array<StaticEntry, 61> kStatic = {{
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
    {"transfer-encoding", ""}, {"user-agent", ""}, {"vary", ""}, {"via", ""}, {"www-authenticate", ""},
}};

bool decode_int(std::string_view in, size_t& pos, int prefix_bits, uint64_t* v) {
  if (pos >= in.size()) return false;
  const uint64_t mask = (1u << prefix_bits) - 1;
  uint64_t x = static_cast<uint8_t>(in[pos++]) & mask;
  if (x < mask) {
    *v = x;
    return true;
  }
  for (int shift = 0; shift <= 56; shift += 7) {
    if (pos >= in.size()) return false;
    uint8_t b = static_cast<uint8_t>(in[pos++]);
    x += uint64_t(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *v = x;
      return true;
    }
  }
  return false;
}

bool decode_string(std::string_view in, size_t& pos, std::string* out) {
  if (pos >= in.size()) return false;
  const bool huff = static_cast<uint8_t>(in[pos]) & 0x80;
  uint64_t len = 0;
  if (!decode_int(in, pos, 7, &len) || len > in.size() - pos) return false;
  std::string_view raw = in.substr(pos, len);
  pos += len;
  if (!huff) {
    out->assign(raw.data(), raw.size());
    return true;
  }
  return huffman_decode(raw, out);
}

void encode_string(std::string& out, std::string_view s) {
  const size_t hl = huffman_encoded_length(s);
  if (hl < s.size()) {
    encode_int(out, hl, 7, 0x80);
    out += huffman_encode(s);
  } else {
    encode_int(out, s.size(), 7, 0x00);
    out.append(s.data(), s.size());
  }
}

}  // namespace

size_t huffman_encoded_length(std::string_view s) {
  uint64_t bits = 0;
  for (unsigned char c : s) bits += kHuffLen[c];
  return (bits + 7) / 8;
}

std::string huffman_encode(std::string_view s) {
  std::string out;
  out.reserve(huffman_encoded_length(s));
  uint64_t acc = 0;
  int nbits = 0;
  for (unsigned char c : s) {
    acc = (acc << kHuffLen[c]) | kHuffCode[c];
    nbits += kHuffLen[c];
    while (nbits >= 8) {
      nbits -= 8;
      out.push_back(static_cast<char>((acc >> nbits) & 0xff));
    }
    acc &= (uint64_t(1) << nbits) - 1;
  }
  if (nbits > 0) {  // pad with the most significant bits of EOS (all ones)
    out.push_back(static_cast<char>(((acc << (8 - nbits)) | ((1u << (8 - nbits)) - 1)) & 0xff));
  }
  return out;
}

bool huffman_decode(std::string_view in, std::string* out) {
  const auto& nodes = tree().nodes();
  out->clear();
  int n = 0;
  int pending_bits = 0;   // bits consumed since the last complete symbol
  bool pending_ones = true;
  for (unsigned char byte : in) {
    for (int b = 7; b >= 0; --b) {
      int bit = (byte >> b) & 1;
      n = nodes[n].child[bit];
      if (n < 0) return false;
      ++pending_bits;
      pending_ones = pending_ones && bit;
      if (nodes[n].sym >= 0) {
        if (nodes[n].sym == 256) return false;  // EOS inside a string
        out->push_back(static_cast<char>(nodes[n].sym));
        n = 0;
        pending_bits = 0;
        pending_ones = true;
      }
    }
  }
  return pending_bits <= 7 && pending_ones;
}

void encode_int(std::string& out, uint64_t v, int prefix_bits, uint8_t first) {
  const uint64_t mask = (1u << prefix_bits) - 1;
  if (v < mask) {
    out.push_back(static_cast<char>(first | v));
    return;
  }
  out.push_back(static_cast<char>(first | mask));
  v -= mask;
  while (v >= 0x80) {
    out.push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  out.push_back(static_cast<char>(v));
}

std::string encode(const HeaderList& headers) {
  std::string out;
  for (const auto& [name, value] : headers) {
    int name_idx = 0, full_idx = 0;
    for (size_t i = 0; i < kStatic.size(); ++i) {
      if (name != kStatic[i].name) continue;
      if (!name_idx) name_idx = static_cast<int>(i + 1);
      if (value == kStatic[i].value) {
        full_idx = static_cast<int>(i + 1);
        break;
      }
    }
    if (full_idx) {
      encode_int(out, full_idx, 7, 0x80);  // indexed header field
      continue;
    }
    // literal without indexing (0000xxxx), indexed name when the static table has it
    encode_int(out, name_idx, 4, 0x00);
    if (!name_idx) encode_string(out, name);
    encode_string(out, value);
  }
  return out;
}

bool Decoder::lookup(uint64_t index, Header* h) const {
  if (index == 0) return false;
  if (index <= kStatic.size()) {
    *h = {kStatic[index - 1].name, kStatic[index - 1].value};
    return true;
  }
  uint64_t d = index - kStatic.size() - 1;
  if (d >= table_.size()) return false;
  *h = table_[d];
  return true;
}

void Decoder::evict() {
  while (size_ > max_size_ && !table_.empty()) {
    size_ -= table_.back().first.size() + table_.back().second.size() + 32;
    table_.pop_back();
  }
}

void Decoder::insert(Header h) {
  size_t sz = h.first.size() + h.second.size() + 32;
  if (sz > max_size_) {  // an oversized entry empties the table (RFC 7541 §4.4)
    table_.clear();
    size_ = 0;
    return;
  }
  size_ += sz;
  table_.push_front(std::move(h));
  evict();
}

bool Decoder::decode(std::string_view in, HeaderList* out, std::string* err) {
  size_t pos = 0;
  bool fields_seen = false;
  while (pos < in.size()) {
    const uint8_t b = static_cast<uint8_t>(in[pos]);
    uint64_t idx = 0;
    if (b & 0x80) {  // indexed
      Header h;
      if (!decode_int(in, pos, 7, &idx) || !lookup(idx, &h)) {
        *err = "invalid indexed header field";
        return false;
      }
      out->push_back(std::move(h));
      fields_seen = true;
    } else if ((b & 0xe0) == 0x20) {  // dynamic table size update
      if (fields_seen) {
        *err = "table size update after a header field";
        return false;
      }
      if (!decode_int(in, pos, 5, &idx) || idx > limit_) {
        *err = "invalid dynamic table size update";
        return false;
      }
      max_size_ = idx;
      evict();
    } else {
      const bool incremental = (b & 0xc0) == 0x40;
      const int prefix = incremental ? 6 : 4;
      Header h;
      if (!decode_int(in, pos, prefix, &idx)) {
        *err = "truncated literal header field";
        return false;
      }
      if (idx) {
        Header named;
        if (!lookup(idx, &named)) {
          *err = "invalid literal name index";
          return false;
        }
        h.first = std::move(named.first);
      } else if (!decode_string(in, pos, &h.first)) {
        *err = "invalid literal header name";
        return false;
      }
      if (!decode_string(in, pos, &h.second)) {
        *err = "invalid literal header value";
        return false;
      }
      if (incremental) insert(h);
      out->push_back(std::move(h));
      fields_seen = true;
    }
  }
  return true;
}

}  // namespace bgc::hpack

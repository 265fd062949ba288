#include "core/protobuf.h"

namespace bgc::pb {

void Writer::varint(uint64_t v) {
  while (v >= 0x80) {
    buf_.push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  buf_.push_back(static_cast<char>(v));
}

void Writer::u64(uint32_t field, uint64_t v) {
  if (v == 0) return;
  tag(field, kVarint);
  varint(v);
}

void Writer::str(uint32_t field, std::string_view v) {
  if (v.empty()) return;
  bytes(field, v);
}

void Writer::bytes(uint32_t field, std::string_view v) {
  tag(field, kLen);
  varint(v.size());
  buf_.append(v.data(), v.size());
}

void Writer::map_entry(uint32_t field, std::string_view key, std::string_view value) {
  Writer e;
  e.str(1, key);
  e.str(2, value);
  message(field, e);
}

uint64_t Reader::read_varint() {
  uint64_t v = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (pos_ >= buf_.size()) throw DecodeError("truncated varint");
    uint8_t b = static_cast<uint8_t>(buf_[pos_++]);
    v |= uint64_t(b & 0x7f) << shift;
    if (!(b & 0x80)) return v;
  }
  throw DecodeError("varint longer than 10 bytes");
}

bool Reader::next() {
  if (pos_ >= buf_.size()) return false;
  uint64_t key = read_varint();
  field_ = static_cast<uint32_t>(key >> 3);
  wt_ = static_cast<WireType>(key & 7);
  if (field_ == 0) throw DecodeError("field number 0");
  switch (wt_) {
    case kVarint:
      scalar_ = read_varint();
      break;
    case kFixed64:
      if (buf_.size() - pos_ < 8) throw DecodeError("truncated fixed64");
      scalar_ = 0;
      for (int i = 0; i < 8; ++i) scalar_ |= uint64_t(static_cast<uint8_t>(buf_[pos_ + i])) << (8 * i);
      pos_ += 8;
      break;
    case kFixed32:
      if (buf_.size() - pos_ < 4) throw DecodeError("truncated fixed32");
      scalar_ = 0;
      for (int i = 0; i < 4; ++i) scalar_ |= uint64_t(static_cast<uint8_t>(buf_[pos_ + i])) << (8 * i);
      pos_ += 4;
      break;
    case kLen: {
      uint64_t n = read_varint();
      if (n > buf_.size() - pos_) throw DecodeError("length-delimited field overruns buffer");
      payload_ = buf_.substr(pos_, n);
      pos_ += n;
      break;
    }
    default:
      throw DecodeError("unsupported wire type " + std::to_string(static_cast<int>(wt_)));
  }
  return true;
}

uint64_t Reader::varint_value() const {
  if (wt_ == kLen) throw DecodeError("field " + std::to_string(field_) + " is length-delimited, expected scalar");
  return scalar_;
}

std::string_view Reader::bytes_value() const {
  if (wt_ != kLen) throw DecodeError("field " + std::to_string(field_) + " is not length-delimited");
  return payload_;
}

std::pair<std::string, std::string> read_map_entry(std::string_view payload) {
  std::pair<std::string, std::string> kv;
  Reader r(payload);
  while (r.next()) {
    if (r.field() == 1) kv.first = r.string_value();
    else if (r.field() == 2) kv.second = r.string_value();
  }
  return kv;
}

}  // namespace bgc::pb

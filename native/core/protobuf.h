// Protocol Buffers wire format (proto3): just enough of an encoder/decoder for the
// kubelet device-plugin API (k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1), which the
// node agent speaks over gRPC without protoc or libprotobuf (neither is in the image).
//
// Writer appends fields in field-number order as the caller emits them; proto3 scalar
// defaults (0, false, "") are skipped like protoc-generated code does.  Reader walks a
// buffer field by field; unknown fields are skipped by wire type, so messages from newer
// kubelets (extra fields) still decode.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>

namespace bgc::pb {

class DecodeError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

enum WireType : uint32_t { kVarint = 0, kFixed64 = 1, kLen = 2, kFixed32 = 5 };

class Writer {
 public:
  void varint(uint64_t v);
  void tag(uint32_t field, WireType wt) { varint((uint64_t(field) << 3) | wt); }
  // Scalars (skipped when equal to the proto3 default).
  void u64(uint32_t field, uint64_t v);
  void i64(uint32_t field, int64_t v) { u64(field, static_cast<uint64_t>(v)); }
  void i32(uint32_t field, int32_t v) { u64(field, static_cast<uint64_t>(static_cast<int64_t>(v))); }
  void boolean(uint32_t field, bool v) { u64(field, v ? 1 : 0); }
  void str(uint32_t field, std::string_view v);
  // Length-delimited, always emitted (repeated string elements, sub-messages — an empty
  // sub-message is still "present").
  void bytes(uint32_t field, std::string_view v);
  void message(uint32_t field, const Writer& sub) { bytes(field, sub.data()); }
  // map<string,string> entry: {1: key, 2: value}
  void map_entry(uint32_t field, std::string_view key, std::string_view value);

  const std::string& data() const { return buf_; }
  std::string take() { return std::move(buf_); }

 private:
  std::string buf_;
};

class Reader {
 public:
  explicit Reader(std::string_view buf) : buf_(buf) {}
  // Advances to the next field; false at end of buffer. Throws DecodeError on malformed input.
  bool next();
  uint32_t field() const { return field_; }
  WireType wire_type() const { return wt_; }
  uint64_t varint_value() const;           // for kVarint fields
  std::string_view bytes_value() const;    // for kLen fields
  int64_t int64_value() const { return static_cast<int64_t>(varint_value()); }
  bool bool_value() const { return varint_value() != 0; }
  std::string string_value() const { return std::string(bytes_value()); }

 private:
  uint64_t read_varint();
  std::string_view buf_;
  size_t pos_ = 0;
  uint32_t field_ = 0;
  WireType wt_ = kVarint;
  uint64_t scalar_ = 0;
  std::string_view payload_;
};

// Decodes one map<string,string> entry payload.
std::pair<std::string, std::string> read_map_entry(std::string_view payload);

}  // namespace bgc::pb

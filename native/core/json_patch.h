// RFC 6901 JSON Pointer, RFC 6902 JSON Patch and RFC 7386 JSON Merge Patch.
//
// The reference only *builds* add/replace operations (src/admission.rs:354-416,
// src/synchronizer.rs:242-286, via the json-patch crate); the in-tree apiserver also
// has to *apply* them, so the full op set is implemented.
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "core/json.h"

namespace bgc::json {

class PatchError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

std::vector<std::string> parse_pointer(const std::string& pointer);
std::string escape_pointer_token(const std::string& token);
const Value* resolve_pointer(const Value& doc, const std::string& pointer);

// Patch builder: mirrors the json-patch crate's PatchOperation serialization
// ({"op":..,"path":..,"value":..}).
class PatchBuilder {
 public:
  PatchBuilder& add(const std::string& path, Value v);
  PatchBuilder& replace(const std::string& path, Value v);
  PatchBuilder& remove(const std::string& path);
  PatchBuilder& test(const std::string& path, Value v);
  bool empty() const { return ops_.empty(); }
  size_t size() const { return ops_.size(); }
  const Value& ops() const { return ops_; }
  std::string dump() const { return ops_.dump(); }

 private:
  Value ops_ = Value::array();
};

// Applies an RFC 6902 patch document (array of ops) to `doc` atomically: on error
// `doc` is left unchanged and PatchError is thrown.
void apply_patch(Value& doc, const Value& patch);
// RFC 7386 merge patch.
void apply_merge_patch(Value& doc, const Value& patch);

}  // namespace bgc::json

// Minimal, fast JSON DOM for the controller stack.
//
// Objects keep insertion order (parallel key/value vectors) so that wire output is
// stable; Kubernetes payloads are small, so linear key lookup beats hashing here.
// Integers are kept as int64/uint64 so quantities and resourceVersions never lose
// precision (serde_json parity for the i64 CSV columns, reference
// src/synchronizer.rs:83-91).
#pragma once

#include <cstdint>
#include <initializer_list>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace bgc::json {

enum class Type : uint8_t { Null, Bool, Int, UInt, Double, String, Array, Object };

class ParseError : public std::runtime_error {
 public:
  ParseError(const std::string& msg, size_t line, size_t column)
      : std::runtime_error(msg + " at line " + std::to_string(line) + " column " +
                           std::to_string(column)),
        line_(line), column_(column) {}
  size_t line() const { return line_; }
  size_t column() const { return column_; }

 private:
  size_t line_, column_;
};

class TypeError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Value {
 public:
  Value() = default;
  Value(std::nullptr_t) {}
  Value(bool b) : type_(Type::Bool) { num_.b = b; }
  Value(int v) : type_(Type::Int) { num_.i = v; }
  Value(long v) : type_(Type::Int) { num_.i = v; }
  Value(long long v) : type_(Type::Int) { num_.i = v; }
  Value(unsigned v) : type_(Type::Int) { num_.i = v; }
  Value(unsigned long v) { set_unsigned(v); }
  Value(unsigned long long v) { set_unsigned(v); }
  Value(double v) : type_(Type::Double) { num_.d = v; }
  Value(const char* s) : type_(Type::String), str_(s) {}
  Value(std::string s) : type_(Type::String), str_(std::move(s)) {}
  Value(std::string_view s) : type_(Type::String), str_(s) {}

  static Value array() { Value v; v.type_ = Type::Array; return v; }
  static Value object() { Value v; v.type_ = Type::Object; return v; }
  static Value array(std::initializer_list<Value> items);
  static Value object(std::initializer_list<std::pair<std::string, Value>> items);

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_bool() const { return type_ == Type::Bool; }
  bool is_int() const { return type_ == Type::Int || type_ == Type::UInt; }
  bool is_number() const { return is_int() || type_ == Type::Double; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }

  bool as_bool() const;
  int64_t as_int() const;
  uint64_t as_uint() const;
  double as_double() const;
  const std::string& as_string() const;
  std::string& as_string_mut();

  // --- array API ---
  size_t size() const;  // array or object element count
  bool empty() const { return size() == 0; }
  const Value& operator[](size_t i) const;
  Value& operator[](size_t i);
  void push_back(Value v);
  const std::vector<Value>& items() const;
  std::vector<Value>& items_mut();
  void erase_index(size_t i);
  void insert_at(size_t i, Value v);

  // --- object API ---
  // find returns nullptr when missing (or when this is not an object).
  const Value* find(std::string_view key) const;
  Value* find_mut(std::string_view key);
  bool contains(std::string_view key) const { return find(key) != nullptr; }
  // operator[] on objects inserts Null when missing (converting Null -> Object).
  Value& operator[](std::string_view key);
  const Value& at(std::string_view key) const;  // throws when missing
  // Returns a static null Value when missing; convenient for optional chains.
  const Value& get(std::string_view key) const;
  void set(std::string_view key, Value v);
  bool erase(std::string_view key);
  const std::vector<std::string>& keys() const;
  const std::vector<Value>& values() const { return items(); }
  std::vector<Value>& values_mut() { return items_mut(); }
  void sort_keys_recursive();

  // Path helpers ("a.b.c" style, object-only) for terse accessors.
  const Value* path(std::initializer_list<std::string_view> keys) const;
  std::string get_string(std::string_view key, const std::string& dflt = "") const;

  bool operator==(const Value& o) const;
  bool operator!=(const Value& o) const { return !(*this == o); }

  std::string dump() const;                  // compact
  std::string dump_pretty(int indent = 2) const;
  void dump_to(std::string& out) const;

 private:
  void set_unsigned(unsigned long long v);
  void require(Type t, const char* what) const;
  void require_object(const char* what);

  Type type_ = Type::Null;
  union {
    bool b;
    int64_t i;
    uint64_t u;
    double d;
  } num_{};
  std::string str_;
  std::vector<Value> arr_;          // array items, or object values
  std::vector<std::string> keys_;   // object keys (parallel to arr_)
  friend class Parser;
};

Value parse(std::string_view text);
// Parses, dropping every object member named `drop_key` (at any depth) without building its
// value: a watch consumer that never reads metadata.managedFields skips the largest part of
// an SSA-managed object.  The dropped value is scanned for balanced brackets and closed
// strings only, not fully validated.
Value parse(std::string_view text, std::string_view drop_key);
// Parses; returns false (and fills err) instead of throwing.
bool try_parse(std::string_view text, Value& out, std::string* err = nullptr);

// Selective parsing: only the members a projection names are built.  Every other value is
// still fully validated (the same syntax errors as parse) but stands in the result as an
// empty value of its own type ("", 0, false, {}, []), so a caller that only tests the
// type or presence of those members sees the same answers without the allocations of
// big subtrees (an AdmissionReview's oldObject and managedFields).
struct Projection {
  enum Mode : uint8_t {
    Keep,     // build the whole value
    Shape,    // validate; keep only its type
    Descend,  // an object: `children` name the members to build, the rest is Shape
  };
  std::string_view key;
  Mode mode = Keep;
  const Projection* children = nullptr;
  size_t n_children = 0;
  // Descend only: members `children` do not name are stepped over with a structural scan
  // (balanced brackets, closed strings; not validated) and left out of the result, instead
  // of standing in as empty values.  For trusted input whose extra members are large (a
  // watch event's managedFields and annotations).
  bool omit_unnamed = false;
};
Value parse_projected(std::string_view text, const Projection& root);
bool try_parse_projected(std::string_view text, const Projection& root, Value& out, std::string* err = nullptr);
// Raw text of a top-level object member's value (structural scan: no parsing, no
// allocation), e.g. raw_member(review, "request") for logging a received document
// without re-serializing it.  Empty when `text` is not an object or has no such key;
// assumes `text` is valid JSON (run it through parse first).
std::string_view raw_member(std::string_view text, std::string_view key);

void escape_string(std::string_view s, std::string& out);
std::string quote(std::string_view s);
const char* type_name(Type t);

extern const Value kNull;

}  // namespace bgc::json

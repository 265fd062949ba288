#include "core/json.h"

#include <cctype>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstring>
#include <numeric>

namespace bgc::json {

const Value kNull;

const char* type_name(Type t) {
  switch (t) {
    case Type::Null: return "null";
    case Type::Bool: return "boolean";
    case Type::Int:
    case Type::UInt: return "integer";
    case Type::Double: return "number";
    case Type::String: return "string";
    case Type::Array: return "array";
    case Type::Object: return "object";
  }
  return "?";
}

Value Value::array(std::initializer_list<Value> items) {
  Value v = array();
  v.arr_.assign(items.begin(), items.end());
  return v;
}

Value Value::object(std::initializer_list<std::pair<std::string, Value>> items) {
  Value v = object();
  v.keys_.reserve(items.size());
  v.arr_.reserve(items.size());
  for (auto& kv : items) v.set(kv.first, kv.second);
  return v;
}

void Value::set_unsigned(unsigned long long v) {
  if (v <= static_cast<unsigned long long>(INT64_MAX)) {
    type_ = Type::Int;
    num_.i = static_cast<int64_t>(v);
  } else {
    type_ = Type::UInt;
    num_.u = v;
  }
}

void Value::require(Type t, const char* what) const {
  if (type_ != t) {
    throw TypeError(std::string(what) + ": expected " + type_name(t) + ", got " +
                    type_name(type_));
  }
}

void Value::require_object(const char* what) {
  if (type_ == Type::Null) {
    type_ = Type::Object;
    return;
  }
  require(Type::Object, what);
}

bool Value::as_bool() const {
  require(Type::Bool, "as_bool");
  return num_.b;
}

int64_t Value::as_int() const {
  if (type_ == Type::Int) return num_.i;
  if (type_ == Type::UInt) throw TypeError("as_int: value out of int64 range");
  if (type_ == Type::Double) {
    double d = num_.d;
    if (std::floor(d) == d && d >= -9.2e18 && d <= 9.2e18) return static_cast<int64_t>(d);
  }
  throw TypeError(std::string("as_int: expected integer, got ") + type_name(type_));
}

uint64_t Value::as_uint() const {
  if (type_ == Type::UInt) return num_.u;
  if (type_ == Type::Int && num_.i >= 0) return static_cast<uint64_t>(num_.i);
  throw TypeError(std::string("as_uint: expected unsigned integer, got ") + type_name(type_));
}

double Value::as_double() const {
  switch (type_) {
    case Type::Int: return static_cast<double>(num_.i);
    case Type::UInt: return static_cast<double>(num_.u);
    case Type::Double: return num_.d;
    default: throw TypeError(std::string("as_double: expected number, got ") + type_name(type_));
  }
}

const std::string& Value::as_string() const {
  require(Type::String, "as_string");
  return str_;
}

std::string& Value::as_string_mut() {
  require(Type::String, "as_string_mut");
  return str_;
}

size_t Value::size() const {
  if (type_ == Type::Array || type_ == Type::Object) return arr_.size();
  return 0;
}

const Value& Value::operator[](size_t i) const {
  require(Type::Array, "index");
  if (i >= arr_.size()) throw TypeError("index out of range");
  return arr_[i];
}

Value& Value::operator[](size_t i) {
  require(Type::Array, "index");
  if (i >= arr_.size()) throw TypeError("index out of range");
  return arr_[i];
}

void Value::push_back(Value v) {
  if (type_ == Type::Null) type_ = Type::Array;
  require(Type::Array, "push_back");
  arr_.push_back(std::move(v));
}

const std::vector<Value>& Value::items() const {
  static const std::vector<Value> kEmpty;
  if (type_ != Type::Array && type_ != Type::Object) return kEmpty;
  return arr_;
}

std::vector<Value>& Value::items_mut() {
  if (type_ != Type::Array && type_ != Type::Object) {
    throw TypeError(std::string("items_mut on ") + type_name(type_));
  }
  return arr_;
}

void Value::erase_index(size_t i) {
  require(Type::Array, "erase_index");
  if (i >= arr_.size()) throw TypeError("index out of range");
  arr_.erase(arr_.begin() + static_cast<long>(i));
}

void Value::insert_at(size_t i, Value v) {
  require(Type::Array, "insert_at");
  if (i > arr_.size()) throw TypeError("index out of range");
  arr_.insert(arr_.begin() + static_cast<long>(i), std::move(v));
}

const Value* Value::find(std::string_view key) const {
  if (type_ != Type::Object) return nullptr;
  for (size_t i = 0; i < keys_.size(); ++i) {
    if (keys_[i] == key) return &arr_[i];
  }
  return nullptr;
}

Value* Value::find_mut(std::string_view key) {
  return const_cast<Value*>(static_cast<const Value*>(this)->find(key));
}

Value& Value::operator[](std::string_view key) {
  require_object("operator[]");
  for (size_t i = 0; i < keys_.size(); ++i) {
    if (keys_[i] == key) return arr_[i];
  }
  if (keys_.capacity() == 0) {  // skip the 1 -> 2 -> 4 regrowth of small objects
    keys_.reserve(4);
    arr_.reserve(4);
  }
  keys_.emplace_back(key);
  arr_.emplace_back();
  return arr_.back();
}

const Value& Value::at(std::string_view key) const {
  const Value* v = find(key);
  if (!v) throw TypeError("missing key: " + std::string(key));
  return *v;
}

const Value& Value::get(std::string_view key) const {
  const Value* v = find(key);
  return v ? *v : kNull;
}

void Value::set(std::string_view key, Value v) { (*this)[key] = std::move(v); }

bool Value::erase(std::string_view key) {
  if (type_ != Type::Object) return false;
  for (size_t i = 0; i < keys_.size(); ++i) {
    if (keys_[i] == key) {
      keys_.erase(keys_.begin() + static_cast<long>(i));
      arr_.erase(arr_.begin() + static_cast<long>(i));
      return true;
    }
  }
  return false;
}

const std::vector<std::string>& Value::keys() const {
  static const std::vector<std::string> kEmpty;
  return type_ == Type::Object ? keys_ : kEmpty;
}

void Value::sort_keys_recursive() {
  if (type_ == Type::Object) {
    std::vector<size_t> idx(keys_.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return keys_[a] < keys_[b]; });
    std::vector<std::string> nk;
    std::vector<Value> nv;
    nk.reserve(idx.size());
    nv.reserve(idx.size());
    for (size_t i : idx) {
      nk.push_back(std::move(keys_[i]));
      nv.push_back(std::move(arr_[i]));
    }
    keys_ = std::move(nk);
    arr_ = std::move(nv);
  }
  if (type_ == Type::Object || type_ == Type::Array) {
    for (auto& v : arr_) v.sort_keys_recursive();
  }
}

const Value* Value::path(std::initializer_list<std::string_view> keys) const {
  const Value* cur = this;
  for (auto k : keys) {
    cur = cur->find(k);
    if (!cur) return nullptr;
  }
  return cur;
}

std::string Value::get_string(std::string_view key, const std::string& dflt) const {
  const Value* v = find(key);
  if (!v || !v->is_string()) return dflt;
  return v->str_;
}

bool Value::operator==(const Value& o) const {
  if (is_number() && o.is_number()) {
    if (type_ == Type::Double || o.type_ == Type::Double) return as_double() == o.as_double();
    if (type_ == Type::UInt || o.type_ == Type::UInt) {
      if (type_ != o.type_) return false;
      return num_.u == o.num_.u;
    }
    return num_.i == o.num_.i;
  }
  if (type_ != o.type_) return false;
  switch (type_) {
    case Type::Null: return true;
    case Type::Bool: return num_.b == o.num_.b;
    case Type::String: return str_ == o.str_;
    case Type::Array: return arr_ == o.arr_;
    case Type::Object: {
      if (keys_.size() != o.keys_.size()) return false;
      for (size_t i = 0; i < keys_.size(); ++i) {
        const Value* ov = o.find(keys_[i]);
        if (!ov || !(arr_[i] == *ov)) return false;
      }
      return true;
    }
    default: return false;
  }
}

// ---------------------------------------------------------------------------
// Serialization

void escape_string(std::string_view s, std::string& out) {
  static const char kHex[] = "0123456789abcdef";
  out.push_back('"');
  size_t run = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    const char* rep = nullptr;
    char buf[7];
    if (c == '"') rep = "\\\"";
    else if (c == '\\') rep = "\\\\";
    else if (c == '\n') rep = "\\n";
    else if (c == '\r') rep = "\\r";
    else if (c == '\t') rep = "\\t";
    else if (c == '\b') rep = "\\b";
    else if (c == '\f') rep = "\\f";
    else if (c < 0x20) {
      buf[0] = '\\'; buf[1] = 'u'; buf[2] = '0'; buf[3] = '0';
      buf[4] = kHex[c >> 4]; buf[5] = kHex[c & 15]; buf[6] = 0;
      rep = buf;
    }
    if (rep) {
      out.append(s.data() + i - run, run);
      run = 0;
      out.append(rep);
    } else {
      ++run;
    }
  }
  out.append(s.data() + s.size() - run, run);
  out.push_back('"');
}

std::string quote(std::string_view s) {
  std::string out;
  out.reserve(s.size() + 2);
  escape_string(s, out);
  return out;
}

static void dump_double(double d, std::string& out) {
  if (!std::isfinite(d)) {
    out.append("null");  // serde_json serializes non-finite floats as null
    return;
  }
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof(buf), d);
  std::string_view sv(buf, static_cast<size_t>(res.ptr - buf));
  out.append(sv);
  // Keep a float a float on round-trip (serde_json prints 1.0 for 1f64).
  if (sv.find_first_of(".eEn") == std::string_view::npos) out.append(".0");
}

static void dump_impl(const Value& v, std::string& out, int indent, int depth);

void Value::dump_to(std::string& out) const { dump_impl(*this, out, -1, 0); }

std::string Value::dump() const {
  std::string out;
  out.reserve(128);
  dump_to(out);
  return out;
}

std::string Value::dump_pretty(int indent) const {
  std::string out;
  dump_impl(*this, out, indent, 0);
  return out;
}

static void newline_indent(std::string& out, int indent, int depth) {
  out.push_back('\n');
  out.append(static_cast<size_t>(indent * depth), ' ');
}

static void dump_impl(const Value& v, std::string& out, int indent, int depth) {
  char buf[32];
  switch (v.type()) {
    case Type::Null: out.append("null"); break;
    case Type::Bool: out.append(v.as_bool() ? "true" : "false"); break;
    case Type::Int: {
      auto r = std::to_chars(buf, buf + sizeof(buf), v.as_int());
      out.append(buf, static_cast<size_t>(r.ptr - buf));
      break;
    }
    case Type::UInt: {
      auto r = std::to_chars(buf, buf + sizeof(buf), v.as_uint());
      out.append(buf, static_cast<size_t>(r.ptr - buf));
      break;
    }
    case Type::Double: dump_double(v.as_double(), out); break;
    case Type::String: escape_string(v.as_string(), out); break;
    case Type::Array: {
      const auto& items = v.items();
      out.push_back('[');
      if (items.empty()) {
        out.push_back(']');
        break;
      }
      for (size_t i = 0; i < items.size(); ++i) {
        if (i) out.push_back(',');
        if (indent >= 0) newline_indent(out, indent, depth + 1);
        dump_impl(items[i], out, indent, depth + 1);
      }
      if (indent >= 0) newline_indent(out, indent, depth);
      out.push_back(']');
      break;
    }
    case Type::Object: {
      const auto& keys = v.keys();
      const auto& vals = v.values();
      out.push_back('{');
      if (keys.empty()) {
        out.push_back('}');
        break;
      }
      for (size_t i = 0; i < keys.size(); ++i) {
        if (i) out.push_back(',');
        if (indent >= 0) newline_indent(out, indent, depth + 1);
        escape_string(keys[i], out);
        out.push_back(':');
        if (indent >= 0) out.push_back(' ');
        dump_impl(vals[i], out, indent, depth + 1);
      }
      if (indent >= 0) newline_indent(out, indent, depth);
      out.push_back('}');
      break;
    }
  }
}

// ---------------------------------------------------------------------------
// Parsing

// Per-thread staging stacks for container children (see parse_value); a Parser never
// nests on one thread, so the stacks start empty for every document.
static thread_local std::vector<Value> t_stage_vals;
static thread_local std::vector<std::string> t_stage_keys;

class Parser {
 public:
  explicit Parser(std::string_view t, std::string_view drop_key = {})
      : s_(t), drop_key_(drop_key), vals_(t_stage_vals), keys_(t_stage_keys) {
    vals_.clear();
    keys_.clear();
  }
  ~Parser() {
    vals_.clear();
    keys_.clear();
    if (vals_.capacity() > 4096) std::vector<Value>().swap(vals_);  // don't pin a huge LIST's worth per thread
    if (keys_.capacity() > 4096) std::vector<std::string>().swap(keys_);
  }

  Value parse_document() {
    Value v;
    skip_ws();
    parse_value(v, 0);
    skip_ws();
    if (p_ != s_.size()) fail("trailing characters");
    return v;
  }

  Value parse_document(const Projection& root) {
    Value v;
    skip_ws();
    parse_projected(v, 0, &root);
    skip_ws();
    if (p_ != s_.size()) fail("trailing characters");
    return v;
  }

 private:
  [[noreturn]] void fail(const std::string& msg) const {
    size_t line = 1, col = 1;
    for (size_t i = 0; i < p_ && i < s_.size(); ++i) {
      if (s_[i] == '\n') {
        ++line;
        col = 1;
      } else {
        ++col;
      }
    }
    throw ParseError(msg, line, col);
  }

  void skip_ws() {
    while (p_ < s_.size()) {
      char c = s_[p_];
      if (c == ' ' || c == '\n' || c == '\r' || c == '\t') ++p_;
      else break;
    }
  }

  void expect_lit(const char* lit) {
    size_t n = std::strlen(lit);
    if (s_.substr(p_, n) != lit) fail("expected value");
    p_ += n;
  }

  void parse_value(Value& out, int depth) {
    if (depth > 512) fail("recursion limit exceeded");
    if (p_ >= s_.size()) fail("EOF while parsing a value");
    char c = s_[p_];
    switch (c) {
      case 'n': expect_lit("null"); out = Value(); return;
      case 't': expect_lit("true"); out = Value(true); return;
      case 'f': expect_lit("false"); out = Value(false); return;
      case '"': {
        out.type_ = Type::String;
        parse_string(out.str_);
        return;
      }
      case '[': {
        ++p_;
        out.type_ = Type::Array;
        skip_ws();
        if (p_ < s_.size() && s_[p_] == ']') {
          ++p_;
          return;
        }
        // Children are staged on a parser-wide stack and moved into an exactly-sized
        // vector at the closing bracket: one allocation per container instead of the
        // 1->2->4->8 regrowth of push_back.
        const size_t base = vals_.size();
        while (true) {
          skip_ws();
          Value child;
          parse_value(child, depth + 1);
          vals_.push_back(std::move(child));
          skip_ws();
          if (p_ >= s_.size()) fail("EOF while parsing a list");
          if (s_[p_] == ',') {
            ++p_;
            continue;
          }
          if (s_[p_] == ']') {
            ++p_;
            out.arr_.reserve(vals_.size() - base);
            for (size_t i = base; i < vals_.size(); ++i) out.arr_.push_back(std::move(vals_[i]));
            vals_.resize(base);
            return;
          }
          fail("expected `,` or `]`");
        }
      }
      case '{': {
        ++p_;
        out.type_ = Type::Object;
        skip_ws();
        if (p_ < s_.size() && s_[p_] == '}') {
          ++p_;
          return;
        }
        const size_t base = vals_.size();
        const size_t kbase = keys_.size();
        while (true) {
          skip_ws();
          if (p_ >= s_.size() || s_[p_] != '"') fail("key must be a string");
          std::string key;
          parse_string(key);
          skip_ws();
          if (p_ >= s_.size() || s_[p_] != ':') fail("expected `:`");
          ++p_;
          skip_ws();
          if (!drop_key_.empty() && key == drop_key_) {
            skip_value();
            skip_ws();
            if (p_ >= s_.size()) fail("EOF while parsing an object");
            if (s_[p_] == ',') {
              ++p_;
              continue;
            }
            if (s_[p_] != '}') fail("expected `,` or `}`");
            ++p_;
            finish_object(out, base, kbase);
            return;
          }
          Value child;
          parse_value(child, depth + 1);
          // Duplicate keys: last one wins (serde_json Value behaviour).
          bool dup = false;
          for (size_t i = kbase; i < keys_.size(); ++i) {
            if (keys_[i] == key) {
              vals_[base + (i - kbase)] = std::move(child);
              dup = true;
              break;
            }
          }
          if (!dup) {
            keys_.push_back(std::move(key));
            vals_.push_back(std::move(child));
          }
          skip_ws();
          if (p_ >= s_.size()) fail("EOF while parsing an object");
          if (s_[p_] == ',') {
            ++p_;
            continue;
          }
          if (s_[p_] == '}') {
            ++p_;
            finish_object(out, base, kbase);
            return;
          }
          fail("expected `,` or `}`");
        }
      }
      default:
        if (c == '-' || (c >= '0' && c <= '9')) {
          parse_number(out);
          return;
        }
        fail("expected value");
    }
  }

  // Projection-driven parse (see json::Projection).  `p` null = not named: Shape.
  void parse_projected(Value& out, int depth, const Projection* p) {
    if (p && p->mode == Projection::Keep) {
      parse_value(out, depth);
      return;
    }
    if (!p || p->mode == Projection::Shape || p_ >= s_.size() || s_[p_] != '{') {
      if (p && p->mode == Projection::Descend) {  // not an object: keep it whole (type errors stay visible)
        parse_value(out, depth);
        return;
      }
      shape_value(out, depth);
      return;
    }
    if (depth > 512) fail("recursion limit exceeded");
    ++p_;
    out.type_ = Type::Object;
    skip_ws();
    if (p_ < s_.size() && s_[p_] == '}') {
      ++p_;
      return;
    }
    const size_t base = vals_.size();
    const size_t kbase = keys_.size();
    while (true) {
      skip_ws();
      if (p_ >= s_.size() || s_[p_] != '"') fail("key must be a string");
      std::string key;
      parse_string(key);
      skip_ws();
      if (p_ >= s_.size() || s_[p_] != ':') fail("expected `:`");
      ++p_;
      skip_ws();
      const Projection* child = nullptr;
      for (size_t i = 0; i < p->n_children; ++i) {
        if (p->children[i].key == key) {
          child = &p->children[i];
          break;
        }
      }
      if (!child && p->omit_unnamed) {
        skip_value();
        skip_ws();
        if (p_ >= s_.size()) fail("EOF while parsing an object");
        if (s_[p_] == ',') {
          ++p_;
          continue;
        }
        if (s_[p_] == '}') {
          ++p_;
          finish_object(out, base, kbase);
          return;
        }
        fail("expected `,` or `}`");
      }
      Value v;
      parse_projected(v, depth + 1, child);
      bool dup = false;
      for (size_t i = kbase; i < keys_.size(); ++i) {
        if (keys_[i] == key) {
          vals_[base + (i - kbase)] = std::move(v);
          dup = true;
          break;
        }
      }
      if (!dup) {
        keys_.push_back(std::move(key));
        vals_.push_back(std::move(v));
      }
      skip_ws();
      if (p_ >= s_.size()) fail("EOF while parsing an object");
      if (s_[p_] == ',') {
        ++p_;
        continue;
      }
      if (s_[p_] == '}') {
        ++p_;
        finish_object(out, base, kbase);
        return;
      }
      fail("expected `,` or `}`");
    }
  }

  // Validates one value exactly as parse_value would, building nothing but an empty value
  // of the same type.
  void shape_value(Value& out, int depth) {
    if (depth > 512) fail("recursion limit exceeded");
    if (p_ >= s_.size()) fail("EOF while parsing a value");
    const char c = s_[p_];
    if (c == '"') {
      static thread_local std::string scratch;
      parse_string(scratch);
      out = Value(std::string());
      return;
    }
    if (c == '[' || c == '{') {
      const bool obj = c == '{';
      ++p_;
      out = obj ? Value::object() : Value::array();
      skip_ws();
      if (p_ < s_.size() && s_[p_] == (obj ? '}' : ']')) {
        ++p_;
        return;
      }
      while (true) {
        skip_ws();
        if (obj) {
          if (p_ >= s_.size() || s_[p_] != '"') fail("key must be a string");
          static thread_local std::string key;
          parse_string(key);
          skip_ws();
          if (p_ >= s_.size() || s_[p_] != ':') fail("expected `:`");
          ++p_;
          skip_ws();
        }
        Value child;
        shape_value(child, depth + 1);
        skip_ws();
        if (p_ >= s_.size()) fail(obj ? "EOF while parsing an object" : "EOF while parsing a list");
        if (s_[p_] == ',') {
          ++p_;
          continue;
        }
        if (s_[p_] == (obj ? '}' : ']')) {
          ++p_;
          return;
        }
        fail(obj ? "expected `,` or `}`" : "expected `,` or `]`");
      }
    }
    parse_value(out, depth);  // literal or number: nothing to save
    if (out.is_number()) out = Value(0);
    else if (out.is_bool()) out = Value(false);
  }

  static int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }

  uint32_t parse_hex4() {
    if (p_ + 4 > s_.size()) fail("EOF while parsing a string");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      int h = hexval(s_[p_ + static_cast<size_t>(i)]);
      if (h < 0) fail("invalid escape");
      v = (v << 4) | static_cast<uint32_t>(h);
    }
    p_ += 4;
    return v;
  }

  static void append_utf8(uint32_t cp, std::string& out) {
    if (cp < 0x80) {
      out.push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }

  void finish_object(Value& out, size_t base, size_t kbase) {
    const size_t n = keys_.size() - kbase;
    out.arr_.reserve(n);
    out.keys_.reserve(n);
    for (size_t i = 0; i < n; ++i) {
      out.keys_.push_back(std::move(keys_[kbase + i]));
      out.arr_.push_back(std::move(vals_[base + i]));
    }
    keys_.resize(kbase);
    vals_.resize(base);
  }

  void skip_string() {
    ++p_;  // opening quote
    while (p_ < s_.size()) {
      const char c = s_[p_];
      if (c == '\\') {
        p_ += 2;
      } else if (c == '"') {
        ++p_;
        return;
      } else {
        ++p_;
      }
    }
    fail("EOF while parsing a string");
  }

  // Steps over one value without materialising it (see parse(text, drop_key)).
  void skip_value() {
    if (p_ >= s_.size()) fail("EOF while parsing a value");
    const char c = s_[p_];
    if (c == '"') {
      skip_string();
      return;
    }
    if (c == '{' || c == '[') {
      int nest = 0;
      while (p_ < s_.size()) {
        const char d = s_[p_];
        if (d == '"') {
          skip_string();
          continue;
        }
        if (d == '{' || d == '[') {
          if (++nest > 512) fail("recursion limit exceeded");
        } else if (d == '}' || d == ']') {
          if (--nest == 0) {
            ++p_;
            return;
          }
        }
        ++p_;
      }
      fail("EOF while parsing a value");
    }
    const size_t start = p_;
    while (p_ < s_.size()) {
      const char d = s_[p_];
      if (d == ',' || d == '}' || d == ']' || d == ' ' || d == '\n' || d == '\r' || d == '\t') break;
      ++p_;
    }
    if (p_ == start) fail("expected value");
  }

  void parse_string(std::string& out) {
    ++p_;  // opening quote
    out.clear();
    size_t start = p_;
    while (true) {
      // fast scan for a run of plain bytes
      while (p_ < s_.size()) {
        unsigned char c = static_cast<unsigned char>(s_[p_]);
        if (c == '"' || c == '\\' || c < 0x20) break;
        ++p_;
      }
      out.append(s_.data() + start, p_ - start);
      if (p_ >= s_.size()) fail("EOF while parsing a string");
      char c = s_[p_];
      if (c == '"') {
        ++p_;
        return;
      }
      if (static_cast<unsigned char>(c) < 0x20) fail("control character in string");
      // escape
      ++p_;
      if (p_ >= s_.size()) fail("EOF while parsing a string");
      char e = s_[p_++];
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = parse_hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (p_ + 6 <= s_.size() && s_[p_] == '\\' && s_[p_ + 1] == 'u') {
              p_ += 2;
              uint32_t lo = parse_hex4();
              if (lo < 0xDC00 || lo > 0xDFFF) fail("lone leading surrogate");
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              fail("lone leading surrogate");
            }
          } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
            fail("lone trailing surrogate");
          }
          append_utf8(cp, out);
          break;
        }
        default: fail("invalid escape");
      }
      start = p_;
    }
  }

  void parse_number(Value& out) {
    size_t start = p_;
    bool neg = false;
    if (s_[p_] == '-') {
      neg = true;
      ++p_;
    }
    if (p_ >= s_.size() || !(s_[p_] >= '0' && s_[p_] <= '9')) fail("invalid number");
    if (s_[p_] == '0' && p_ + 1 < s_.size() && s_[p_ + 1] >= '0' && s_[p_ + 1] <= '9') {
      fail("invalid number");
    }
    while (p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '9') ++p_;
    bool is_float = false;
    if (p_ < s_.size() && s_[p_] == '.') {
      is_float = true;
      ++p_;
      if (p_ >= s_.size() || !(s_[p_] >= '0' && s_[p_] <= '9')) fail("invalid number");
      while (p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '9') ++p_;
    }
    if (p_ < s_.size() && (s_[p_] == 'e' || s_[p_] == 'E')) {
      is_float = true;
      ++p_;
      if (p_ < s_.size() && (s_[p_] == '+' || s_[p_] == '-')) ++p_;
      if (p_ >= s_.size() || !(s_[p_] >= '0' && s_[p_] <= '9')) fail("invalid number");
      while (p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '9') ++p_;
    }
    const char* b = s_.data() + start;
    const char* e = s_.data() + p_;
    if (!is_float) {
      if (neg) {
        int64_t v;
        auto r = std::from_chars(b, e, v);
        if (r.ec == std::errc()) {
          out = Value(static_cast<long long>(v));
          return;
        }
      } else {
        uint64_t v;
        auto r = std::from_chars(b, e, v);
        if (r.ec == std::errc()) {
          out = Value(static_cast<unsigned long long>(v));
          return;
        }
      }
    }
    double d;
    auto r = std::from_chars(b, e, d);
    if (r.ec != std::errc() && r.ec != std::errc::result_out_of_range) fail("invalid number");
    out = Value(d);
  }

  std::string_view s_;
  std::string_view drop_key_;
  size_t p_ = 0;
  std::vector<Value>& vals_;
  std::vector<std::string>& keys_;
};

namespace {
// index just past the string that starts at text[i] == '"'
size_t skip_string(std::string_view t, size_t i) {
  for (++i; i < t.size(); ++i) {
    if (t[i] == '\\') ++i;
    else if (t[i] == '"') return i + 1;
  }
  return t.size();
}
// index just past the value that starts at text[i]
size_t skip_value(std::string_view t, size_t i) {
  if (i >= t.size()) return i;
  if (t[i] == '"') return skip_string(t, i);
  if (t[i] == '{' || t[i] == '[') {
    int depth = 0;
    for (; i < t.size(); ++i) {
      const char c = t[i];
      if (c == '"') {
        i = skip_string(t, i) - 1;
      } else if (c == '{' || c == '[') {
        ++depth;
      } else if (c == '}' || c == ']') {
        if (--depth == 0) return i + 1;
      }
    }
    return t.size();
  }
  while (i < t.size() && t[i] != ',' && t[i] != '}' && t[i] != ']' && !std::isspace(static_cast<unsigned char>(t[i]))) ++i;
  return i;
}
size_t skip_ws(std::string_view t, size_t i) {
  while (i < t.size() && std::isspace(static_cast<unsigned char>(t[i]))) ++i;
  return i;
}
}  // namespace

std::string_view raw_member(std::string_view t, std::string_view key) {
  size_t i = skip_ws(t, 0);
  if (i >= t.size() || t[i] != '{') return {};
  ++i;
  while (true) {
    i = skip_ws(t, i);
    if (i >= t.size() || t[i] != '"') return {};
    const size_t k0 = i + 1, k1 = skip_string(t, i);
    const std::string_view k = t.substr(k0, k1 - 1 - k0);  // raw (escaped) key text
    i = skip_ws(t, k1);
    if (i >= t.size() || t[i] != ':') return {};
    i = skip_ws(t, i + 1);
    const size_t v0 = i, v1 = skip_value(t, i);
    if (k == key) return t.substr(v0, v1 - v0);
    i = skip_ws(t, v1);
    if (i >= t.size() || t[i] != ',') return {};
    ++i;
  }
}

Value parse(std::string_view text) { return Parser(text).parse_document(); }
Value parse(std::string_view text, std::string_view drop_key) { return Parser(text, drop_key).parse_document(); }

Value parse_projected(std::string_view text, const Projection& root) { return Parser(text).parse_document(root); }

bool try_parse_projected(std::string_view text, const Projection& root, Value& out, std::string* err) {
  try {
    out = parse_projected(text, root);
    return true;
  } catch (const ParseError& e) {
    if (err) *err = e.what();
    return false;
  }
}

bool try_parse(std::string_view text, Value& out, std::string* err) {
  try {
    out = parse(text);
    return true;
  } catch (const ParseError& e) {
    if (err) *err = e.what();
    return false;
  }
}

}  // namespace bgc::json

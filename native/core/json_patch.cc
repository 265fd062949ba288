#include "core/json_patch.h"

#include <charconv>

namespace bgc::json {

std::vector<std::string> parse_pointer(const std::string& pointer) {
  std::vector<std::string> out;
  if (pointer.empty()) return out;
  if (pointer[0] != '/') throw PatchError("invalid pointer: " + pointer);
  size_t i = 1;
  std::string cur;
  while (i <= pointer.size()) {
    if (i == pointer.size() || pointer[i] == '/') {
      out.push_back(cur);
      cur.clear();
      ++i;
      continue;
    }
    char c = pointer[i];
    if (c == '~') {
      if (i + 1 >= pointer.size()) throw PatchError("invalid pointer escape: " + pointer);
      char n = pointer[i + 1];
      if (n == '0') cur.push_back('~');
      else if (n == '1') cur.push_back('/');
      else throw PatchError("invalid pointer escape: " + pointer);
      i += 2;
      continue;
    }
    cur.push_back(c);
    ++i;
  }
  return out;
}

std::string escape_pointer_token(const std::string& token) {
  std::string out;
  for (char c : token) {
    if (c == '~') out += "~0";
    else if (c == '/') out += "~1";
    else out.push_back(c);
  }
  return out;
}

static bool parse_index(const std::string& tok, size_t len, bool allow_end, size_t& out) {
  if (allow_end && tok == "-") {
    out = len;
    return true;
  }
  if (tok.empty() || (tok.size() > 1 && tok[0] == '0')) return false;
  for (char c : tok) {
    if (c < '0' || c > '9') return false;
  }
  size_t v = 0;
  auto r = std::from_chars(tok.data(), tok.data() + tok.size(), v);
  if (r.ec != std::errc()) return false;
  if (v > len || (!allow_end && v == len)) return false;
  out = v;
  return true;
}

static Value* walk(Value& doc, const std::vector<std::string>& toks, size_t upto) {
  Value* cur = &doc;
  for (size_t i = 0; i < upto; ++i) {
    const std::string& t = toks[i];
    if (cur->is_object()) {
      cur = cur->find_mut(t);
      if (!cur) return nullptr;
    } else if (cur->is_array()) {
      size_t idx;
      if (!parse_index(t, cur->size(), false, idx)) return nullptr;
      cur = &(*cur)[idx];
    } else {
      return nullptr;
    }
  }
  return cur;
}

const Value* resolve_pointer(const Value& doc, const std::string& pointer) {
  auto toks = parse_pointer(pointer);
  return walk(const_cast<Value&>(doc), toks, toks.size());
}

PatchBuilder& PatchBuilder::add(const std::string& path, Value v) {
  ops_.push_back(Value::object({{"op", "add"}, {"path", path}, {"value", std::move(v)}}));
  return *this;
}
PatchBuilder& PatchBuilder::replace(const std::string& path, Value v) {
  ops_.push_back(Value::object({{"op", "replace"}, {"path", path}, {"value", std::move(v)}}));
  return *this;
}
PatchBuilder& PatchBuilder::remove(const std::string& path) {
  ops_.push_back(Value::object({{"op", "remove"}, {"path", path}}));
  return *this;
}
PatchBuilder& PatchBuilder::test(const std::string& path, Value v) {
  ops_.push_back(Value::object({{"op", "test"}, {"path", path}, {"value", std::move(v)}}));
  return *this;
}

namespace {

void op_add(Value& doc, const std::string& path, Value v) {
  auto toks = parse_pointer(path);
  if (toks.empty()) {
    doc = std::move(v);
    return;
  }
  Value* parent = walk(doc, toks, toks.size() - 1);
  if (!parent) throw PatchError("path not found: " + path);
  const std::string& last = toks.back();
  if (parent->is_object()) {
    parent->set(last, std::move(v));
  } else if (parent->is_array()) {
    size_t idx;
    if (!parse_index(last, parent->size(), true, idx)) throw PatchError("invalid array index: " + path);
    parent->insert_at(idx, std::move(v));
  } else {
    throw PatchError("parent is not a container: " + path);
  }
}

Value op_remove(Value& doc, const std::string& path) {
  auto toks = parse_pointer(path);
  if (toks.empty()) {
    Value old = std::move(doc);
    doc = Value();
    return old;
  }
  Value* parent = walk(doc, toks, toks.size() - 1);
  if (!parent) throw PatchError("path not found: " + path);
  const std::string& last = toks.back();
  if (parent->is_object()) {
    Value* cur = parent->find_mut(last);
    if (!cur) throw PatchError("path not found: " + path);
    Value old = std::move(*cur);
    parent->erase(last);
    return old;
  }
  if (parent->is_array()) {
    size_t idx;
    if (!parse_index(last, parent->size(), false, idx)) throw PatchError("invalid array index: " + path);
    Value old = std::move((*parent)[idx]);
    parent->erase_index(idx);
    return old;
  }
  throw PatchError("parent is not a container: " + path);
}

void op_replace(Value& doc, const std::string& path, Value v) {
  auto toks = parse_pointer(path);
  Value* target = walk(doc, toks, toks.size());
  if (!target) throw PatchError("path not found: " + path);
  *target = std::move(v);
}

const Value& require_field(const Value& op, const char* name) {
  const Value* v = op.find(name);
  if (!v) throw PatchError(std::string("missing field `") + name + "`");
  return *v;
}

std::string require_path(const Value& op, const char* name) {
  const Value& v = require_field(op, name);
  if (!v.is_string()) throw PatchError(std::string("field `") + name + "` must be a string");
  return v.as_string();
}

}  // namespace

void apply_patch(Value& doc, const Value& patch) {
  if (!patch.is_array()) throw PatchError("patch must be an array of operations");
  Value work = doc;
  for (const Value& op : patch.items()) {
    if (!op.is_object()) throw PatchError("patch operation must be an object");
    std::string kind = require_path(op, "op");
    if (kind == "add") {
      op_add(work, require_path(op, "path"), require_field(op, "value"));
    } else if (kind == "remove") {
      op_remove(work, require_path(op, "path"));
    } else if (kind == "replace") {
      op_replace(work, require_path(op, "path"), require_field(op, "value"));
    } else if (kind == "move") {
      std::string from = require_path(op, "from");
      std::string path = require_path(op, "path");
      if (path.size() > from.size() && path.compare(0, from.size(), from) == 0 &&
          path[from.size()] == '/') {
        throw PatchError("cannot move a value into one of its children");
      }
      Value v = op_remove(work, from);
      op_add(work, path, std::move(v));
    } else if (kind == "copy") {
      std::string from = require_path(op, "from");
      const Value* src = resolve_pointer(work, from);
      if (!src) throw PatchError("path not found: " + from);
      Value copy = *src;
      op_add(work, require_path(op, "path"), std::move(copy));
    } else if (kind == "test") {
      std::string path = require_path(op, "path");
      const Value* cur = resolve_pointer(work, path);
      if (!cur || !(*cur == require_field(op, "value"))) throw PatchError("test failed: " + path);
    } else {
      throw PatchError("unknown op: " + kind);
    }
  }
  doc = std::move(work);
}

void apply_merge_patch(Value& doc, const Value& patch) {
  if (!patch.is_object()) {
    doc = patch;
    return;
  }
  if (!doc.is_object()) doc = Value::object();
  const auto& keys = patch.keys();
  const auto& vals = patch.values();
  for (size_t i = 0; i < keys.size(); ++i) {
    if (vals[i].is_null()) {
      doc.erase(keys[i]);
    } else {
      apply_merge_patch(doc[keys[i]], vals[i]);
    }
  }
}

}  // namespace bgc::json

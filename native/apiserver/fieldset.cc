#include "apiserver/fieldset.h"

#include "core/json_patch.h"

namespace bgc::apiserver {

using json::Value;

namespace {

enum class ListKind { Atomic, KeyedByUid, Set };

ListKind list_kind(const std::string& path) {
  if (path == "/metadata/ownerReferences") return ListKind::KeyedByUid;
  if (path == "/metadata/finalizers") return ListKind::Set;
  return ListKind::Atomic;
}

bool ignored(const std::string& path, bool include_status) {
  static const std::set<std::string> kIgnored = {
      "/apiVersion", "/kind", "/metadata/name", "/metadata/namespace", "/metadata/resourceVersion",
      "/metadata/uid", "/metadata/generation", "/metadata/creationTimestamp", "/metadata/managedFields",
      "/metadata/selfLink", "/metadata/deletionTimestamp", "/metadata/deletionGracePeriodSeconds"};
  if (kIgnored.count(path)) return true;
  if (!include_status && (path == "/status" || path.rfind("/status/", 0) == 0)) return true;
  return false;
}

void collect(const Value& v, const std::string& path, FieldSet& out, bool include_status) {
  if (!path.empty() && ignored(path, include_status)) return;
  if (v.is_object() && !v.empty()) {
    const auto& keys = v.keys();
    const auto& vals = v.values();
    for (size_t i = 0; i < keys.size(); ++i) {
      collect(vals[i], path + "/" + json::escape_pointer_token(keys[i]), out, include_status);
    }
    return;
  }
  if (v.is_array() && !v.empty()) {
    ListKind lk = list_kind(path);
    if (lk == ListKind::KeyedByUid) {
      for (const auto& item : v.items()) {
        out.insert(path + "/[uid=" + json::escape_pointer_token(item.get_string("uid")) + "]");
      }
      return;
    }
    if (lk == ListKind::Set) {
      for (const auto& item : v.items()) out.insert(path + "/[=" + json::escape_pointer_token(item.dump()) + "]");
      return;
    }
  }
  if (!path.empty()) out.insert(path);
}

// RFC 6901 tokens of a field path without allocating: a token is a view into the path,
// unescaped into a scratch buffer only when it contains '~' (rare in field paths).
class Tokens {
 public:
  explicit Tokens(std::string_view p) : p_(p), i_(p.empty() ? 1 : 1), end_(p.empty()) {}
  bool next(std::string_view& tok) {
    if (end_ || i_ > p_.size()) return false;
    size_t j = p_.find('/', i_);
    std::string_view raw = p_.substr(i_, j == std::string_view::npos ? std::string_view::npos : j - i_);
    if (j == std::string_view::npos) end_ = true;
    else i_ = j + 1;
    if (raw.find('~') == std::string_view::npos) {
      tok = raw;
      return true;
    }
    scratch_.clear();
    for (size_t k = 0; k < raw.size(); ++k) {
      if (raw[k] == '~' && k + 1 < raw.size()) {
        scratch_.push_back(raw[k + 1] == '1' ? '/' : '~');
        ++k;
      } else {
        scratch_.push_back(raw[k]);
      }
    }
    tok = scratch_;
    return true;
  }
  bool last() const { return end_; }  // after next(): the token just returned was the final one

 private:
  std::string_view p_;
  size_t i_;
  bool end_;
  std::string scratch_;
};

bool is_item_token(std::string_view t) { return t.size() >= 3 && t.front() == '[' && t.back() == ']'; }

// index of the list item matching an item token, or -1
long find_item(const Value& arr, std::string_view tok) {
  std::string_view inner = tok.substr(1, tok.size() - 2);
  if (inner.substr(0, 4) == "uid=") {
    std::string_view uid = inner.substr(4);
    for (size_t i = 0; i < arr.size(); ++i) {
      const Value& u = arr[i].get("uid");
      if (u.is_string() && u.as_string() == uid) return static_cast<long>(i);
    }
    return -1;
  }
  if (!inner.empty() && inner.front() == '=') {
    Value want;
    if (!json::try_parse(inner.substr(1), want, nullptr)) return -1;
    for (size_t i = 0; i < arr.size(); ++i) {
      if (arr[i] == want) return static_cast<long>(i);
    }
  }
  return -1;
}

}  // namespace

FieldSet leaves(const Value& obj, bool include_status) {
  FieldSet fs;
  collect(obj, "", fs, include_status);
  return fs;
}

const Value* get_path(const Value& root, const std::string& path) {
  const Value* cur = &root;
  Tokens ts(path);
  std::string_view t;
  while (ts.next(t)) {
    if (is_item_token(t)) {
      if (!cur->is_array()) return nullptr;
      long i = find_item(*cur, t);
      if (i < 0) return nullptr;
      cur = &(*cur)[static_cast<size_t>(i)];
    } else {
      cur = cur->find(t);
      if (!cur) return nullptr;
    }
  }
  return cur;
}

bool remove_path(Value& root, const std::string& path) {
  Value* cur = &root;
  Tokens ts(path);
  std::string_view t;
  while (ts.next(t)) {
    const bool last = ts.last();
    if (is_item_token(t)) {
      if (!cur->is_array()) return false;
      long i = find_item(*cur, t);
      if (i < 0) return false;
      if (last) {
        cur->erase_index(static_cast<size_t>(i));
        return true;
      }
      cur = &(*cur)[static_cast<size_t>(i)];
    } else {
      if (last) return cur->erase(t);
      cur = cur->find_mut(t);
      if (!cur) return false;
    }
  }
  return false;
}

void set_path(Value& root, const std::string& path, const Value& v) {
  Value* cur = &root;
  Tokens ts(path);
  std::string_view t;
  while (ts.next(t)) {
    const bool last = ts.last();
    if (is_item_token(t)) {
      if (!cur->is_array()) *cur = Value::array();
      long i = find_item(*cur, t);
      if (i < 0) {
        cur->push_back(last ? v : Value::object());
        cur = &(*cur)[cur->size() - 1];
      } else {
        cur = &(*cur)[static_cast<size_t>(i)];
        if (last) *cur = v;
      }
      continue;
    }
    if (!cur->is_object()) *cur = Value::object();
    if (last) {
      (*cur)[t] = v;
    } else {
      cur = &(*cur)[t];
    }
  }
}

void diff_leaves(const Value& before, const Value& after, FieldSet& changed, FieldSet& removed, bool include_status) {
  FieldSet b = leaves(before, include_status);
  FieldSet a = leaves(after, include_status);
  for (const auto& p : a) {
    const Value* bv = b.count(p) ? get_path(before, p) : nullptr;
    const Value* av = get_path(after, p);
    if (!bv || !av || !(*bv == *av)) changed.insert(p);
  }
  for (const auto& p : b) {
    if (!a.count(p)) removed.insert(p);
  }
}

void diff_member_leaves(const Value& before, const Value& after, const std::string& key, FieldSet& changed,
                        FieldSet& removed) {
  const std::string base = "/" + json::escape_pointer_token(key);
  FieldSet b, a;
  if (const Value* v = before.find(key)) collect(*v, base, b, true);
  if (const Value* v = after.find(key)) collect(*v, base, a, true);
  for (const auto& p : a) {
    const Value* bv = b.count(p) ? get_path(before, p) : nullptr;
    const Value* av = get_path(after, p);
    if (!bv || !av || !(*bv == *av)) changed.insert(p);
  }
  for (const auto& p : b) {
    if (!a.count(p)) removed.insert(p);
  }
}

std::string display_path(const std::string& path) {
  std::string out;
  Tokens ts(path);
  std::string_view t;
  while (ts.next(t)) {
    if (!is_item_token(t)) out += '.';
    out.append(t.data(), t.size());
  }
  return out;
}

Value fields_v1(const FieldSet& fs) {
  Value root = Value::object();
  for (const auto& p : fs) {
    Value* cur = &root;
    Tokens ts(p);
    std::string_view t;
    std::string key;
    while (ts.next(t)) {
      key.clear();
      if (is_item_token(t)) {
        std::string_view inner = t.substr(1, t.size() - 2);
        if (inner.substr(0, 4) == "uid=") key = "k:{\"uid\":" + json::quote(std::string(inner.substr(4))) + "}";
        else key.append("v:").append(inner.substr(1));
      } else {
        key.append("f:").append(t);
      }
      cur = &(*cur)[key];
      if (cur->is_null()) *cur = Value::object();
    }
  }
  return root;
}

}  // namespace bgc::apiserver

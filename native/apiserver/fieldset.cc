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

std::vector<std::string> split(const std::string& path) {
  std::vector<std::string> toks;
  size_t i = 1;
  while (i <= path.size() && !path.empty()) {
    size_t j = path.find('/', i);
    std::string t = path.substr(i, j == std::string::npos ? std::string::npos : j - i);
    // unescape
    std::string u;
    for (size_t k = 0; k < t.size(); ++k) {
      if (t[k] == '~' && k + 1 < t.size()) {
        u.push_back(t[k + 1] == '1' ? '/' : '~');
        ++k;
      } else {
        u.push_back(t[k]);
      }
    }
    toks.push_back(u);
    if (j == std::string::npos) break;
    i = j + 1;
  }
  return toks;
}

bool is_item_token(const std::string& t) { return t.size() >= 3 && t.front() == '[' && t.back() == ']'; }

// index of the list item matching an item token, or -1
long find_item(const Value& arr, const std::string& tok) {
  std::string inner = tok.substr(1, tok.size() - 2);
  if (inner.rfind("uid=", 0) == 0) {
    std::string uid = inner.substr(4);
    for (size_t i = 0; i < arr.size(); ++i) {
      if (arr[i].get_string("uid") == uid) return static_cast<long>(i);
    }
    return -1;
  }
  if (inner.rfind("=", 0) == 0) {
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
  for (const auto& t : split(path)) {
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
  auto toks = split(path);
  if (toks.empty()) return false;
  Value* cur = &root;
  for (size_t k = 0; k + 1 < toks.size(); ++k) {
    const auto& t = toks[k];
    if (is_item_token(t)) {
      if (!cur->is_array()) return false;
      long i = find_item(*cur, t);
      if (i < 0) return false;
      cur = &(*cur)[static_cast<size_t>(i)];
    } else {
      cur = cur->find_mut(t);
      if (!cur) return false;
    }
  }
  const auto& last = toks.back();
  if (is_item_token(last)) {
    if (!cur->is_array()) return false;
    long i = find_item(*cur, last);
    if (i < 0) return false;
    cur->erase_index(static_cast<size_t>(i));
    return true;
  }
  return cur->erase(last);
}

void set_path(Value& root, const std::string& path, const Value& v) {
  auto toks = split(path);
  Value* cur = &root;
  for (size_t k = 0; k < toks.size(); ++k) {
    const auto& t = toks[k];
    bool last = k + 1 == toks.size();
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

std::string display_path(const std::string& path) {
  std::string out;
  for (const auto& t : split(path)) {
    if (is_item_token(t)) out += t;
    else out += "." + t;
  }
  return out;
}

Value fields_v1(const FieldSet& fs) {
  Value root = Value::object();
  for (const auto& p : fs) {
    Value* cur = &root;
    for (const auto& t : split(p)) {
      std::string key;
      if (is_item_token(t)) {
        std::string inner = t.substr(1, t.size() - 2);
        if (inner.rfind("uid=", 0) == 0) key = "k:{\"uid\":" + json::quote(inner.substr(4)) + "}";
        else key = "v:" + inner.substr(1);
      } else {
        key = "f:" + t;
      }
      cur = &(*cur)[key];
      if (cur->is_null()) *cur = Value::object();
    }
  }
  return root;
}

}  // namespace bgc::apiserver

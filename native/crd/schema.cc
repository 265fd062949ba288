#include "crd/schema.h"

#include <cctype>
#include <stdexcept>

#include "core/yaml.h"

namespace bgc::crd {

using json::Value;

const Value& k8s_definitions() {
  static const Value defs = json::parse(kK8sOpenApiDefs);
  return defs;
}

Value inline_refs(const Value& schema) {
  if (schema.is_array()) {
    Value out = Value::array();
    for (const auto& v : schema.items()) out.push_back(inline_refs(v));
    return out;
  }
  if (!schema.is_object()) return schema;
  Value out = Value::object();
  if (const Value* ref = schema.find("$ref")) {
    const Value* target = k8s_definitions().find(ref->as_string());
    if (!target) throw std::runtime_error("unknown schema $ref: " + ref->as_string());
    out = inline_refs(*target);
  }
  const auto& keys = schema.keys();
  const auto& vals = schema.values();
  for (size_t i = 0; i < keys.size(); ++i) {
    if (keys[i] == "$ref") continue;
    out.set(keys[i], inline_refs(vals[i]));
  }
  return out;
}

Value k8s_type_schema(const std::string& name) { return inline_refs(Value::object({{"$ref", name}})); }

namespace {

// kube-derive/schemars modelling of reference src/crd.rs.
Value optional(Value s) {
  s.set("nullable", true);
  return s;
}

Value described(Value s, const std::string& desc) {
  s.set("description", desc);
  return s;
}

Value build_ub_schema() {
  // struct RoleBinding { role_ref: RoleRef, subjects: Option<Vec<Subject>> }  (crd.rs:37-42)
  Value rb = Value::object();
  rb["properties"]["role_ref"] = Value::object({{"$ref", "RoleRef"}});
  rb["properties"]["subjects"] =
      optional(Value::object({{"items", Value::object({{"$ref", "Subject"}})}, {"type", "array"}}));
  rb["required"] = Value::array({"role_ref"});
  rb["type"] = "object";

  // struct UserBootstrapSpec  (crd.rs:19-30); doc comments become descriptions.
  Value spec = Value::object();
  spec["properties"]["kube_username"] =
      optional(described(Value::object({{"type", "string"}}), "Kubernetes username"));
  spec["properties"]["quota"] =
      optional(described(Value::object({{"$ref", "ResourceQuotaSpec"}}), "ResourceQuota in namespace"));
  spec["properties"]["role"] = optional(described(
      Value::object({{"$ref", "Role"}}), "Role in namespace. Optional. If not specified, additional Role is not created."));
  spec["properties"]["rolebinding"] = optional(described(
      rb, "RoleBinding in namespace If not specified, admission controller will create default RoleBinding"));
  spec["type"] = "object";

  // struct UserBootstrapStatus { synchronized_with_sheet: bool }  (crd.rs:32-35)
  Value status = Value::object();
  status["properties"]["synchronized_with_sheet"] = Value::object({{"type", "boolean"}});
  status["required"] = Value::array({"synchronized_with_sheet"});
  status["type"] = "object";

  Value root = Value::object();
  root["description"] = "Auto-generated derived type for UserBootstrapSpec via `CustomResource`";
  root["properties"]["spec"] = spec;
  root["properties"]["status"] = optional(status);
  root["required"] = Value::array({"spec"});
  root["title"] = kKind;
  root["type"] = "object";
  Value out = inline_refs(root);
  out.sort_keys_recursive();
  return out;
}

}  // namespace

const Value& userbootstrap_schema() {
  static const Value s = build_ub_schema();
  return s;
}

Value userbootstrap_crd() {
  Value names = Value::object();
  names["categories"] = Value::array();
  names["kind"] = kKind;
  names["plural"] = kPlural;
  names["shortNames"] = Value::array({kShortName});
  names["singular"] = kSingular;

  Value version = Value::object();
  version["additionalPrinterColumns"] = Value::array();
  version["name"] = kVersion;
  version["schema"]["openAPIV3Schema"] = userbootstrap_schema();
  version["served"] = true;
  version["storage"] = true;
  version["subresources"]["status"] = Value::object();

  Value crd = Value::object();
  crd["apiVersion"] = "apiextensions.k8s.io/v1";
  crd["kind"] = "CustomResourceDefinition";
  crd["metadata"]["name"] = std::string(kPlural) + "." + kGroup;
  crd["spec"]["group"] = kGroup;
  crd["spec"]["names"] = names;
  crd["spec"]["scope"] = "Cluster";
  crd["spec"]["versions"] = Value::array({version});
  crd.sort_keys_recursive();
  return crd;
}

std::string crd_yaml() { return yaml::emit(userbootstrap_crd()); }

// ---------------------------------------------------------------------------
// Validation

bool is_rfc3339(const std::string& s) {
  // YYYY-MM-DDTHH:MM:SS[.frac](Z|+HH:MM|-HH:MM)
  auto dig = [&](size_t i, size_t n) {
    if (i + n > s.size()) return false;
    for (size_t k = 0; k < n; ++k) {
      if (!std::isdigit(static_cast<unsigned char>(s[i + k]))) return false;
    }
    return true;
  };
  if (!dig(0, 4) || s.size() < 20 || s[4] != '-' || !dig(5, 2) || s[7] != '-' || !dig(8, 2)) return false;
  if (s[10] != 'T' && s[10] != 't' && s[10] != ' ') return false;
  if (!dig(11, 2) || s[13] != ':' || !dig(14, 2) || s[16] != ':' || !dig(17, 2)) return false;
  size_t i = 19;
  if (i < s.size() && s[i] == '.') {
    ++i;
    size_t st = i;
    while (i < s.size() && std::isdigit(static_cast<unsigned char>(s[i]))) ++i;
    if (i == st) return false;
  }
  if (i < s.size() && (s[i] == 'Z' || s[i] == 'z')) return i + 1 == s.size();
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) {
    return dig(i + 1, 2) && i + 3 < s.size() && s[i + 3] == ':' && dig(i + 4, 2) && i + 6 == s.size();
  }
  return false;
}

namespace {

bool type_matches(const Value& v, const std::string& t) {
  if (t == "string") return v.is_string();
  if (t == "integer") return v.is_int();
  if (t == "number") return v.is_number();
  if (t == "boolean") return v.is_bool();
  if (t == "object") return v.is_object();
  if (t == "array") return v.is_array();
  return true;
}

// The path of the node being validated, kept as segments and rendered only when an error
// is recorded: building "spec.role.rules[3].verbs" strings for every visited node made the
// walk allocation-bound (admission runs it on every review, reference admission.rs:341-347).
struct PathStack {
  struct Seg {
    std::string_view key;
    size_t index;  // SIZE_MAX: a key segment
  };
  std::vector<Seg> segs;
  std::string render() const {
    std::string out;
    for (const auto& g : segs) {
      if (g.index != SIZE_MAX) {
        out += "[" + std::to_string(g.index) + "]";
      } else {
        if (!out.empty()) out += ".";
        out.append(g.key);
      }
    }
    return out;
  }
  std::string render_with(std::string_view key) const {
    std::string out = render();
    if (!out.empty()) out += ".";
    out.append(key);
    return out;
  }
};

void validate_rec(const Value& v, const Value& s, PathStack& path, const ValidateOptions& opts,
                  std::vector<ValidationError>& errs) {
  if (!s.is_object()) return;
  if (v.is_null()) {
    if (s.get("nullable").is_bool() && s.get("nullable").as_bool()) return;
    // Absent-vs-null: for serde Option<T> fields null is fine; a non-nullable null is
    // a type error.
    const Value& t = s.get("type");
    if (t.is_string()) errs.push_back({path.render(), "null", "expected " + t.as_string()});
    return;
  }
  const Value& t = s.get("type");
  if (t.is_string() && !type_matches(v, t.as_string())) {
    errs.push_back({path.render(), "type", "expected " + t.as_string()});
    return;
  }
  if (const Value* fmt = s.find("format"); fmt && fmt->is_string() && fmt->as_string() == "date-time") {
    if (v.is_string() && !is_rfc3339(v.as_string())) errs.push_back({path.render(), "format", "expected RFC 3339 date-time"});
  }
  if (v.is_object()) {
    const Value& props = s.get("properties");
    if (props.is_object()) {
      const auto& keys = props.keys();
      const auto& vals = props.values();
      for (size_t i = 0; i < keys.size(); ++i) {
        if (const Value* child = v.find(keys[i])) {
          path.segs.push_back({keys[i], SIZE_MAX});
          validate_rec(*child, vals[i], path, opts, errs);
          path.segs.pop_back();
        }
      }
    }
    if (const Value* req = s.find("required"); req && req->is_array()) {
      for (const auto& r : req->items()) {
        const std::string& k = r.as_string();
        if (opts.serde && k == "metadata") continue;
        if (!v.contains(k)) errs.push_back({path.render_with(k), "required", "missing field `" + k + "`"});
      }
    }
    if (const Value* ap = s.find("additionalProperties"); ap && ap->is_object()) {
      const auto& keys = v.keys();
      const auto& vals = v.values();
      for (size_t i = 0; i < keys.size(); ++i) {
        path.segs.push_back({keys[i], SIZE_MAX});
        validate_rec(vals[i], *ap, path, opts, errs);
        path.segs.pop_back();
      }
    }
  } else if (v.is_array()) {
    if (const Value* items = s.find("items")) {
      for (size_t i = 0; i < v.size(); ++i) {
        path.segs.push_back({{}, i});
        validate_rec(v[i], *items, path, opts, errs);
        path.segs.pop_back();
      }
    }
  }
}

const Value* value_at(const Value& root, const std::string& path) {
  // path uses '.' and [i]; keys in this schema never contain dots except map keys,
  // which is fine for error rendering (best effort).
  const Value* cur = &root;
  size_t i = 0;
  while (cur && i < path.size()) {
    if (path[i] == '.') {
      ++i;
      continue;
    }
    if (path[i] == '[') {
      size_t close = path.find(']', i);
      size_t idx = static_cast<size_t>(std::stoul(path.substr(i + 1, close - i - 1)));
      cur = cur->is_array() && idx < cur->size() ? &(*cur)[idx] : nullptr;
      i = close + 1;
      continue;
    }
    size_t end = path.find_first_of(".[", i);
    std::string key = path.substr(i, end == std::string::npos ? std::string::npos : end - i);
    cur = cur->find(key);
    i = end == std::string::npos ? path.size() : end;
  }
  return cur;
}

std::string serde_unexpected(const Value& v) {
  switch (v.type()) {
    case json::Type::Null: return "null";
    case json::Type::Bool: return std::string("boolean `") + (v.as_bool() ? "true" : "false") + "`";
    case json::Type::Int:
    case json::Type::UInt: return "integer `" + v.dump() + "`";
    case json::Type::Double: return "floating point `" + v.dump() + "`";
    case json::Type::String: return "string " + json::quote(v.as_string());
    case json::Type::Array: return "sequence";
    case json::Type::Object: return "map";
  }
  return "value";
}

std::string serde_expected(const std::string& detail) {
  std::string t = detail.rfind("expected ", 0) == 0 ? detail.substr(9) : detail;
  if (t == "string") return "a string";
  if (t == "integer") return "i64";
  if (t == "boolean") return "a boolean";
  if (t == "object") return "struct";
  if (t == "array") return "a sequence";
  if (t == "number") return "f64";
  return t;
}

}  // namespace

std::vector<ValidationError> validate(const Value& value, const Value& schema, const ValidateOptions& opts) {
  std::vector<ValidationError> errs;
  PathStack path;
  validate_rec(value, schema, path, opts, errs);
  return errs;
}

std::string serde_error_message(const Value& value, const ValidationError& e) {
  if (e.kind == "required") return e.detail + " at " + e.path;
  if (e.kind == "format") return "invalid value for " + e.path + ": " + e.detail;
  const Value* v = value_at(value, e.path);
  std::string got = v ? serde_unexpected(*v) : "unit value";
  return "invalid type: " + got + ", expected " + serde_expected(e.detail) + " at " + e.path;
}

UserBootstrapShape inspect_userbootstrap(const Value& obj) {
  if (!obj.is_object()) throw std::runtime_error("invalid type: " + serde_unexpected(obj) + ", expected struct UserBootstrap");
  ValidateOptions o;
  o.serde = true;
  auto errs = validate(obj, userbootstrap_schema(), o);
  if (!errs.empty()) throw std::runtime_error(serde_error_message(obj, errs.front()));
  if (!obj.contains("metadata")) throw std::runtime_error("missing field `metadata`");
  UserBootstrapShape sh;
  const Value& spec = obj.get("spec");
  if (const Value* ku = spec.find("kube_username"); ku && !ku->is_null()) sh.kube_username = &ku->as_string();
  if (const Value* q = spec.find("quota"); q && !q->is_null()) sh.has_quota = true;
  if (const Value* r = spec.find("role"); r && !r->is_null()) sh.has_role = true;
  if (const Value* rb = spec.find("rolebinding"); rb && !rb->is_null()) sh.has_rolebinding = true;
  return sh;
}

UserBootstrap parse_userbootstrap(const Value& obj) {
  (void)inspect_userbootstrap(obj);  // validation (throws)
  UserBootstrap ub;
  ub.raw = obj;
  const Value& meta = obj.get("metadata");
  ub.name = meta.get_string("name");
  ub.uid = meta.get_string("uid");
  ub.resource_version = meta.get_string("resourceVersion");
  const Value& spec = obj.get("spec");
  if (const Value* ku = spec.find("kube_username"); ku && !ku->is_null()) {
    ub.has_kube_username = true;
    ub.kube_username = ku->as_string();
  }
  if (const Value* q = spec.find("quota"); q && !q->is_null()) {
    ub.has_quota = true;
    ub.quota = *q;
  }
  if (const Value* r = spec.find("role"); r && !r->is_null()) {
    ub.has_role = true;
    ub.role = *r;
  }
  if (const Value* rb = spec.find("rolebinding"); rb && !rb->is_null()) {
    ub.has_rolebinding = true;
    ub.rolebinding.role_ref = rb->get("role_ref");
    ub.rolebinding.subjects = rb->get("subjects");
  }
  if (const Value* st = obj.find("status"); st && !st->is_null()) {
    ub.has_status = true;
    ub.synchronized_with_sheet = st->get("synchronized_with_sheet").as_bool();
  }
  return ub;
}

}  // namespace bgc::crd

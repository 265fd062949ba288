#include "admission/policy.h"

#include <algorithm>
#include <iterator>

#include "core/crypto.h"
#include "core/json_patch.h"
#include "core/log.h"
#include "core/trace.h"
#include "core/metrics.h"
#include "crd/schema.h"

namespace bgc::admission {

using json::Value;

Config Config::from_env(const EnvConfig& env) {
  Config c;
  c.listen_addr = env.str("listen_addr");
  c.listen_port = env.u16("listen_port");
  c.cert_path = env.str("cert_path");
  c.key_path = env.str("key_path");
  c.oidc_username_prefix = env.str("oidc_username_prefix");
  c.default_role_name = env.str("default_role_name");
  c.authorized_group_names = env.comma_list("authorized_group_names");
  c.log_full_request = env.boolean_or("log_full_request", true);
  c.cert_reload_interval_secs = env.u64_or("cert_reload_interval_secs", 60);
  c.http2 = env.boolean_or("http2", true);
  c.http2_inline = env.boolean_or("http2_inline", true);
  return c;
}

Username Username::classify(const std::string& username, const std::string& prefix) {
  Username u;
  u.original_username = username;
  if (username.compare(0, prefix.size(), prefix) == 0) {
    u.kube_username = username.substr(prefix.size());
    u.kind = UserKind::Normal;
  } else {
    u.kube_username = username;
    u.kind = UserKind::Admin;
  }
  return u;
}

namespace {

Decision allow(const std::string& uid, int rule) {
  Decision d;
  d.uid = uid;
  d.rule = rule;
  return d;
}

Decision deny(const std::string& uid, const std::string& msg, int rule) {
  LOG_ERROR("admission") << msg;
  Decision d;
  d.uid = uid;
  d.allowed = false;
  d.message = msg;
  d.rule = rule;
  return d;
}

// Q3 fix: the uid is echoed so the apiserver reports a clean rejection
// rather than a webhook protocol error; the outcome (request refused) is unchanged.
Decision invalid(const std::string& uid, const std::string& msg, int rule) {
  LOG_ERROR("admission") << msg;
  Decision d;
  d.uid = uid;
  d.allowed = false;
  d.invalid = true;
  d.message = msg;
  d.rule = rule;
  return d;
}

}  // namespace

Decision mutate(const Value& req, const Config& cfg) {
  const std::string uid = req.get_string("uid");
  const Value& user_info = req.get("userInfo");

  // rule 1: username missing
  const Value& uname = user_info.get("username");
  if (!uname.is_string()) return invalid(uid, "cannot get requester's username from request", 1);
  // rule 2
  Username username = Username::classify(uname.as_string(), cfg.oidc_username_prefix);

  // rule 3: any group in authorized_group_names
  bool is_in_group = false;
  for (const Value& g : user_info.get("groups").items()) {
    if (g.is_string() && std::find(cfg.authorized_group_names.begin(), cfg.authorized_group_names.end(),
                                   g.as_string()) != cfg.authorized_group_names.end()) {
      is_in_group = true;
      break;
    }
  }

  const std::string op = req.get_string("operation");
  if (op == "CREATE") {
    if (username.kind == UserKind::Normal && !is_in_group) return deny(uid, "user is not in authorized group", 4);
  } else if (op == "DELETE") {
    if (username.kind == UserKind::Normal) return deny(uid, "normal user is not allowed to delete resource", 5);
    return allow(uid, 6);
  } else if (op == "UPDATE") {
    if (username.kind == UserKind::Normal) return deny(uid, "normal user is not allowed to update resource", 7);
  } else {
    return invalid(uid, "invalid operation", 8);
  }

  // rule 9: no object
  const Value& obj = req.get("object");
  if (obj.is_null()) return allow(uid, 9);

  // rule 10: resource name
  const Value& name_v = obj.get("metadata").get("name");
  if (!name_v.is_string()) return invalid(uid, "cannot get resource name from request", 10);
  const std::string& resource_name = name_v.as_string();

  // rule 11
  if (username.kind == UserKind::Normal && username.kube_username != resource_name) {
    return deny(uid, "username not match with resource name", 11);
  }

  // rule 12: must parse as UserBootstrap
  crd::UserBootstrapShape ub;
  try {
    ub = crd::inspect_userbootstrap(obj);
  } catch (const std::exception& e) {
    LOG_ERROR("admission") << "Request is not UserBootstrap resource: " << e.what();
    return invalid(uid, e.what(), 12);
  }

  // The patch is written as JSON text: ops in the reference's order, each
  // {"op":...,"path":...,"value":...} as serde_json emits json_patch::PatchOperation.
  std::string patches;
  auto add_op = [&](std::string_view path) {
    patches += patches.empty() ? "[{\"op\":\"add\",\"path\":" : ",{\"op\":\"add\",\"path\":";
    json::escape_string(path, patches);
    patches += ",\"value\":";
  };
  if (username.kind == UserKind::Normal) {
    // rule 13: always (over)write kube_username for normal users
    add_op("/spec/kube_username");
    json::escape_string(username.kube_username, patches);
    patches += '}';
  } else if (!ub.kube_username || ub.kube_username->empty()) {
    // rule 14
    return deny(uid, "kube_username field is empty. you are an admin, so fill it", 14);
  }

  // rule 15
  if (ub.has_quota && username.kind == UserKind::Normal) {
    return deny(uid, "quota field is not empty. you are a normal user, so leave it empty", 15);
  }

  if (!ub.has_rolebinding) {
    // rule 16: default RoleBinding (two ops, exactly as the reference emits them)
    add_op("/spec/rolebinding");
    patches += "{}}";
    const std::string& subject_name =
        username.kind == UserKind::Normal ? username.original_username : *ub.kube_username;
    add_op("/spec/rolebinding");
    patches += "{\"role_ref\":{\"apiGroup\":\"rbac.authorization.k8s.io\",\"kind\":\"ClusterRole\",\"name\":";
    json::escape_string(cfg.default_role_name, patches);
    patches += "},\"subjects\":[{\"apiGroup\":\"rbac.authorization.k8s.io\",\"kind\":\"User\",\"name\":";
    json::escape_string(subject_name, patches);
    patches += "}]}}";
  } else if (username.kind == UserKind::Normal) {
    // rule 17
    return deny(uid, "rolebinding field is not empty. you are a normal user, so leave it empty", 17);
  }

  Decision d = allow(uid, patches.empty() ? 18 : 19);
  if (!patches.empty()) d.patch = std::move(patches) + "]";
  return d;
}

std::string review_response(const Decision& d, const std::string& api_version) {
  std::string out;
  out.reserve(160 + d.uid.size() + d.message.size() + d.patch.size() * 4 / 3);
  out += "{\"apiVersion\":";
  json::escape_string(api_version.empty() ? std::string_view("admission.k8s.io/v1") : std::string_view(api_version), out);
  out += ",\"kind\":\"AdmissionReview\",\"response\":{\"uid\":";
  json::escape_string(d.uid, out);
  out += d.allowed ? ",\"allowed\":true" : ",\"allowed\":false";
  if (!d.allowed) {
    out += d.invalid ? ",\"status\":{\"status\":\"Failure\",\"code\":400,\"reason\":\"BadRequest\",\"message\":"
                     : ",\"status\":{\"message\":";
    json::escape_string(d.message, out);
    out += '}';
  }
  if (!d.patch.empty()) {
    out += ",\"patch\":\"";
    out += crypto::base64_encode(d.patch);  // base64: nothing to escape
    out += "\",\"patchType\":\"JSONPatch\"";
  }
  out += "}}";
  return out;
}

namespace {

// What handle_review and mutate() read from an AdmissionReview (reference
// src/admission.rs:184-431): the request's identity and user, the object's name and the
// parts of a UserBootstrap (spec, status), and only the shape of everything else — the
// request's oldObject and both objects' managedFields are the bulk of an UPDATE review
// and are never looked at.
using P = json::Projection;
const P kObjectMeta[] = {{"name", P::Keep}, {"uid", P::Keep}, {"resourceVersion", P::Keep}};
const P kObject[] = {{"apiVersion", P::Keep}, {"kind", P::Keep}, {"spec", P::Keep}, {"status", P::Keep},
                     {"metadata", P::Descend, kObjectMeta, std::size(kObjectMeta)}};
const P kOldObject[] = {{"metadata", P::Shape}};
const P kRequest[] = {{"uid", P::Keep}, {"operation", P::Keep}, {"userInfo", P::Keep},
                      {"object", P::Descend, kObject, std::size(kObject)},
                      {"oldObject", P::Descend, kOldObject, std::size(kOldObject)}};
const P kReview[] = {{"apiVersion", P::Keep}, {"kind", P::Keep}, {"request", P::Descend, kRequest, std::size(kRequest)}};
const P kReviewRoot{"", P::Descend, kReview, std::size(kReview)};

}  // namespace

HttpResult handle_review(const std::string& body, const std::string& content_type, const Config& cfg) {
  const int64_t t_recv = trace::armed() ? metrics::now_ns() : 0;
  HttpResult r;
  if (content_type.find("application/json") == std::string::npos) {
    r.status = 415;
    r.content_type = "text/plain; charset=utf-8";
    r.body = "Expected request with `Content-Type: application/json`";
    return r;
  }
  Value review;
  std::string err;
  if (!json::try_parse_projected(body, kReviewRoot, review, &err)) {
    r.status = 400;
    r.content_type = "text/plain; charset=utf-8";
    r.body = "Failed to parse the request body as JSON: " + err;
    return r;
  }
  // Shape checks of AdmissionReview<DynamicObject> (kube-core deserialization).
  auto reject = [&](const std::string& why) {
    r.status = 422;
    r.content_type = "text/plain; charset=utf-8";
    r.body = "Failed to deserialize the JSON body into the target type: " + why;
    return r;
  };
  if (!review.is_object()) return reject("invalid type: expected struct AdmissionReview");
  const std::string api_version = review.get_string("apiVersion", "admission.k8s.io/v1");
  const Value& req = review.get("request");
  if (req.is_null()) {
    // try_into() fails -> AdmissionResponse::invalid
    r.decision = invalid("", "request missing in AdmissionReview", 0);
    r.body = review_response(r.decision, api_version);
    return r;
  }
  if (!req.is_object()) return reject("request: invalid type, expected struct AdmissionRequest");
  for (const char* f : {"uid", "kind", "resource", "operation", "userInfo"}) {
    if (!req.contains(f)) return reject(std::string("request: missing field `") + f + "`");
  }
  if (!req.get("uid").is_string()) return reject("request.uid: invalid type, expected a string");
  const std::string op = req.get_string("operation");
  if (op != "CREATE" && op != "UPDATE" && op != "DELETE" && op != "CONNECT") {
    return reject("request.operation: unknown variant `" + op + "`");
  }
  for (const char* f : {"object", "oldObject"}) {
    const Value& o = req.get(f);
    if (!o.is_null() && (!o.is_object() || !o.get("metadata").is_object())) {
      return reject(std::string("request.") + f + ": missing field `metadata`");
    }
  }
  if (cfg.log_full_request) {
    // the request as the API server sent it (raw slice of the body: re-serializing the
    // parsed object cost ~10 % of the webhook's CPU at RUST_LOG=info)
    LOG_INFO("admission") << "received admission request req=" << json::raw_member(body, "request");
  } else {
    LOG_DEBUG("admission") << "received admission request uid=" << req.get_string("uid");
  }
  r.decision = mutate(req, cfg);
  r.body = review_response(r.decision, api_version);
  if (trace::armed()) {
    const Value& o = req.get("object").is_object() ? req.get("object") : req.get("oldObject");
    const std::string name = o.get("metadata").get_string("name");
    trace::mark_at(name, "adm.review0." + op, t_recv);
    trace::mark(name, "adm.review1." + op);
  }
  return r;
}

}  // namespace bgc::admission

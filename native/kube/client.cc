#include "kube/client.h"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <thread>
#include <fstream>

#include "core/crypto.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/net.h"
#include "core/yaml.h"

namespace bgc::kube {

using json::Value;

static const char* kSaDir = "/var/run/secrets/kubernetes.io/serviceaccount";

static bool file_exists(const std::string& p) {
  std::ifstream f(p);
  return f.good();
}

static std::string trim(std::string s) {
  while (!s.empty() && (s.back() == '\n' || s.back() == '\r' || s.back() == ' ')) s.pop_back();
  return s;
}

KubeConfig KubeConfig::in_cluster() {
  const char* host = std::getenv("KUBERNETES_SERVICE_HOST");
  const char* port = std::getenv("KUBERNETES_SERVICE_PORT");
  if (!host || !port) throw std::runtime_error("not running in a cluster (KUBERNETES_SERVICE_HOST unset)");
  KubeConfig c;
  std::string h = host;
  if (h.find(':') != std::string::npos) h = "[" + h + "]";
  c.server = "https://" + h + ":" + port;
  c.token_file = std::string(kSaDir) + "/token";
  c.token = trim(net::read_file(c.token_file));
  c.ca_pem = net::read_file(std::string(kSaDir) + "/ca.crt");
  c.source = "in-cluster";
  return c;
}

static std::string data_or_file(const Value& obj, const std::string& key, const std::string& base_dir) {
  std::string d = obj.get_string(key + "-data");
  if (!d.empty()) return crypto::base64_decode(d);
  std::string f = obj.get_string(key);
  if (f.empty()) return "";
  if (f[0] != '/') f = base_dir + "/" + f;
  return net::read_file(f);
}

KubeConfig KubeConfig::from_kubeconfig(const std::string& path, const std::string& context) {
  Value kc = yaml::parse(net::read_file(path));
  std::string base_dir = path.substr(0, path.rfind('/'));
  std::string ctx_name = context.empty() ? kc.get_string("current-context") : context;
  const Value* ctx = nullptr;
  for (const auto& c : kc.get("contexts").items()) {
    if (c.get_string("name") == ctx_name) ctx = &c.get("context");
  }
  if (!ctx) throw std::runtime_error("kubeconfig: context not found: " + ctx_name);
  std::string cluster_name = ctx->get_string("cluster");
  std::string user_name = ctx->get_string("user");
  KubeConfig c;
  for (const auto& cl : kc.get("clusters").items()) {
    if (cl.get_string("name") != cluster_name) continue;
    const Value& cv = cl.get("cluster");
    c.server = cv.get_string("server");
    c.ca_pem = data_or_file(cv, "certificate-authority", base_dir);
    c.insecure = cv.get("insecure-skip-tls-verify").is_bool() && cv.get("insecure-skip-tls-verify").as_bool();
    c.tls_server_name = cv.get_string("tls-server-name");
  }
  if (c.server.empty()) throw std::runtime_error("kubeconfig: cluster not found: " + cluster_name);
  for (const auto& u : kc.get("users").items()) {
    if (u.get_string("name") != user_name) continue;
    const Value& uv = u.get("user");
    c.token = uv.get_string("token");
    c.token_file = uv.get_string("tokenFile");
    // relative paths in a kubeconfig are relative to the kubeconfig file (client-go)
    if (!c.token_file.empty() && c.token_file[0] != '/') c.token_file = base_dir + "/" + c.token_file;
    if (!c.token_file.empty() && c.token.empty()) c.token = trim(net::read_file(c.token_file));
    c.client_cert_pem = data_or_file(uv, "client-certificate", base_dir);
    c.client_key_pem = data_or_file(uv, "client-key", base_dir);
    c.impersonate_user = uv.get_string("as");
    for (const auto& g : uv.get("as-groups").items()) c.impersonate_groups.push_back(g.as_string());
  }
  c.source = "kubeconfig:" + path;
  return c;
}

KubeConfig KubeConfig::infer() {
  if (const char* s = std::getenv("BGC_KUBE_SERVER")) {
    KubeConfig c;
    c.server = s;
    if (const char* t = std::getenv("BGC_KUBE_TOKEN")) c.token = t;
    if (const char* ca = std::getenv("BGC_KUBE_CA_FILE")) c.ca_pem = net::read_file(ca);
    if (const char* u = std::getenv("BGC_KUBE_AS")) c.impersonate_user = u;
    c.source = "env";
    return c;
  }
  std::string path;
  if (const char* k = std::getenv("KUBECONFIG")) {
    path = k;
    size_t colon = path.find(':');
    if (colon != std::string::npos) path = path.substr(0, colon);
  } else if (const char* home = std::getenv("HOME")) {
    std::string p = std::string(home) + "/.kube/config";
    if (file_exists(p)) path = p;
  }
  if (!path.empty()) return from_kubeconfig(path);
  return in_cluster();
}

// ---------------------------------------------------------------------------

KubeClient::KubeClient(KubeConfig cfg) : cfg_(std::move(cfg)) {
  http::ClientOptions o;
  o.base_url = cfg_.server;
  o.timeout_ms = cfg_.timeout_ms;
  o.tls_server_name = cfg_.tls_server_name;
  o.http2 = cfg_.http2;
  if (cfg_.server.rfind("https", 0) == 0) {
    o.tls = net::TlsContext::client(cfg_.ca_pem, cfg_.insecure, cfg_.client_cert_pem, cfg_.client_key_pem);
  }
  http_ = std::make_unique<http::Client>(o);
  token_ = cfg_.token;
  token_read_ = std::chrono::steady_clock::now();
}

http::Headers KubeClient::auth_headers() {
  http::Headers h;
  std::string tok;
  {
    std::lock_guard<std::mutex> lk(token_mu_);
    auto now = std::chrono::steady_clock::now();
    if (!cfg_.token_file.empty() && now - token_read_ > std::chrono::seconds(60)) {
      try {
        token_ = trim(net::read_file(cfg_.token_file));
      } catch (const std::exception& e) {
        LOG_WARN("kube") << "token refresh failed: " << e.what();
      }
      token_read_ = now;
    }
    tok = token_;
  }
  if (!tok.empty()) h.set("Authorization", "Bearer " + tok);
  if (!cfg_.impersonate_user.empty()) h.set("Impersonate-User", cfg_.impersonate_user);
  for (const auto& g : cfg_.impersonate_groups) h.add("Impersonate-Group", g);
  h.set("Accept", "application/json");
  return h;
}

void throw_api_error(const http::Response& r) {
  Value st;
  std::string reason = http::status_text(r.status);
  std::string msg = r.body;
  if (json::try_parse(r.body, st, nullptr) && st.is_object()) {
    if (st.get("reason").is_string()) reason = st.get_string("reason");
    if (st.get("message").is_string()) msg = st.get_string("message");
  }
  throw ApiError(r.status, reason, msg, st);
}

// Seconds to wait before retrying a throttled response, or -1 when it is not one.
static int retry_after_seconds(const http::Response& r, int cap) {
  const std::string* ra = r.headers.get("Retry-After");
  if (r.status != 429 && !(r.status >= 500 && r.status < 600 && ra)) return -1;
  int secs = 1;
  if (ra && !ra->empty() && std::isdigit(static_cast<unsigned char>((*ra)[0]))) secs = std::atoi(ra->c_str());
  return std::clamp(secs, 0, cap);
}

http::Response KubeClient::raw(const std::string& method, const std::string& path, const std::string& body,
                               const std::string& content_type, const std::string& accept) {
  static auto& throttled = metrics::Registry::global().counter(
      "bgc_kube_client_throttled_total", "Requests the apiserver throttled (429 / Retry-After) and that were retried");
  for (int attempt = 0;; ++attempt) {
    http::Headers h = auth_headers();
    if (!body.empty() || method == "POST" || method == "PUT" || method == "PATCH") h.set("Content-Type", content_type);
    if (!accept.empty()) h.set("Accept", accept);
    http::Response r = http_->request(method, path, body, &h);
    const int wait_s = retry_after_seconds(r, cfg_.max_retry_after_s);
    if (wait_s < 0 || attempt >= cfg_.max_throttle_retries) return r;
    throttled.inc();
    throttled_.fetch_add(1);
    LOG_DEBUG("kube") << method << " " << path << ": " << r.status << ", retrying after " << wait_s << "s";
    std::this_thread::sleep_for(std::chrono::seconds(wait_s));
  }
}

Value KubeClient::call(const std::string& method, const std::string& path, const std::string& body,
                       const std::string& content_type, const std::string& accept) {
  http::Response r = raw(method, path, body, content_type, accept);
  if (r.status < 200 || r.status >= 300) throw_api_error(r);
  if (r.body.empty()) return Value();
  return json::parse(r.body);
}

static std::string with_params(std::string path, const std::vector<std::pair<std::string, std::string>>& ps) {
  bool first = path.find('?') == std::string::npos;
  for (auto& [k, v] : ps) {
    if (v.empty()) continue;
    path += first ? "?" : "&";
    first = false;
    path += k + "=" + http::url_encode(v);
  }
  return path;
}

Value KubeClient::get(const ResourceType& rt, const std::string& ns, const std::string& name) {
  return call("GET", rt.object_path(ns, name));
}

std::optional<Value> KubeClient::get_opt(const ResourceType& rt, const std::string& ns, const std::string& name) {
  http::Response r = raw("GET", rt.object_path(ns, name));
  if (r.status == 404) return std::nullopt;
  if (r.status < 200 || r.status >= 300) throw_api_error(r);
  return json::parse(r.body);
}

Value KubeClient::list(const ResourceType& rt, const std::string& ns, const ListOptions& o) {
  std::string path = with_params(rt.collection_path(ns), {{"labelSelector", o.label_selector},
                                                          {"fieldSelector", o.field_selector},
                                                          {"resourceVersion", o.resource_version},
                                                          {"limit", o.limit ? std::to_string(o.limit) : ""},
                                                          {"continue", o.continue_token}});
  return call("GET", path, "", "application/json", o.metadata_only ? kAcceptMetadataList : "");
}

Value KubeClient::create(const ResourceType& rt, const std::string& ns, const Value& body,
                         const std::string& field_manager) {
  return call("POST", with_params(rt.collection_path(ns), {{"fieldManager", field_manager}}), body.dump());
}

Value KubeClient::replace(const ResourceType& rt, const std::string& ns, const std::string& name, const Value& body,
                          const std::string& field_manager) {
  return call("PUT", with_params(rt.object_path(ns, name), {{"fieldManager", field_manager}}), body.dump());
}

Value KubeClient::replace_status(const ResourceType& rt, const std::string& ns, const std::string& name,
                                 const Value& body) {
  return call("PUT", rt.object_path(ns, name) + "/status", body.dump());
}

Value KubeClient::apply(const ResourceType& rt, const std::string& ns, const std::string& name, const Value& body,
                        const std::string& field_manager, bool force) {
  std::string path =
      with_params(rt.object_path(ns, name), {{"fieldManager", field_manager}, {"force", force ? "true" : ""}});
  return call("PATCH", path, body.dump(), "application/apply-patch+yaml");
}

std::string KubeClient::apply_rv(const ResourceType& rt, const std::string& ns, const std::string& name,
                                 const std::string& body_json, const std::string& field_manager, bool force) {
  std::string path =
      with_params(rt.object_path(ns, name), {{"fieldManager", field_manager}, {"force", force ? "true" : ""}});
  http::Response r = raw("PATCH", path, body_json, "application/apply-patch+yaml");
  if (r.status < 200 || r.status >= 300) throw_api_error(r);
  std::string_view md = json::raw_member(r.body, "metadata");
  if (md.empty()) return "";
  return json::parse(md, "managedFields").get_string("resourceVersion");
}

Value KubeClient::apply_status(const ResourceType& rt, const std::string& ns, const std::string& name,
                               const Value& body, const std::string& field_manager, bool force) {
  std::string path = with_params(rt.object_path(ns, name) + "/status",
                                 {{"fieldManager", field_manager}, {"force", force ? "true" : ""}});
  return call("PATCH", path, body.dump(), "application/apply-patch+yaml");
}

Value KubeClient::patch_json(const ResourceType& rt, const std::string& ns, const std::string& name, const Value& ops,
                             const std::string& field_manager) {
  return call("PATCH", with_params(rt.object_path(ns, name), {{"fieldManager", field_manager}}), ops.dump(),
              "application/json-patch+json");
}

Value KubeClient::patch_merge(const ResourceType& rt, const std::string& ns, const std::string& name,
                              const Value& patch, const std::string& subresource, const std::string& field_manager) {
  std::string path = rt.object_path(ns, name) + (subresource.empty() ? "" : "/" + subresource);
  return call("PATCH", with_params(path, {{"fieldManager", field_manager}}), patch.dump(),
              "application/merge-patch+json");
}

Value KubeClient::remove(const ResourceType& rt, const std::string& ns, const std::string& name,
                         const std::string& propagation) {
  Value opts = Value::object({{"kind", "DeleteOptions"}, {"apiVersion", "v1"}, {"propagationPolicy", propagation}});
  return call("DELETE", rt.object_path(ns, name), opts.dump());
}

std::unique_ptr<http::StreamingResponse> KubeClient::watch(const ResourceType& rt, const std::string& ns,
                                                           const WatchOptions& o) {
  std::string path = with_params(rt.collection_path(ns), {{"watch", "1"},
                                                          {"resourceVersion", o.resource_version},
                                                          {"labelSelector", o.label_selector},
                                                          {"fieldSelector", o.field_selector},
                                                          {"timeoutSeconds", std::to_string(o.timeout_seconds)},
                                                          {"allowWatchBookmarks", o.allow_bookmarks ? "true" : ""},
                                                          {"sendInitialEvents", o.send_initial_events ? "true" : ""},
                                                          {"resourceVersionMatch", o.send_initial_events ? "NotOlderThan" : ""}});
  http::Headers h = auth_headers();
  if (o.metadata_only) h.set("Accept", kAcceptMetadata);
  auto s = http_->stream("GET", path, &h);
  if (s->status < 200 || s->status >= 300) {
    http::Response r;
    r.status = s->status;
    r.body = s->read_all(5000);
    throw_api_error(r);
  }
  return s;
}

}  // namespace bgc::kube

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
#include "core/subprocess.h"
#include "core/yaml.h"

#include <ctime>

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

namespace {

std::string dir_of(const std::string& path) {
  const size_t slash = path.rfind('/');
  return slash == std::string::npos ? "." : path.substr(0, slash);
}

// Merges kubeconfig files: named entries of clusters/contexts/users keep the first
// definition, each tagged with the directory of its file ("__dir").
Value merge_kubeconfigs(const std::vector<std::string>& paths, std::vector<std::string>* loaded) {
  Value merged = Value::object();
  merged["clusters"] = Value::array();
  merged["contexts"] = Value::array();
  merged["users"] = Value::array();
  for (const auto& path : paths) {
    if (path.empty() || !file_exists(path)) continue;
    Value kc = yaml::parse(net::read_file(path));
    if (!kc.is_object()) continue;
    loaded->push_back(path);
    const std::string dir = dir_of(path);
    if (merged.get_string("current-context").empty() && !kc.get_string("current-context").empty()) {
      merged["current-context"] = kc.get_string("current-context");
    }
    for (const char* section : {"clusters", "contexts", "users"}) {
      Value& dst = merged[section];
      for (const auto& e : kc.get(section).items()) {
        const std::string name = e.get_string("name");
        bool seen = false;
        for (const auto& d : dst.items()) seen = seen || d.get_string("name") == name;
        if (seen) continue;
        Value copy = e;
        copy["__dir"] = dir;
        dst.push_back(std::move(copy));
      }
    }
  }
  return merged;
}

const Value* named(const Value& list, const std::string& name, const char* field) {
  for (const auto& e : list.items()) {
    if (e.get_string("name") == name) return &e;
  }
  (void)field;
  return nullptr;
}

}  // namespace

KubeConfig KubeConfig::from_kubeconfig(const std::string& path, const std::string& context) {
  if (!file_exists(path)) throw std::runtime_error("kubeconfig: cannot read " + path);
  return from_kubeconfigs({path}, context);
}

KubeConfig KubeConfig::from_kubeconfigs(const std::vector<std::string>& paths, const std::string& context) {
  std::vector<std::string> loaded;
  Value kc = merge_kubeconfigs(paths, &loaded);
  if (loaded.empty()) throw std::runtime_error("kubeconfig: none of the files exists");
  std::string ctx_name = context.empty() ? kc.get_string("current-context") : context;
  const Value* ctx_entry = named(kc.get("contexts"), ctx_name, "context");
  if (!ctx_entry) throw std::runtime_error("kubeconfig: context not found: " + ctx_name);
  const Value& ctx = ctx_entry->get("context");
  std::string cluster_name = ctx.get_string("cluster");
  std::string user_name = ctx.get_string("user");
  KubeConfig c;
  if (const Value* cl = named(kc.get("clusters"), cluster_name, "cluster")) {
    const Value& cv = cl->get("cluster");
    const std::string dir = cl->get_string("__dir");
    c.server = cv.get_string("server");
    c.ca_pem = data_or_file(cv, "certificate-authority", dir);
    c.insecure = cv.get("insecure-skip-tls-verify").is_bool() && cv.get("insecure-skip-tls-verify").as_bool();
    c.tls_server_name = cv.get_string("tls-server-name");
  }
  if (c.server.empty()) throw std::runtime_error("kubeconfig: cluster not found: " + cluster_name);
  if (const Value* u = named(kc.get("users"), user_name, "user")) {
    const Value& uv = u->get("user");
    const std::string base_dir = u->get_string("__dir");
    c.token = uv.get_string("token");
    c.token_file = uv.get_string("tokenFile");
    // relative paths in a kubeconfig are relative to the kubeconfig file (client-go)
    if (!c.token_file.empty() && c.token_file[0] != '/') c.token_file = base_dir + "/" + c.token_file;
    if (!c.token_file.empty() && c.token.empty()) c.token = trim(net::read_file(c.token_file));
    c.client_cert_pem = data_or_file(uv, "client-certificate", base_dir);
    c.client_key_pem = data_or_file(uv, "client-key", base_dir);
    c.impersonate_user = uv.get_string("as");
    for (const auto& g : uv.get("as-groups").items()) c.impersonate_groups.push_back(g.as_string());
    if (!uv.get_string("username").empty()) c.basic_auth = uv.get_string("username") + ":" + uv.get_string("password");
    const Value& ex = uv.get("exec");
    if (ex.is_object()) {
      ExecPlugin e;
      e.api_version = ex.get_string("apiVersion");
      e.command = ex.get_string("command");
      // a command with a path separator is relative to the kubeconfig (client-go); a bare
      // name is looked up on PATH
      if (e.command.find('/') != std::string::npos && e.command[0] != '/') {
        while (e.command.rfind("./", 0) == 0) e.command.erase(0, 2);
        e.command = base_dir + "/" + e.command;
      }
      for (const auto& a : ex.get("args").items()) e.args.push_back(a.as_string());
      for (const auto& kv : ex.get("env").items()) e.env.emplace_back(kv.get_string("name"), kv.get_string("value"));
      e.provide_cluster_info = ex.get("provideClusterInfo").is_bool() && ex.get("provideClusterInfo").as_bool();
      e.interactive_mode = ex.get_string("interactiveMode");
      e.install_hint = ex.get_string("installHint");
      if (e.command.empty()) throw std::runtime_error("kubeconfig: exec plugin of user " + user_name + " has no command");
      if (e.api_version != "client.authentication.k8s.io/v1" && e.api_version != "client.authentication.k8s.io/v1beta1") {
        throw std::runtime_error("kubeconfig: exec plugin apiVersion " + e.api_version + " is not supported");
      }
      c.exec = std::move(e);
    }
    const Value& ap = uv.get("auth-provider");
    if (ap.is_object()) {
      c.auth_provider = ap.get_string("name");
      c.auth_provider_config = ap.get("config");
      if (c.auth_provider == "oidc") {
        // kube-client 0.84 without its `oidc` feature: the stored id-token, no refresh
        c.token = c.auth_provider_config.get_string("id-token");
        if (c.token.empty()) throw std::runtime_error("kubeconfig: no id-token for the oidc auth-provider");
      } else if (c.auth_provider != "gcp") {
        throw std::runtime_error("kubeconfig: auth-provider " + c.auth_provider + " is not supported");
      }
    }
  }
  c.source = "kubeconfig:";
  for (size_t i = 0; i < loaded.size(); ++i) c.source += (i ? ":" : "") + loaded[i];
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
  if (const char* k = std::getenv("KUBECONFIG"); k && *k) {
    std::vector<std::string> paths;
    std::string v = k;
    size_t start = 0;
    while (true) {
      size_t colon = v.find(':', start);
      paths.push_back(v.substr(start, colon == std::string::npos ? std::string::npos : colon - start));
      if (colon == std::string::npos) break;
      start = colon + 1;
    }
    return from_kubeconfigs(paths);
  }
  if (const char* home = std::getenv("HOME")) {
    std::string p = std::string(home) + "/.kube/config";
    if (file_exists(p)) return from_kubeconfig(p);
  }
  return in_cluster();
}

// ---------------------------------------------------------------------------

std::shared_ptr<http::Client> KubeClient::make_http(const KubeConfig& cfg) {
  http::ClientOptions o;
  o.base_url = cfg.server;
  o.timeout_ms = cfg.timeout_ms;
  o.tls_server_name = cfg.tls_server_name;
  // BGC_KUBE_HTTP2=1: request/response calls multiplexed over one HTTP/2 connection
  const char* h2 = std::getenv("BGC_KUBE_HTTP2");
  o.http2 = cfg.http2 || (h2 && std::string(h2) == "1");
  if (cfg.server.rfind("https", 0) == 0) {
    o.tls = net::TlsContext::client(cfg.ca_pem, cfg.insecure, cfg.client_cert_pem, cfg.client_key_pem);
  }
  return std::make_shared<http::Client>(o);
}

KubeClient::KubeClient(KubeConfig cfg) : cfg_(std::move(cfg)) {
  // an exec plugin may hand out a client certificate instead of (or with) a token: it has
  // to be known before the first TLS context is built
  if (cfg_.exec && cfg_.client_cert_pem.empty()) plugin_token(true);
  http_ = make_http(cfg_);
  if (!has_plugin()) token_ = cfg_.token;
  token_read_ = std::chrono::steady_clock::now();
}

KubeConfig KubeClient::config() const {
  std::lock_guard<std::mutex> lk(token_mu_);
  return cfg_;
}

std::shared_ptr<http::Client> KubeClient::http() const {
  std::lock_guard<std::mutex> lk(http_mu_);
  return http_;
}

namespace {

// RFC 3339 timestamp -> system_clock (false when malformed)
bool parse_rfc3339(const std::string& s, std::chrono::system_clock::time_point* out) {
  int Y, M, D, h, m, sec;
  if (std::sscanf(s.c_str(), "%d-%d-%dT%d:%d:%d", &Y, &M, &D, &h, &m, &sec) != 6) return false;
  std::tm tm{};
  tm.tm_year = Y - 1900;
  tm.tm_mon = M - 1;
  tm.tm_mday = D;
  tm.tm_hour = h;
  tm.tm_min = m;
  tm.tm_sec = sec;
  time_t t = timegm(&tm);
  size_t i = 19;
  if (i < s.size() && s[i] == '.') {
    ++i;
    while (i < s.size() && std::isdigit(static_cast<unsigned char>(s[i]))) ++i;
  }
  if (i < s.size() && (s[i] == '+' || s[i] == '-') && i + 5 < s.size() + 1) {
    int oh = 0, om = 0;
    if (std::sscanf(s.c_str() + i + 1, "%d:%d", &oh, &om) == 2) {
      const long off = (oh * 3600L + om * 60L) * (s[i] == '+' ? 1 : -1);
      t -= off;
    }
  }
  *out = std::chrono::system_clock::from_time_t(t);
  return true;
}

// "{.credential.access_token}" -> value at that path of `v` (gcp auth-provider keys)
std::string json_path_string(const Value& v, std::string key) {
  if (!key.empty() && key.front() == '{') key = key.substr(1);
  if (!key.empty() && key.back() == '}') key.pop_back();
  const Value* cur = &v;
  size_t start = key.empty() || key[0] != '.' ? 0 : 1;
  while (cur && start <= key.size()) {
    size_t dot = key.find('.', start);
    std::string part = key.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
    if (!part.empty()) cur = cur->find(part);
    if (dot == std::string::npos) break;
    start = dot + 1;
  }
  return cur && cur->is_string() ? cur->as_string() : "";
}

}  // namespace

std::string KubeClient::plugin_token(bool force) {
  std::lock_guard<std::mutex> lk(token_mu_);
  const auto now = std::chrono::system_clock::now();
  if (!force && plugin_fetched_ && now + std::chrono::seconds(10) < token_expiry_) return token_;
  static auto& refreshes = metrics::Registry::global().counter(
      "bgc_kube_client_credential_refreshes_total", "Credentials fetched from a kubeconfig exec plugin or auth-provider");
  if (cfg_.exec) {
    const auto& e = *cfg_.exec;
    // services run without a terminal: a plugin that must prompt cannot run (client-go
    // refuses the same way when stdin is not a terminal)
    if (e.interactive_mode == "Always") {
      throw std::runtime_error("exec credential plugin " + e.command +
                               " requires interactive mode (interactiveMode: Always), but standard input is not a terminal");
    }
    Value info = Value::object({{"apiVersion", e.api_version}, {"kind", "ExecCredential"}});
    Value spec = Value::object({{"interactive", false}});
    if (e.provide_cluster_info) {
      Value cluster = Value::object({{"server", cfg_.server}});
      if (!cfg_.ca_pem.empty()) cluster["certificate-authority-data"] = crypto::base64_encode(cfg_.ca_pem);
      if (cfg_.insecure) cluster["insecure-skip-tls-verify"] = true;
      if (!cfg_.tls_server_name.empty()) cluster["tls-server-name"] = cfg_.tls_server_name;
      spec["cluster"] = cluster;
    }
    info["spec"] = spec;
    std::vector<std::string> argv{e.command};
    argv.insert(argv.end(), e.args.begin(), e.args.end());
    auto env = e.env;
    env.emplace_back("KUBERNETES_EXEC_INFO", info.dump());
    RunResult r = run_command(argv, env, cfg_.exec_timeout_ms);
    if (r.exit_code != 0) {
      std::string msg = "exec credential plugin " + e.command + " failed (" +
                        (r.timed_out ? std::string("timed out") : "exit " + std::to_string(r.exit_code)) +
                        "): " + r.err.substr(0, 500);
      if (r.err.rfind("cannot run ", 0) == 0 && !e.install_hint.empty()) msg += "\n" + e.install_hint;
      throw std::runtime_error(msg);
    }
    Value cred;
    std::string perr;
    if (!json::try_parse(r.out, cred, &perr)) throw std::runtime_error("exec credential plugin output: " + perr);
    if (cred.get_string("kind") != "ExecCredential" || cred.get_string("apiVersion") != e.api_version) {
      throw std::runtime_error("exec credential plugin returned " + cred.get_string("apiVersion") + " " +
                               cred.get_string("kind") + ", expected " + e.api_version + " ExecCredential");
    }
    const Value& st = cred.get("status");
    token_ = st.get_string("token");
    const std::string cert = st.get_string("clientCertificateData"), key = st.get_string("clientKeyData");
    if (!cert.empty() && (cert != cfg_.client_cert_pem || key != cfg_.client_key_pem)) {
      cfg_.client_cert_pem = cert;
      cfg_.client_key_pem = key;
      // a new client certificate: new connections must present it, so the TLS context
      // and the connection pool are rebuilt (not at construction: no client exists yet)
      std::lock_guard<std::mutex> hl(http_mu_);
      if (http_) {
        http_ = make_http(cfg_);
        tls_rebuilds_.fetch_add(1);
        LOG_INFO("kube") << "exec credential plugin rotated the client certificate; TLS context rebuilt";
      }
    }
    if (token_.empty() && cfg_.client_cert_pem.empty()) {
      throw std::runtime_error("exec credential plugin returned neither a token nor a client certificate");
    }
    token_expiry_ = std::chrono::system_clock::time_point::max();
    if (!st.get_string("expirationTimestamp").empty() && !parse_rfc3339(st.get_string("expirationTimestamp"), &token_expiry_)) {
      throw std::runtime_error("exec credential plugin: bad expirationTimestamp " + st.get_string("expirationTimestamp"));
    }
  } else {  // gcp auth-provider
    const Value& pc = cfg_.auth_provider_config;
    std::chrono::system_clock::time_point exp = std::chrono::system_clock::time_point::max();
    const bool has_exp = !pc.get_string("expiry").empty() && parse_rfc3339(pc.get_string("expiry"), &exp);
    const std::string cached = pc.get_string("access-token");
    if (!force && !plugin_fetched_ && !cached.empty() && (!has_exp || now + std::chrono::seconds(10) < exp)) {
      token_ = cached;
      token_expiry_ = exp;
    } else {
      const std::string cmd = pc.get_string("cmd-path");
      if (cmd.empty()) throw std::runtime_error("gcp auth-provider: token expired and no cmd-path to refresh it");
      std::vector<std::string> argv{cmd};
      std::string args = pc.get_string("cmd-args");
      size_t start = 0;
      while (start < args.size()) {
        size_t sp = args.find(' ', start);
        std::string a = args.substr(start, sp == std::string::npos ? std::string::npos : sp - start);
        if (!a.empty()) argv.push_back(a);
        if (sp == std::string::npos) break;
        start = sp + 1;
      }
      RunResult r = run_command(argv, {}, cfg_.exec_timeout_ms);
      if (r.exit_code != 0) throw std::runtime_error("gcp auth-provider command failed: " + r.err.substr(0, 500));
      Value out = json::parse(r.out);
      const std::string tk = pc.get_string("token-key").empty() ? "{.access_token}" : pc.get_string("token-key");
      token_ = json_path_string(out, tk);
      if (token_.empty()) throw std::runtime_error("gcp auth-provider: no token at " + tk);
      token_expiry_ = std::chrono::system_clock::time_point::max();
      const std::string ek = pc.get_string("expiry-key");
      if (!ek.empty()) parse_rfc3339(json_path_string(out, ek), &token_expiry_);
    }
  }
  plugin_fetched_ = true;
  credential_refreshes_.fetch_add(1);
  refreshes.inc();
  return token_;
}

http::Headers KubeClient::auth_headers() {
  http::Headers h;
  std::string tok;
  if (has_plugin()) {
    tok = plugin_token(false);
  } else {
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
  else if (!cfg_.basic_auth.empty()) h.set("Authorization", "Basic " + crypto::base64_encode(cfg_.basic_auth));
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
    http::Response r = http()->request(method, path, body, &h);
    if (r.status == 401 && has_plugin() && attempt == 0) {
      // the plugin's credential was revoked or rotated early: fetch a fresh one, retry once
      LOG_INFO("kube") << method << " " << path << ": 401, refreshing the plugin credential";
      plugin_token(true);
      continue;
    }
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

namespace {
std::string response_rv(const http::Response& r) {
  // only metadata.resourceVersion is needed: located by scanning, no tree built
  std::string_view md = json::raw_member(r.body, "metadata");
  if (md.empty()) return "";
  std::string_view rv = json::raw_member(md, "resourceVersion");
  if (rv.size() >= 2 && rv.front() == '"' && rv.back() == '"' && rv.find('\\') == std::string_view::npos) {
    return std::string(rv.substr(1, rv.size() - 2));
  }
  if (rv.empty()) return "";
  const Value v = json::parse(rv);
  return v.is_string() ? v.as_string() : "";
}
}  // namespace

std::string KubeClient::replace_status_rv(const ResourceType& rt, const std::string& ns, const std::string& name,
                                          const Value& body) {
  http::Response r = raw("PUT", rt.object_path(ns, name) + "/status", body.dump(), "application/json");
  if (r.status < 200 || r.status >= 300) throw_api_error(r);
  return response_rv(r);
}

std::string KubeClient::patch_json_rv(const ResourceType& rt, const std::string& ns, const std::string& name,
                                      const Value& ops, const std::string& field_manager) {
  http::Response r = raw("PATCH", with_params(rt.object_path(ns, name), {{"fieldManager", field_manager}}), ops.dump(),
                         "application/json-patch+json");
  if (r.status < 200 || r.status >= 300) throw_api_error(r);
  return response_rv(r);
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
  // only metadata.resourceVersion is needed: located by scanning, no tree built
  std::string_view md = json::raw_member(r.body, "metadata");
  if (md.empty()) return "";
  std::string_view rv = json::raw_member(md, "resourceVersion");
  if (rv.size() >= 2 && rv.front() == '"' && rv.back() == '"' && rv.find('\\') == std::string_view::npos) {
    return std::string(rv.substr(1, rv.size() - 2));
  }
  if (rv.empty()) return "";
  const Value v = json::parse(rv);
  return v.is_string() ? v.as_string() : "";
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

void KubeClient::reset_connections() {
  if (auto h = http()) h->close_idle();
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
  auto s = http()->stream("GET", path, &h);
  if (s->status < 200 || s->status >= 300) {
    http::Response r;
    r.status = s->status;
    r.body = s->read_all(5000);
    throw_api_error(r);
  }
  return s;
}

}  // namespace bgc::kube

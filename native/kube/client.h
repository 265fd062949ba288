// Kubernetes API client: config inference + typed REST verbs (kube-client 0.84
// equivalent; reference uses `Client::try_default()` at src/controller.rs:224 and
// src/synchronizer.rs:392, `PatchParams::apply(..).force()` at src/controller.rs:67,
// `replace_status` at src/synchronizer.rs:302, JSON patch at :323-330).
#pragma once

#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "core/http.h"
#include "core/json.h"
#include "kube/resource.h"

namespace bgc::kube {

struct KubeConfig {
  std::string server;           // https://10.96.0.1:443 or http://127.0.0.1:port
  std::string token;            // bearer token (static)
  std::string token_file;       // re-read periodically (bound SA tokens rotate)
  std::string ca_pem;
  std::string client_cert_pem;
  std::string client_key_pem;
  bool insecure = false;
  std::string tls_server_name;
  std::string impersonate_user;
  std::vector<std::string> impersonate_groups;
  // users[].user.exec: a credential plugin (client.authentication.k8s.io ExecCredential
  // v1 / v1beta1) run as a child process; its token is cached until its
  // expirationTimestamp and re-fetched on a 401 (client-go / kube-client behaviour).
  struct ExecPlugin {
    std::string api_version;
    std::string command;
    std::vector<std::string> args;
    std::vector<std::pair<std::string, std::string>> env;
    bool provide_cluster_info = false;
    std::string interactive_mode;  // Never | IfAvailable | Always ("" = IfAvailable)
    std::string install_hint;      // shown when the command cannot be run
  };
  std::optional<ExecPlugin> exec;
  // users[].user.auth-provider (kube-client 0.84 without its oidc feature): "oidc" uses the
  // stored id-token; "gcp" uses access-token until expiry, then runs cmd-path.
  std::string auth_provider;
  json::Value auth_provider_config;
  std::string basic_auth;       // users[].user.username:password
  int exec_timeout_ms = 30000;
  int timeout_ms = 30000;
  // https: offer HTTP/2 and multiplex request/response calls on one connection, as
  // client-go does (watches keep their own HTTP/1.1 streams).
  bool http2 = false;
  // Throttling (HTTP 429, or 5xx with Retry-After): wait as the server asks — capped at
  // max_retry_after_s, 1 s when no header — and retry up to this many times (client-go
  // retries 429 with Retry-After up to 10 times).  0 = surface the error at once.
  int max_throttle_retries = 10;
  int max_retry_after_s = 10;
  std::string source;           // "in-cluster" | "kubeconfig:<path>" | "env"

  // Inference order (kube-client `Config::infer`): $BGC_KUBE_SERVER override (tests),
  // $KUBECONFIG / ~/.kube/config, then the in-cluster service account.
  static KubeConfig infer();
  static KubeConfig in_cluster();
  static KubeConfig from_kubeconfig(const std::string& path, const std::string& context = "");
  // $KUBECONFIG with several files: merged as client-go merges them — the first file that
  // defines a cluster, context or user name wins, and so does the first current-context;
  // relative paths stay relative to the file that defined the entry.
  static KubeConfig from_kubeconfigs(const std::vector<std::string>& paths, const std::string& context = "");
};

class ApiError : public std::runtime_error {
 public:
  ApiError(int code, std::string reason, const std::string& message, json::Value status = {})
      : std::runtime_error("ApiError(" + std::to_string(code) + " " + reason + "): " + message),
        code_(code), reason_(std::move(reason)), message_(message), status_(std::move(status)) {}
  int code() const { return code_; }
  const std::string& reason() const { return reason_; }
  const std::string& message() const { return message_; }
  const json::Value& status() const { return status_; }

 private:
  int code_;
  std::string reason_;
  std::string message_;
  json::Value status_;
};

// metadata_only: ask for PartialObjectMetadata(List) (meta.k8s.io/v1) instead of the full
// objects, as client-go's metadata informers and kube-rs' metadata_watcher do: the apiserver
// sends only each object's metadata.
struct ListOptions {
  std::string label_selector;
  std::string field_selector;
  std::string resource_version;
  int64_t limit = 0;
  std::string continue_token;
  bool metadata_only = false;
};

struct WatchOptions {
  std::string resource_version;
  std::string label_selector;
  std::string field_selector;
  int timeout_seconds = 290;
  bool allow_bookmarks = true;
  // Streaming list: replay the current state as ADDED events, ended by a BOOKMARK
  // annotated k8s.io/initial-events-end (sendInitialEvents + resourceVersionMatch).
  bool send_initial_events = false;
  bool metadata_only = false;  // events carry PartialObjectMetadata
};

// Accept headers of metadata-only requests (with a plain-JSON fallback, as client-go sends).
constexpr const char kAcceptMetadataList[] =
    "application/json;as=PartialObjectMetadataList;g=meta.k8s.io;v=v1,application/json";
constexpr const char kAcceptMetadata[] =
    "application/json;as=PartialObjectMetadata;g=meta.k8s.io;v=v1,application/json";

class KubeClient {
 public:
  explicit KubeClient(KubeConfig cfg);

  json::Value get(const ResourceType& rt, const std::string& ns, const std::string& name);
  std::optional<json::Value> get_opt(const ResourceType& rt, const std::string& ns, const std::string& name);
  json::Value list(const ResourceType& rt, const std::string& ns = "", const ListOptions& opts = {});
  json::Value create(const ResourceType& rt, const std::string& ns, const json::Value& body,
                     const std::string& field_manager = "");
  json::Value replace(const ResourceType& rt, const std::string& ns, const std::string& name, const json::Value& body,
                      const std::string& field_manager = "");
  // The same writes returning only the written object's resourceVersion: the response is
  // not parsed beyond metadata (managedFields skipped), for callers that need nothing else.
  std::string replace_status_rv(const ResourceType& rt, const std::string& ns, const std::string& name,
                                const json::Value& body);
  std::string patch_json_rv(const ResourceType& rt, const std::string& ns, const std::string& name,
                            const json::Value& ops, const std::string& field_manager = "");
  json::Value replace_status(const ResourceType& rt, const std::string& ns, const std::string& name,
                             const json::Value& body);
  // Server-side apply (application/apply-patch+yaml; JSON is valid YAML).
  json::Value apply(const ResourceType& rt, const std::string& ns, const std::string& name, const json::Value& body,
                    const std::string& field_manager, bool force);
  json::Value apply_status(const ResourceType& rt, const std::string& ns, const std::string& name,
                           const json::Value& body, const std::string& field_manager, bool force);
  // Server-side apply of an already serialized body, for callers that only need the
  // result's resourceVersion: only the response's `metadata` (minus managedFields) is
  // parsed, not the whole object.
  std::string apply_rv(const ResourceType& rt, const std::string& ns, const std::string& name,
                       const std::string& body_json, const std::string& field_manager, bool force);
  json::Value patch_json(const ResourceType& rt, const std::string& ns, const std::string& name,
                         const json::Value& ops, const std::string& field_manager = "");
  json::Value patch_merge(const ResourceType& rt, const std::string& ns, const std::string& name,
                          const json::Value& patch, const std::string& subresource = "",
                          const std::string& field_manager = "");
  json::Value remove(const ResourceType& rt, const std::string& ns, const std::string& name,
                     const std::string& propagation = "Background");
  std::unique_ptr<http::StreamingResponse> watch(const ResourceType& rt, const std::string& ns,
                                                 const WatchOptions& opts);

  // Low level: throws ApiError on non-2xx.
  json::Value call(const std::string& method, const std::string& path, const std::string& body = "",
                   const std::string& content_type = "application/json", const std::string& accept = "");
  http::Response raw(const std::string& method, const std::string& path, const std::string& body = "",
                     const std::string& content_type = "application/json", const std::string& accept = "");
  // A snapshot: an exec plugin's refresh may replace the client certificate at any time.
  KubeConfig config() const;
  // Drops every pooled idle connection (a watch found the path to the apiserver dead).
  void reset_connections();
  uint64_t tls_rebuilds() const { return tls_rebuilds_.load(); }
  uint64_t throttled() const { return throttled_.load(); }
  uint64_t credential_refreshes() const { return credential_refreshes_.load(); }

 private:
  http::Headers auth_headers();
  // Token from the exec plugin / gcp auth-provider, refreshed when expired or `force`d.
  std::string plugin_token(bool force);
  bool has_plugin() const { return cfg_.exec.has_value() || cfg_.auth_provider == "gcp"; }
  // An HTTP client for the current credentials (TLS client certificate included).
  static std::shared_ptr<http::Client> make_http(const KubeConfig& cfg);
  std::shared_ptr<http::Client> http() const;
  KubeConfig cfg_;  // client_cert/key under token_mu_ (exec plugin refreshes)
  // Replaced when an exec plugin hands out a new client certificate (client-go rotates
  // its TLS certificate the same way): requests in flight finish on the old client.
  std::shared_ptr<http::Client> http_;
  mutable std::mutex http_mu_;
  std::atomic<uint64_t> tls_rebuilds_{0};
  mutable std::mutex token_mu_;
  std::string token_;
  std::chrono::steady_clock::time_point token_read_{};
  std::chrono::system_clock::time_point token_expiry_ = std::chrono::system_clock::time_point::max();
  bool plugin_fetched_ = false;
  std::atomic<uint64_t> throttled_{0};
  std::atomic<uint64_t> credential_refreshes_{0};
};

// Raises ApiError for a non-2xx response (parsing a metav1.Status body when present).
[[noreturn]] void throw_api_error(const http::Response& r);

}  // namespace bgc::kube

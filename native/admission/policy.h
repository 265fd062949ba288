// UserBootstrap admission policy (mutating + validating), a pure function.
//
// Reference: src/admission.rs:206-431 (Username classifier + mutate()), decision
// table reproduced in SURVEY.md §3.2.  Rule numbers in comments refer to that table.
#pragma once

#include <string>
#include <vector>

#include "core/env_config.h"
#include "core/json.h"

namespace bgc::admission {

struct Config {
  std::string listen_addr = "0.0.0.0";
  uint16_t listen_port = 12321;
  std::string cert_path;
  std::string key_path;
  std::string oidc_username_prefix = "oidc:";
  std::string default_role_name = "edit";
  std::vector<std::string> authorized_group_names{"gpu", "admin"};
  // Additions (not in the reference): request logging detail and cert poll period.
  bool log_full_request = true;          // reference logs the full request (admission.rs:199)
  uint64_t cert_reload_interval_secs = 60;  // admission.rs:112
  bool http2 = true;  // ALPN h2 + http/1.1, as axum-server's rustls acceptor (admission.rs:141)
  // h2: run /mutate on the connection reader when the connection has nothing else in
  // flight (no worker hand-off; profiles/admission_h2_inline_r3/)
  bool http2_inline = true;

  // envy semantics: every reference field is required (admission.rs:22-39).
  static Config from_env(const EnvConfig& env);
};

enum class UserKind { Normal, Admin };

struct Username {
  std::string original_username;
  std::string kube_username;
  UserKind kind = UserKind::Admin;
  // admission.rs:217-238: prefix => Normal (prefix stripped), otherwise Admin.
  static Username classify(const std::string& username, const std::string& prefix);
};

struct Decision {
  std::string uid;
  bool allowed = true;
  bool invalid = false;       // AdmissionResponse::invalid (malformed request)
  std::string message;        // deny / invalid reason
  std::string patch;          // JSON Patch ops (a JSON array's text), empty for none
  int rule = 0;               // which decision-table row fired (observability/tests)
};

// Applies the policy to an AdmissionRequest object (the `request` member of an
// AdmissionReview).
Decision mutate(const json::Value& request, const Config& cfg);

// Full HTTP-level handling of a POST /mutate body. Returns the HTTP status and body.
// 400/415/422 mirror axum's Json extractor rejections for bodies that are not
// AdmissionReviews at all.
struct HttpResult {
  int status = 200;
  std::string body;
  std::string content_type = "application/json";
  Decision decision;
};
HttpResult handle_review(const std::string& body, const std::string& content_type, const Config& cfg);

// AdmissionReview{response} JSON for a decision. `api_version` echoes the request's.
// The AdmissionReview response document's JSON text (written directly: the webhook answers
// every UserBootstrap write, and building and dumping a Value tree was its largest cost).
std::string review_response(const Decision& d, const std::string& api_version);

}  // namespace bgc::admission

// Google service-account OAuth2 (JWT bearer grant, RS256) and Drive v3 export, without
// an SDK.  Replaces yup-oauth2 8.1 ServiceAccountAuthenticator + google-drive3 5.0
// `files().export(id, "text/csv")` (reference src/synchronizer.rs:178-206).
//
// Endpoints can be redirected for tests only: BGC_GOOGLE_TOKEN_URL, BGC_GOOGLE_API_BASE
// (and BGC_GOOGLE_CA_FILE to trust a test CA).  In production the reference's
// https-only connector with native roots is mirrored.
#pragma once

#include <chrono>
#include <memory>
#include <mutex>
#include <string>

#include "core/http.h"
#include "core/json.h"

namespace bgc::sync {

struct ServiceAccountKey {
  std::string client_email;
  std::string private_key;      // PEM
  std::string private_key_id;
  std::string token_uri = "https://oauth2.googleapis.com/token";
  std::string project_id;
  static ServiceAccountKey from_json(const json::Value& v);
  static ServiceAccountKey from_file(const std::string& path);
};

class GoogleAuth {
 public:
  GoogleAuth(ServiceAccountKey key, std::string scope);
  // Cached token, refreshed 60 s before expiry.
  std::string token();
  // The signed assertion (exposed for tests).
  std::string make_assertion(int64_t now_unix) const;
  uint64_t fetches() const { return fetches_; }

 private:
  ServiceAccountKey key_;
  std::string scope_;
  std::string token_url_;
  std::mutex mu_;
  std::string token_;
  std::chrono::steady_clock::time_point expiry_{};
  uint64_t fetches_ = 0;
  std::shared_ptr<net::TlsContext> tls_;
};

class GoogleApiError : public std::runtime_error {
 public:
  GoogleApiError(int status, const std::string& msg) : std::runtime_error(msg), status_(status) {}
  int status() const { return status_; }

 private:
  int status_;
};

class DriveClient {
 public:
  explicit DriveClient(GoogleAuth& auth);
  // GET /drive/v3/files/{id}/export?mimeType=... ; throws GoogleApiError on non-2xx
  // ("request failed", synchronizer.rs:202-204) and on non-UTF-8 bodies.
  std::string export_file(const std::string& file_id, const std::string& mime = "text/csv");
  // GET /drive/v3/files/{id}?fields=version: Drive bumps `version` on every change to the
  // file, so polling this metadata call (a few hundred bytes) tells when an export is
  // worth doing.  Returns the version string; throws GoogleApiError on non-2xx.
  std::string file_version(const std::string& file_id);

 private:
  GoogleAuth& auth_;
  std::unique_ptr<http::Client> http_;
  std::string base_path_;
};

bool valid_utf8(const std::string& s);

constexpr const char* kDriveReadonlyScope = "https://www.googleapis.com/auth/drive.readonly";

}  // namespace bgc::sync

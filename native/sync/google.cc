#include "sync/google.h"

#include <cstdlib>

#include "core/crypto.h"
#include "core/log.h"
#include "core/net.h"

namespace bgc::sync {

using json::Value;

ServiceAccountKey ServiceAccountKey::from_json(const Value& v) {
  ServiceAccountKey k;
  k.client_email = v.get_string("client_email");
  k.private_key = v.get_string("private_key");
  k.private_key_id = v.get_string("private_key_id");
  k.project_id = v.get_string("project_id");
  std::string t = v.get_string("token_uri");
  if (!t.empty()) k.token_uri = t;
  if (k.client_email.empty() || k.private_key.empty()) {
    throw std::runtime_error("invalid service account key: client_email/private_key missing");
  }
  return k;
}

ServiceAccountKey ServiceAccountKey::from_file(const std::string& path) {
  return from_json(json::parse(net::read_file(path)));
}

static std::shared_ptr<net::TlsContext> test_tls() {
  if (const char* ca = std::getenv("BGC_GOOGLE_CA_FILE")) return net::TlsContext::client(net::read_file(ca), false);
  return nullptr;
}

GoogleAuth::GoogleAuth(ServiceAccountKey key, std::string scope) : key_(std::move(key)), scope_(std::move(scope)) {
  const char* override_url = std::getenv("BGC_GOOGLE_TOKEN_URL");
  token_url_ = override_url ? override_url : key_.token_uri;
  tls_ = test_tls();
}

std::string GoogleAuth::make_assertion(int64_t now) const {
  Value header = Value::object({{"alg", "RS256"}, {"typ", "JWT"}});
  if (!key_.private_key_id.empty()) header["kid"] = key_.private_key_id;
  Value claims = Value::object({{"iss", key_.client_email},
                                {"scope", scope_},
                                {"aud", key_.token_uri},
                                {"exp", static_cast<long long>(now + 3600)},
                                {"iat", static_cast<long long>(now)}});
  return crypto::jwt_rs256(header.dump(), claims.dump(), key_.private_key);
}

std::string GoogleAuth::token() {
  std::lock_guard<std::mutex> lk(mu_);
  auto now = std::chrono::steady_clock::now();
  if (!token_.empty() && now + std::chrono::seconds(60) < expiry_) return token_;
  int64_t unix_now = std::chrono::duration_cast<std::chrono::seconds>(std::chrono::system_clock::now().time_since_epoch()).count();
  std::string body = "grant_type=" + http::url_encode("urn:ietf:params:oauth:grant-type:jwt-bearer") +
                     "&assertion=" + http::url_encode(make_assertion(unix_now));
  http::Headers h;
  h.set("Content-Type", "application/x-www-form-urlencoded");
  http::Response r = http::fetch("POST", token_url_, body, &h, tls_, 30000);
  ++fetches_;
  if (r.status < 200 || r.status >= 300) {
    throw GoogleApiError(r.status, "google auth error: token endpoint returned " + std::to_string(r.status) + ": " + r.body);
  }
  Value v = json::parse(r.body);
  token_ = v.get_string("access_token");
  if (token_.empty()) throw GoogleApiError(r.status, "google auth error: no access_token in response");
  int64_t expires = v.get("expires_in").is_int() ? v.get("expires_in").as_int() : 3600;
  expiry_ = now + std::chrono::seconds(expires);
  return token_;
}

DriveClient::DriveClient(GoogleAuth& auth) : auth_(auth) {
  const char* base = std::getenv("BGC_GOOGLE_API_BASE");
  std::string url = base ? base : "https://www.googleapis.com";
  http::Url u = http::parse_url(url);
  if (!base && u.scheme != "https") throw std::runtime_error("https only");
  http::ClientOptions o;
  o.base_url = u.scheme + "://" + u.host + ":" + std::to_string(u.port);
  o.tls = test_tls();
  o.timeout_ms = 60000;
  base_path_ = u.path;
  http_ = std::make_unique<http::Client>(o);
}

bool valid_utf8(const std::string& s) {
  size_t i = 0;
  while (i < s.size()) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (n == 0 || i + n > s.size()) return false;
    for (size_t k = 1; k < n; ++k) {
      if ((static_cast<unsigned char>(s[i + k]) & 0xC0) != 0x80) return false;
    }
    i += n;
  }
  return true;
}

std::string DriveClient::export_file(const std::string& file_id, const std::string& mime) {
  http::Headers h;
  h.set("Authorization", "Bearer " + auth_.token());
  std::string path = base_path_ + "/drive/v3/files/" + http::url_encode(file_id) + "/export?mimeType=" +
                     http::url_encode(mime) + "&alt=media";
  http::Response r = http_->request("GET", path, "", &h);
  if (r.status < 200 || r.status >= 300) throw GoogleApiError(r.status, "request failed");
  if (!valid_utf8(r.body)) throw GoogleApiError(r.status, "file is not utf8");
  return r.body;
}

std::string DriveClient::file_version(const std::string& file_id) {
  http::Headers h;
  h.set("Authorization", "Bearer " + auth_.token());
  std::string path = base_path_ + "/drive/v3/files/" + http::url_encode(file_id) + "?fields=version";
  http::Response r = http_->request("GET", path, "", &h);
  if (r.status < 200 || r.status >= 300) throw GoogleApiError(r.status, "request failed");
  Value v = json::parse(r.body);
  const Value& ver = v.get("version");  // int64 rendered as a JSON string by Drive
  if (ver.is_string()) return ver.as_string();
  if (ver.is_int()) return std::to_string(ver.as_int());
  throw GoogleApiError(r.status, "no version in file metadata");
}

}  // namespace bgc::sync

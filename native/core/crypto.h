// Hashing, encoding, JWT signing and certificate helpers on OpenSSL 3.
//
// sha256_hex replaces the `sha256` crate used by the admission cert reloader
// (reference src/admission.rs:96-101); rs256 JWTs replace yup-oauth2's service
// account flow (reference src/synchronizer.rs:178-181).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace bgc::crypto {

std::string sha256_hex(std::string_view data);
std::string sha256_raw(std::string_view data);

std::string base64_encode(std::string_view data, bool url = false, bool pad = true);
// Accepts both alphabets, optional padding, ignores whitespace. Throws on garbage.
std::string base64_decode(std::string_view data);

std::string random_bytes(size_t n);
std::string uuid_v4();

// RS256 (RSASSA-PKCS1-v1_5 SHA-256) signature with a PEM private key.
std::string rs256_sign(const std::string& pem_private_key, std::string_view data);
bool rs256_verify(const std::string& pem_public_key_or_cert, std::string_view data,
                  std::string_view signature);

// Compact JWS: base64url(header).base64url(claims).base64url(sig)
std::string jwt_rs256(const std::string& header_json, const std::string& claims_json,
                      const std::string& pem_private_key);

struct KeyPair {
  std::string private_key_pem;
  std::string public_key_pem;
};
KeyPair generate_rsa(int bits = 2048);

struct CertBundle {
  std::string ca_cert_pem;
  std::string ca_key_pem;
  std::string cert_pem;
  std::string key_pem;
};
// Self-signed CA plus a leaf certificate signed by it (what the chart gets from
// cert-manager, reference charts/.../templates/certificate.yaml:1-51). Used by tests,
// the bench and `bgc-certgen`.
// key_type "ec" (P-256, the default: a TLS handshake signs with ECDSA in ~30 us instead of
// an RSA-2048 private-key operation of ~1 ms — the chart's cert-manager Certificate asks
// for the same) or "rsa" (2048 bit).
CertBundle make_ca_and_leaf(const std::string& common_name,
                            const std::vector<std::string>& dns_names,
                            int valid_days = 90, const std::string& key_type = "ec");

}  // namespace bgc::crypto

#include "core/crypto.h"

#include <unistd.h>

#include <openssl/bio.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rand.h>
#include <openssl/rsa.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>

#include <memory>
#include <stdexcept>

namespace bgc::crypto {

namespace {

std::string ssl_error(const std::string& what) {
  unsigned long e = ERR_get_error();
  char buf[256];
  ERR_error_string_n(e, buf, sizeof(buf));
  return what + ": " + buf;
}

struct BioDel {
  void operator()(BIO* b) const { BIO_free(b); }
};
struct PkeyDel {
  void operator()(EVP_PKEY* k) const { EVP_PKEY_free(k); }
};
struct MdCtxDel {
  void operator()(EVP_MD_CTX* c) const { EVP_MD_CTX_free(c); }
};
struct X509Del {
  void operator()(X509* x) const { X509_free(x); }
};
using BioPtr = std::unique_ptr<BIO, BioDel>;
using PkeyPtr = std::unique_ptr<EVP_PKEY, PkeyDel>;
using X509Ptr = std::unique_ptr<X509, X509Del>;

std::string bio_to_string(BIO* b) {
  char* data = nullptr;
  long n = BIO_get_mem_data(b, &data);
  return std::string(data, static_cast<size_t>(n));
}

PkeyPtr load_private_key(const std::string& pem) {
  BioPtr bio(BIO_new_mem_buf(pem.data(), static_cast<int>(pem.size())));
  EVP_PKEY* k = PEM_read_bio_PrivateKey(bio.get(), nullptr, nullptr, nullptr);
  if (!k) throw std::runtime_error(ssl_error("failed to parse private key"));
  return PkeyPtr(k);
}

PkeyPtr load_public_key(const std::string& pem) {
  {
    BioPtr bio(BIO_new_mem_buf(pem.data(), static_cast<int>(pem.size())));
    EVP_PKEY* k = PEM_read_bio_PUBKEY(bio.get(), nullptr, nullptr, nullptr);
    if (k) return PkeyPtr(k);
  }
  ERR_clear_error();
  BioPtr bio(BIO_new_mem_buf(pem.data(), static_cast<int>(pem.size())));
  X509Ptr cert(PEM_read_bio_X509(bio.get(), nullptr, nullptr, nullptr));
  if (!cert) throw std::runtime_error(ssl_error("failed to parse public key/cert"));
  EVP_PKEY* k = X509_get_pubkey(cert.get());
  if (!k) throw std::runtime_error(ssl_error("certificate has no public key"));
  return PkeyPtr(k);
}

std::string key_to_pem(EVP_PKEY* k, bool priv) {
  BioPtr bio(BIO_new(BIO_s_mem()));
  int ok = priv ? PEM_write_bio_PrivateKey(bio.get(), k, nullptr, nullptr, 0, nullptr, nullptr)
                : PEM_write_bio_PUBKEY(bio.get(), k);
  if (!ok) throw std::runtime_error(ssl_error("PEM write failed"));
  return bio_to_string(bio.get());
}

std::string cert_to_pem(X509* x) {
  BioPtr bio(BIO_new(BIO_s_mem()));
  if (!PEM_write_bio_X509(bio.get(), x)) throw std::runtime_error(ssl_error("PEM write failed"));
  return bio_to_string(bio.get());
}

}  // namespace

std::string sha256_raw(std::string_view data) {
  unsigned char md[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  if (!EVP_Digest(data.data(), data.size(), md, &len, EVP_sha256(), nullptr)) {
    throw std::runtime_error(ssl_error("sha256"));
  }
  return std::string(reinterpret_cast<char*>(md), len);
}

std::string sha256_hex(std::string_view data) {
  static const char kHex[] = "0123456789abcdef";
  std::string raw = sha256_raw(data);
  std::string out;
  out.reserve(raw.size() * 2);
  for (unsigned char c : raw) {
    out.push_back(kHex[c >> 4]);
    out.push_back(kHex[c & 15]);
  }
  return out;
}

std::string base64_encode(std::string_view data, bool url, bool pad) {
  static const char kStd[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  static const char kUrl[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
  const char* tbl = url ? kUrl : kStd;
  std::string out;
  out.reserve((data.size() + 2) / 3 * 4);
  size_t i = 0;
  const auto* p = reinterpret_cast<const unsigned char*>(data.data());
  for (; i + 2 < data.size(); i += 3) {
    uint32_t v = (uint32_t(p[i]) << 16) | (uint32_t(p[i + 1]) << 8) | p[i + 2];
    out.push_back(tbl[(v >> 18) & 63]);
    out.push_back(tbl[(v >> 12) & 63]);
    out.push_back(tbl[(v >> 6) & 63]);
    out.push_back(tbl[v & 63]);
  }
  size_t rem = data.size() - i;
  if (rem == 1) {
    uint32_t v = uint32_t(p[i]) << 16;
    out.push_back(tbl[(v >> 18) & 63]);
    out.push_back(tbl[(v >> 12) & 63]);
    if (pad) out.append("==");
  } else if (rem == 2) {
    uint32_t v = (uint32_t(p[i]) << 16) | (uint32_t(p[i + 1]) << 8);
    out.push_back(tbl[(v >> 18) & 63]);
    out.push_back(tbl[(v >> 12) & 63]);
    out.push_back(tbl[(v >> 6) & 63]);
    if (pad) out.push_back('=');
  }
  return out;
}

std::string base64_decode(std::string_view data) {
  auto val = [](char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+' || c == '-') return 62;
    if (c == '/' || c == '_') return 63;
    return -1;
  };
  std::string out;
  uint32_t acc = 0;
  int bits = 0;
  for (char c : data) {
    if (c == '=' || c == '\n' || c == '\r' || c == ' ' || c == '\t') continue;
    int v = val(c);
    if (v < 0) throw std::runtime_error("invalid base64 input");
    acc = (acc << 6) | static_cast<uint32_t>(v);
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out.push_back(static_cast<char>((acc >> bits) & 0xFF));
    }
  }
  return out;
}

std::string random_bytes(size_t n) {
  std::string out(n, '\0');
  if (RAND_bytes(reinterpret_cast<unsigned char*>(out.data()), static_cast<int>(n)) != 1) {
    throw std::runtime_error(ssl_error("RAND_bytes"));
  }
  return out;
}

std::string uuid_v4() {
  // UUIDs come from the same CSPRNG, drawn 4 KiB at a time into a per-thread pool:
  // RAND_bytes costs microseconds per call in OpenSSL 3 (provider dispatch, DRBG locks),
  // which made it 5.6 % of kube-lite's CPU at four UIDs per tenant.  The pool is
  // discarded after a fork, so a child never repeats its parent's UUIDs.
  thread_local unsigned char pool[4096];
  thread_local size_t used = sizeof(pool);
  thread_local pid_t owner = 0;
  const pid_t pid = ::getpid();
  if (used + 16 > sizeof(pool) || owner != pid) {
    if (RAND_bytes(pool, static_cast<int>(sizeof(pool))) != 1) throw std::runtime_error(ssl_error("RAND_bytes"));
    used = 0;
    owner = pid;
  }
  std::string b(reinterpret_cast<const char*>(pool + used), 16);
  OPENSSL_cleanse(pool + used, 16);
  used += 16;
  b[6] = static_cast<char>((b[6] & 0x0F) | 0x40);
  b[8] = static_cast<char>((b[8] & 0x3F) | 0x80);
  static const char kHex[] = "0123456789abcdef";
  std::string out;
  for (int i = 0; i < 16; ++i) {
    if (i == 4 || i == 6 || i == 8 || i == 10) out.push_back('-');
    unsigned char c = static_cast<unsigned char>(b[static_cast<size_t>(i)]);
    out.push_back(kHex[c >> 4]);
    out.push_back(kHex[c & 15]);
  }
  return out;
}

std::string rs256_sign(const std::string& pem_private_key, std::string_view data) {
  PkeyPtr key = load_private_key(pem_private_key);
  std::unique_ptr<EVP_MD_CTX, MdCtxDel> ctx(EVP_MD_CTX_new());
  if (EVP_DigestSignInit(ctx.get(), nullptr, EVP_sha256(), nullptr, key.get()) != 1) {
    throw std::runtime_error(ssl_error("DigestSignInit"));
  }
  size_t len = 0;
  if (EVP_DigestSign(ctx.get(), nullptr, &len, reinterpret_cast<const unsigned char*>(data.data()),
                     data.size()) != 1) {
    throw std::runtime_error(ssl_error("DigestSign(len)"));
  }
  std::string sig(len, '\0');
  if (EVP_DigestSign(ctx.get(), reinterpret_cast<unsigned char*>(sig.data()), &len,
                     reinterpret_cast<const unsigned char*>(data.data()), data.size()) != 1) {
    throw std::runtime_error(ssl_error("DigestSign"));
  }
  sig.resize(len);
  return sig;
}

bool rs256_verify(const std::string& pem, std::string_view data, std::string_view signature) {
  PkeyPtr key = load_public_key(pem);
  std::unique_ptr<EVP_MD_CTX, MdCtxDel> ctx(EVP_MD_CTX_new());
  if (EVP_DigestVerifyInit(ctx.get(), nullptr, EVP_sha256(), nullptr, key.get()) != 1) return false;
  int rc = EVP_DigestVerify(ctx.get(), reinterpret_cast<const unsigned char*>(signature.data()),
                            signature.size(), reinterpret_cast<const unsigned char*>(data.data()),
                            data.size());
  ERR_clear_error();
  return rc == 1;
}

std::string jwt_rs256(const std::string& header_json, const std::string& claims_json,
                      const std::string& pem_private_key) {
  std::string signing_input =
      base64_encode(header_json, true, false) + "." + base64_encode(claims_json, true, false);
  std::string sig = rs256_sign(pem_private_key, signing_input);
  return signing_input + "." + base64_encode(sig, true, false);
}

KeyPair generate_rsa(int bits) {
  EVP_PKEY* k = EVP_RSA_gen(static_cast<unsigned int>(bits));
  if (!k) throw std::runtime_error(ssl_error("RSA keygen"));
  PkeyPtr key(k);
  return {key_to_pem(key.get(), true), key_to_pem(key.get(), false)};
}

namespace {

void add_ext(X509* cert, X509* issuer, int nid, const std::string& value) {
  X509V3_CTX ctx;
  X509V3_set_ctx_nodb(&ctx);
  X509V3_set_ctx(&ctx, issuer, cert, nullptr, nullptr, 0);
  X509_EXTENSION* ex = X509V3_EXT_conf_nid(nullptr, &ctx, nid, value.c_str());
  if (!ex) throw std::runtime_error(ssl_error("X509V3_EXT_conf_nid"));
  X509_add_ext(cert, ex, -1);
  X509_EXTENSION_free(ex);
}

X509Ptr make_cert(EVP_PKEY* subject_key, const std::string& cn, X509* issuer_cert,
                  EVP_PKEY* issuer_key, bool is_ca, const std::vector<std::string>& dns, int days) {
  X509Ptr x(X509_new());
  X509_set_version(x.get(), 2);
  std::string serial = random_bytes(8);
  BIGNUM* bn = BN_bin2bn(reinterpret_cast<const unsigned char*>(serial.data()), 8, nullptr);
  BN_set_negative(bn, 0);
  BN_to_ASN1_INTEGER(bn, X509_get_serialNumber(x.get()));
  BN_free(bn);
  X509_gmtime_adj(X509_getm_notBefore(x.get()), -3600);
  X509_gmtime_adj(X509_getm_notAfter(x.get()), static_cast<long>(days) * 86400L);
  X509_set_pubkey(x.get(), subject_key);
  X509_NAME* name = X509_get_subject_name(x.get());
  X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, reinterpret_cast<const unsigned char*>(cn.c_str()),
                             -1, -1, 0);
  X509* iss = issuer_cert ? issuer_cert : x.get();
  X509_set_issuer_name(x.get(), X509_get_subject_name(iss));
  if (is_ca) {
    add_ext(x.get(), iss, NID_basic_constraints, "critical,CA:TRUE");
    add_ext(x.get(), iss, NID_key_usage, "critical,keyCertSign,cRLSign,digitalSignature");
  } else {
    add_ext(x.get(), iss, NID_basic_constraints, "critical,CA:FALSE");
    // keyEncipherment only means something for RSA key transport
    add_ext(x.get(), iss, NID_key_usage,
            EVP_PKEY_get_base_id(subject_key) == EVP_PKEY_RSA ? "critical,digitalSignature,keyEncipherment"
                                                              : "critical,digitalSignature");
    add_ext(x.get(), iss, NID_ext_key_usage, "serverAuth,clientAuth");
    std::string san;
    for (const auto& d : dns) {
      if (!san.empty()) san += ",";
      bool ip = !d.empty() && d.find_first_not_of("0123456789.") == std::string::npos;
      san += (ip ? "IP:" : "DNS:") + d;
    }
    if (!san.empty()) add_ext(x.get(), iss, NID_subject_alt_name, san);
  }
  add_ext(x.get(), iss, NID_subject_key_identifier, "hash");
  if (!X509_sign(x.get(), issuer_key, EVP_sha256())) throw std::runtime_error(ssl_error("X509_sign"));
  return x;
}

}  // namespace

CertBundle make_ca_and_leaf(const std::string& common_name, const std::vector<std::string>& dns_names,
                            int valid_days, const std::string& key_type) {
  if (key_type != "ec" && key_type != "rsa") throw std::invalid_argument("key_type must be ec or rsa");
  auto gen = [&]() -> EVP_PKEY* { return key_type == "ec" ? EVP_EC_gen("P-256") : EVP_RSA_gen(2048); };
  PkeyPtr ca_key(gen());
  PkeyPtr leaf_key(gen());
  if (!ca_key || !leaf_key) throw std::runtime_error(ssl_error("keygen"));
  X509Ptr ca = make_cert(ca_key.get(), common_name + "-ca", nullptr, ca_key.get(), true, {}, 36500);
  X509Ptr leaf = make_cert(leaf_key.get(), common_name, ca.get(), ca_key.get(), false, dns_names, valid_days);
  CertBundle b;
  b.ca_cert_pem = cert_to_pem(ca.get());
  b.ca_key_pem = key_to_pem(ca_key.get(), true);
  b.cert_pem = cert_to_pem(leaf.get());
  b.key_pem = key_to_pem(leaf_key.get(), true);
  return b;
}

}  // namespace bgc::crypto

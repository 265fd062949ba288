// bgc-certgen: self-signed CA + webhook serving certificate for clusters without
// cert-manager (the chart's certificate.yaml does the same through cert-manager).
//   bgc-certgen <out-dir> <common-name> [dns-name ...]
// Writes ca.crt, ca.key, tls.crt, tls.key and caBundle.b64 (for the webhook config).
#include <cstdio>
#include <string>
#include <vector>

#include "core/crypto.h"
#include "core/net.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: bgc-certgen <out-dir> <common-name> [dns-name ...]\n");
    return 2;
  }
  std::string dir = argv[1];
  std::vector<std::string> dns;
  for (int i = 3; i < argc; ++i) dns.emplace_back(argv[i]);
  if (dns.empty()) dns.emplace_back(argv[2]);
  try {
    auto b = bgc::crypto::make_ca_and_leaf(argv[2], dns, 90);
    bgc::net::write_file(dir + "/ca.crt", b.ca_cert_pem);
    bgc::net::write_file(dir + "/ca.key", b.ca_key_pem);
    bgc::net::write_file(dir + "/tls.crt", b.cert_pem);
    bgc::net::write_file(dir + "/tls.key", b.key_pem);
    bgc::net::write_file(dir + "/caBundle.b64", bgc::crypto::base64_encode(b.ca_cert_pem) + "\n");
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  return 0;
}

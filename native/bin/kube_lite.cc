// kube-lite: standalone in-memory Kubernetes API server (see apiserver/server.h).
//
//   kube-lite --port 0 --port-file /tmp/port --token-file tokens.csv
//             --service-override bgc/bgc-admission=127.0.0.1:12321 --manifest crd.yaml
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "apiserver/server.h"
#include "core/cancel.h"
#include "core/http.h"
#include "core/json.h"
#include "core/log.h"
#include "core/net.h"
#include "core/process.h"
#include "core/stall.h"
#include "core/yaml.h"

using namespace bgc;

static void usage() {
  std::fprintf(stderr,
               "usage: kube-lite [--addr A] [--port P] [--port-file F] [--token-file F] [--no-anonymous]\n"
               "                 [--tls-cert F --tls-key F] [--service-override ns/name=host:port]...\n"
               "                 [--bookmark-ms N] [--history N] [--watch-coalesce-us N] [--gc-workers N]\n"
               "                 [--opaque-rv] [--continue-ttl-ms N] [--webhook-http1|--webhook-http2] [--webhook-h2-connections N]\n"
               "                 [--write-latency-ms F] [--store-shards N] [--no-selector-transitions]\n"
               "                 [--instant-namespace-deletion]\n"
               "                 [--manifest file.{json,yaml}]...\n");
}

int main(int argc, char** argv) {
  // A test server: no malloc_trim passes (one stalls kube-lite for 110-130 ms on the bench's
  // heap, which would show up in the measured latencies).  BGC_MALLOC_TRIM_SECS still wins.
  setenv("BGC_MALLOC_TRIM_SECS", "0", /*overwrite=*/0);
  // Nor the services' bounded-footprint allocator settings (core/process.cc tune_malloc): a
  // test fixture is tuned for throughput, the bench's CR/s being mostly kube-lite's CPU —
  // glibc's arena count, 64 MiB heap growth, no trimming below 512 MiB.
  setenv("BGC_MALLOC_ARENA_MAX", "0", 0);
  setenv("BGC_MALLOC_TOP_PAD_KB", "65536", 0);
  setenv("BGC_MALLOC_TRIM_THRESHOLD_KB", "524288", 0);
  process_init();
  apiserver::Options o;
  std::string port_file;
  std::vector<std::string> manifests;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        usage();
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--addr") o.addr = next();
    else if (a == "--port") o.port = static_cast<uint16_t>(std::atoi(next().c_str()));
    else if (a == "--port-file") port_file = next();
    else if (a == "--token-file") o.token_file = next();
    else if (a == "--no-anonymous") o.anonymous_admin = false;
    else if (a == "--tls-cert") o.tls_cert_file = next();
    else if (a == "--tls-key") o.tls_key_file = next();
    else if (a == "--client-ca-file") o.client_ca_file = next();
    else if (a == "--bookmark-ms") o.bookmark_interval_ms = std::atoi(next().c_str());
    else if (a == "--history") o.history_limit = static_cast<size_t>(std::atol(next().c_str()));
    else if (a == "--watch-coalesce-us") o.watch_coalesce_us = std::atoi(next().c_str());
    else if (a == "--gc-workers") o.gc_workers = std::atoi(next().c_str());
    else if (a == "--write-latency-ms") o.write_latency_us = static_cast<int64_t>(std::atof(next().c_str()) * 1000.0);
    else if (a == "--opaque-rv") o.opaque_rv = true;
    else if (a == "--no-selector-transitions") o.selector_transitions = false;
    else if (a == "--instant-namespace-deletion") o.namespace_termination = false;
    else if (a == "--webhook-http1") o.webhook_http2 = false;
    else if (a == "--webhook-http2") o.webhook_http2 = true;
    else if (a == "--webhook-h2-connections") o.webhook_h2_connections = static_cast<size_t>(std::atoi(next().c_str()));
    else if (a == "--store-shards") o.store_shards = static_cast<size_t>(std::max(1, std::atoi(next().c_str())));
    else if (a == "--continue-ttl-ms") o.continue_ttl_ms = std::atoi(next().c_str());
    else if (a == "--manifest") manifests.push_back(next());
    else if (a == "--service-override") {
      std::string v = next();
      size_t eq = v.find('=');
      if (eq == std::string::npos) {
        usage();
        return 2;
      }
      o.service_overrides[v.substr(0, eq)] = v.substr(eq + 1);
    } else if (a == "-h" || a == "--help") {
      usage();
      return 0;
    } else {
      usage();
      return 2;
    }
  }
  auto stop = std::make_shared<CancelToken>();
  install_shutdown_signals(stop);
  apiserver::ApiServer srv(o);
  try {
    srv.start();
    stall::start("kube-lite");  // after start(): debug endpoints are on, stalls are kept
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  std::string base = std::string(o.tls_cert_file.empty() ? "http" : "https") + "://" + o.addr + ":" +
                     std::to_string(srv.port());
  // preload manifests (e.g. the CRD) through the regular API
  for (const auto& m : manifests) {
    std::string text = net::read_file(m);
    std::vector<json::Value> docs;
    if (!text.empty() && text[0] == '{') docs.push_back(json::parse(text));
    else docs = yaml::parse_all(text);
    for (const auto& d : docs) {
      std::string api_version = d.get_string("apiVersion");
      std::string kind = d.get_string("kind");
      std::string plural;
      for (char c : kind) plural.push_back(static_cast<char>(std::tolower(static_cast<unsigned char>(c))));
      plural += plural.back() == 's' ? "es" : (plural.back() == 'y' ? "" : "s");
      if (kind.back() == 'y') plural = plural.substr(0, plural.size() - 1) + "ies";
      std::string path = (api_version.find('/') == std::string::npos ? "/api/" : "/apis/") + api_version + "/" + plural;
      auto r = http::fetch("POST", "http://127.0.0.1:" + std::to_string(srv.port()) + path, d.dump());
      if (r.status >= 300) {
        std::fprintf(stderr, "Error: manifest %s (%s): %d %s\n", m.c_str(), kind.c_str(), r.status, r.body.c_str());
        return 1;
      }
    }
  }
  if (!port_file.empty()) {
    net::write_file(port_file + ".tmp", std::to_string(srv.port()));
    std::rename((port_file + ".tmp").c_str(), port_file.c_str());
  }
  LOG_INFO("apiserver") << "kube-lite serving on " << base;
  stop->wait();
  srv.stop();
  return 0;
}

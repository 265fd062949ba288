// admission: TLS webhook server — POST /mutate (AdmissionReview v1), GET /health,
// GET /metrics — with certificate hot reload.  Reference: src/admission.rs:96-204.
#include <cstdio>
#include <memory>
#include <thread>

#include "admission/policy.h"
#include "core/cancel.h"
#include "core/crypto.h"
#include "core/env_config.h"
#include "core/http.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/stall.h"
#include "core/net.h"
#include "core/process.h"

using namespace bgc;

// sha256 over cert‖key (reference admission.rs:96-101)
static std::string cert_hash(const std::string& cert, const std::string& key) {
  return crypto::sha256_hex(net::read_file(cert) + net::read_file(key));
}

int main() {
  process_init();
  admission::Config cfg;
  try {
    cfg = admission::Config::from_env(EnvConfig("CONF_"));
    metrics::configure_debug(EnvConfig("CONF_"));  // /debug/samples: off unless CONF_DEBUG_ENDPOINTS
    stall::start("admission");  // 1 ms oversleep sampler: bgc_stall_* (core/stall.h)
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  auto stop = std::make_shared<CancelToken>();
  install_shutdown_signals(stop);

  std::shared_ptr<net::TlsContext> tls;
  try {
    tls = net::TlsContext::server_from_files(cfg.cert_path, cfg.key_path);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: failed to read cert: %s\n", e.what());
    return 1;
  }

  auto& reg = metrics::Registry::global();
  auto& hist_allowed = reg.histogram("bgc_admission_duration_seconds", "Admission handler latency", {{"allowed", "true"}});
  auto& hist_denied = reg.histogram("bgc_admission_duration_seconds", "Admission handler latency", {{"allowed", "false"}});
  auto& ring = reg.samples("admission");

  http::ServerOptions so;
  so.addr = cfg.listen_addr;
  so.port = cfg.listen_port;
  so.tls = tls;
  so.name = "admission";
  so.http2 = cfg.http2;
  if (cfg.http2_inline) so.h2_inline_paths = {"/mutate"};
  http::Server server(so);
  http::add_standard_routes(server);
  server.handle("POST", "/mutate", [&](http::Request& req, http::ResponseWriter& w) {
    int64_t t0 = metrics::now_ns();
    auto r = admission::handle_review(req.body, req.headers.get_or("Content-Type"), cfg);
    w.send(r.status, r.body, r.content_type);
    double secs = static_cast<double>(metrics::now_ns() - t0) * 1e-9;
    (r.decision.allowed ? hist_allowed : hist_denied).observe(secs);
    ring.add(secs);
  });

  try {
    server.start();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  LOG_INFO("admission") << "starting tls server on " << cfg.listen_addr << ":" << server.port();

  // Cert reloader (admission.rs:104-126). Q14 fix: errors are logged and retried
  // instead of silently ending the reload task.
  std::thread reloader([&] {
    std::string hash;
    try {
      hash = cert_hash(cfg.cert_path, cfg.key_path);
    } catch (const std::exception& e) {
      LOG_ERROR("admission") << "cert hash failed: " << e.what();
    }
    while (!stop->wait_for(std::chrono::seconds(cfg.cert_reload_interval_secs))) {
      try {
        std::string h = cert_hash(cfg.cert_path, cfg.key_path);
        if (h != hash) {
          LOG_INFO("admission") << "cert changed, reloading...";
          tls->reload_from_files(cfg.cert_path, cfg.key_path);
          LOG_INFO("admission") << "cert reloading done.";
          hash = h;
        }
      } catch (const std::exception& e) {
        LOG_ERROR("admission") << "cert reload failed (will retry): " << e.what();
      }
    }
  });

  stop->wait();
  server.stop(std::chrono::milliseconds(10000));  // 10 s graceful drain (admission.rs:93)
  reloader.join();
  LOG_INFO("admission") << "received signal. shutting down...";
  return 0;
}

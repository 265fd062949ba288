// synchronizer: Google Sheet -> UserBootstrap quota/status; serves /health, /metrics.
// Reference: src/synchronizer.rs:381-435.
#include <cstdio>
#include <memory>

#include "core/cancel.h"
#include "core/env_config.h"
#include "kube/runtime.h"
#include "core/http.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/stall.h"
#include "core/process.h"
#include "kube/client.h"
#include "kube/leader.h"
#include "sync/google.h"
#include "sync/synchronizer.h"

using namespace bgc;

int main() {
  process_init();
  sync::Config cfg;
  try {
    cfg = sync::Config::from_env(EnvConfig("CONF_"));
    metrics::configure_debug(EnvConfig("CONF_"));  // /debug/samples: off unless CONF_DEBUG_ENDPOINTS
    stall::start("synchronizer");  // 1 ms oversleep sampler: bgc_stall_* (core/stall.h)
    kube::Watcher::configure_from_env(EnvConfig("CONF_"));  // list paging, watch idle deadline, TCP keepalive
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  std::unique_ptr<sync::GoogleAuth> auth;
  try {
    auth = std::make_unique<sync::GoogleAuth>(sync::ServiceAccountKey::from_file(cfg.google_service_account_json_path),
                                              sync::kDriveReadonlyScope);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  std::unique_ptr<kube::KubeClient> client;
  try {
    client = std::make_unique<kube::KubeClient>(kube::KubeConfig::infer());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: failed to infer kubernetes config: %s\n", e.what());
    return 1;
  }
  auto stop = std::make_shared<CancelToken>();
  install_shutdown_signals(stop);

  http::ServerOptions so;
  so.addr = cfg.listen_addr;
  so.port = cfg.listen_port;
  so.name = "synchronizer";
  http::Server health(so);
  http::add_standard_routes(health);
  try {
    health.start();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  LOG_INFO("synchronizer") << "starting http server on " << cfg.listen_addr << ":" << health.port();

  std::unique_ptr<sync::DriveClient> drive;
  try {
    drive = std::make_unique<sync::DriveClient>(*auth);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  // Standbys wait here; losing the lease stops the loop (kubelet restarts us).  The elector
  // lives in main's scope so its renew thread runs as long as the loop does.
  bool standby_stopped = false;
  std::unique_ptr<kube::LeaderElector> leader = kube::lead_or_wait(*client, cfg.lease, stop, &standby_stopped);
  if (standby_stopped) {
    health.stop();
    return 0;
  }
  std::string file_id = cfg.google_file_id;
  sync::Synchronizer s(*client, [&] { return drive->export_file(file_id, "text/csv"); }, cfg);
  s.set_version_source([&] { return drive->file_version(file_id); });
  int rc = s.run(*stop);
  if (rc == 0 && leader && leader->lost()) rc = 1;  // a lost lease is a failure: restart as a standby
  health.stop(std::chrono::milliseconds(1000));
  if (rc == 0) {
    LOG_INFO("synchronizer") << "synchronizer gracefully shutted down";
  }
  return rc;
}

// controller: watches UserBootstraps (+ owned Namespaces, ResourceQuotas, Roles,
// RoleBindings) and reconciles them; serves /health, /metrics on CONF_LISTEN_ADDR:PORT.
// Reference: src/controller.rs:215-287.
#include <cstdio>
#include <unistd.h>
#include <memory>

#include "controller/reconcile.h"
#include "core/cancel.h"
#include "core/env_config.h"
#include "core/http.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/stall.h"
#include "core/process.h"
#include "kube/leader.h"
#include "kube/runtime.h"

using namespace bgc;

int main() {
  ProcessDefaults defaults;
  defaults.malloc_arena_max = 16;  // see tune_malloc (core/process.cc)
  process_init(defaults);
  controller::Config cfg;
  try {
    cfg = controller::Config::from_env(EnvConfig("CONF_"));
    metrics::configure_debug(EnvConfig("CONF_"));  // /debug/samples: off unless CONF_DEBUG_ENDPOINTS
    stall::start("controller");  // 1 ms oversleep sampler: bgc_stall_* (core/stall.h)
    kube::Watcher::configure_from_env(EnvConfig("CONF_"));  // list paging, watch idle deadline, TCP keepalive
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  auto stop = std::make_shared<CancelToken>();
  install_shutdown_signals(stop);

  std::unique_ptr<kube::KubeClient> client;
  try {
    client = std::make_unique<kube::KubeClient>(kube::KubeConfig::infer());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: failed to infer kubernetes config: %s\n", e.what());
    return 1;
  }

  http::ServerOptions so;
  so.addr = cfg.listen_addr;
  so.port = cfg.listen_port;
  so.name = "controller";
  http::Server health(so);
  http::add_standard_routes(health);
  try {
    health.start();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  LOG_INFO("controller") << "starting server on " << cfg.listen_addr << ":" << health.port();

  // The elector lives in main's scope so its renew thread runs until the controller exits.
  bool standby_stopped = false;
  std::unique_ptr<kube::LeaderElector> leader = kube::lead_or_wait(*client, cfg.lease, stop, &standby_stopped);
  if (standby_stopped) {
    health.stop();
    return 0;
  }

  kube::Controller::Options co;
  co.workers = cfg.workers;
  co.child_delete_delay = std::chrono::milliseconds(cfg.child_delete_delay_ms);
  co.debounce = std::chrono::milliseconds(cfg.debounce_ms);
  if (cfg.projected_watch) {
    co.primary_projection = &controller::user_bootstrap_event_projection();
    co.child_projection = &controller::child_event_projection();
  }
  kube::Controller ctrl(*client, kube::types::UserBootstrap, co);
  const std::string sel = cfg.label_children ? controller::child_label_selector() : "";
  ctrl.owns(kube::types::Namespace, nullptr, sel, cfg.metadata_watches);
  ctrl.owns(kube::types::ResourceQuota, nullptr, sel, cfg.metadata_watches);
  ctrl.owns(kube::types::Role, nullptr, sel, cfg.metadata_watches);
  ctrl.owns(kube::types::RoleBinding, nullptr, sel, cfg.metadata_watches);
  controller::Reconciler rec(*client, ctrl, cfg);
  std::unique_ptr<kube::EventRecorder> events;
  if (cfg.events) {
    kube::EventOptions eo;
    eo.component = "bacchus-gpu-controller";
    char host[256] = {0};
    ::gethostname(host, sizeof(host) - 1);
    eo.host = host;
    events = std::make_unique<kube::EventRecorder>(*client, eo);
    rec.set_event_recorder(events.get());
  }
  auto& echoes = metrics::Registry::global().counter(
      "bgc_controller_own_write_events_total", "Child watch events dropped as echoes of our own applies");
  ctrl.set_child_filter([&](const kube::ResourceType& rt, const json::Value& child) {
    if (!rec.is_own_write(rt, child)) return true;
    echoes.inc();
    return false;
  });
  ctrl.set_child_deleted_hook([&](const kube::ResourceType& rt, const json::Value& child) {
    rec.forget(rt, child);
    return true;
  });
  ctrl.set_primary_deleted_hook([&](const json::Value& ub) { rec.forget_owner(kube::meta_name(ub)); });
  ctrl.run(
      *stop, [&](const kube::ObjPtr& o) { return rec.reconcile(o); },
      [&](const kube::ObjPtr& o, const std::exception& e) { return rec.error_policy(o, e); });
  health.stop(std::chrono::milliseconds(1000));
  LOG_INFO("controller") << "controller gracefully shutted down";
  return leader && leader->lost() ? 1 : 0;  // a lost lease is a failure: restart as a standby
}

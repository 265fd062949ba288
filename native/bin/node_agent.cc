// node-agent: DaemonSet process on every MI355X node.  Discovers GPUs (amdsmi), runs
// optional HIP health diagnostics, advertises amd.com/gpu + topology labels on its Node,
// and keeps a telemetry side thread (amdsmi gpu_metrics) feeding health + /metrics.
#include <cstdio>
#include <memory>
#include <string>

#include "core/cancel.h"
#include "core/env_config.h"
#include "kube/runtime.h"
#include "core/http.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/stall.h"
#include "core/process.h"
#include "gpu/device.h"
#include "gpu/diag_runner.h"
#include "gpu/node_agent.h"
#include "kube/client.h"

using namespace bgc;

int main(int argc, char** argv) {
  // a diagnostics worker (gpu/diag_runner.h): one request, then exit
  if (argc > 1 && std::string(argv[1]) == "--diag-worker") return gpu::diag_worker_main();
  process_init();
  gpu::NodeAgentConfig cfg;
  try {
    cfg = gpu::NodeAgentConfig::from_env(EnvConfig("CONF_"));
    metrics::configure_debug(EnvConfig("CONF_"));  // /debug/samples: off unless CONF_DEBUG_ENDPOINTS
    stall::start("node-agent");  // 1 ms oversleep sampler: bgc_stall_* (core/stall.h)
    kube::Watcher::configure_from_env(EnvConfig("CONF_"));  // list paging, watch idle deadline, TCP keepalive
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  auto stop = std::make_shared<CancelToken>();
  install_shutdown_signals(stop);
  std::unique_ptr<kube::KubeClient> client;
  std::unique_ptr<gpu::NodeAgent> agent;
  try {
    client = std::make_unique<kube::KubeClient>(kube::KubeConfig::infer());
    agent = std::make_unique<gpu::NodeAgent>(*client, gpu::make_backend(cfg.backend, cfg.mock_fixture_path), cfg);
    agent->init();
    agent->publish();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  http::ServerOptions so;
  so.addr = cfg.listen_addr;
  so.port = cfg.listen_port;
  so.name = "node_agent";
  http::Server server(so);
  http::add_standard_routes(server);
  server.handle("GET", "/gpus", [&](http::Request&, http::ResponseWriter& w) { w.send_json(200, agent->describe().dump()); });
  try {
    server.start();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  LOG_INFO("node_agent") << "serving on " << cfg.listen_addr << ":" << server.port();
  agent->start();
  stop->wait();
  arm_shutdown_deadline(std::chrono::seconds(cfg.shutdown_timeout_secs));
  agent->stop();
  server.stop(std::chrono::milliseconds(1000));
  return 0;
}

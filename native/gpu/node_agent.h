// MI355X node agent (north-star N3): advertises each healthy MI355X as an `amd.com/gpu`
// extended resource and publishes topology labels so RCCL TP/DP/PP pods can be
// co-scheduled on one xGMI island.
//
//   labels       amd.com/gpu.present=true, .family=gfx950, .product=MI355X, .count=8,
//                .vram-gb=288, .xgmi-hive-id=<hex>, .compute-partition=SPX,
//                .memory-partition=NPS1, .cu-count=256, .healthy-count=8, .diag=passed
//   annotation   amd.com/gpu.topology = JSON [{index,uuid,bdf,hive,node,numa}]
//   status       capacity/allocatable amd.com/gpu, condition AMDGPUHealthy
//
// Labels go through server-side apply on the Node, capacity/condition through SSA on
// nodes/status, both with field manager "bacchus-gpu-node-agent" so kubelet-owned
// fields are untouched.  Health flips from the telemetry side thread re-apply status.
// The agent also watches its own Node (fieldSelector metadata.name=<node>): a Node that
// is deleted and re-registered (drain / re-add) or whose labels/capacity drift is
// re-published immediately instead of on the next heartbeat.  Without create_node the
// agent never creates the Node itself; it waits for the kubelet to register it.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "core/env_config.h"
#include "core/json.h"
#include "gpu/device.h"
#include "gpu/device_plugin.h"
#include "gpu/telemetry.h"
#include "kube/client.h"

namespace bgc::gpu {

constexpr const char* kNodeAgentManager = "bacchus-gpu-node-agent";

struct NodeAgentConfig {
  std::string listen_addr = "0.0.0.0";
  uint16_t listen_port = 12324;
  std::string node_name;
  std::string backend = "auto";       // auto | amdsmi | mock
  std::string mock_fixture_path;
  uint64_t poll_interval_ms = 1000;
  uint64_t heartbeat_secs = 30;
  std::string resource_name = "amd.com/gpu";
  // When every GPU runs a sub-device compute partition (DPX/QPX/CPX: one logical device
  // per partition), the devices are advertised under this name instead — the key the
  // synchronizer writes for the sheet's partition column (reference: the MIG column,
  // src/synchronizer.rs:276).  Empty = always `resource_name`.
  std::string partition_resource_name = "amd.com/gpu-partition";
  std::string label_prefix = "amd.com/gpu";
  int max_gpus = 0;                    // 0 = all discovered
  bool run_diag = false;               // HIP HBM + MFMA check before advertising
  uint64_t diag_hbm_bytes = 1ULL << 30;
  bool create_node = false;            // test clusters without a kubelet
  // Kubelet device plugin (gpu/device_plugin.h).  When on, the kubelet owns the
  // amd.com/gpu capacity/allocatable counts, so the Node status patch carries only the
  // AMDGPUHealthy condition; labels and topology are published as before.
  bool device_plugin = false;
  std::string device_plugin_dir = "/var/lib/kubelet/device-plugins";
  std::string device_plugin_socket = "bgc-amd-gpu.sock";
  std::string dev_root = "/dev";
  std::string sysfs_root = "/sys";
  static NodeAgentConfig from_env(const EnvConfig& env);
};

struct DiagOutcome {
  bool ran = false;
  bool passed = true;
  json::Value per_gpu = json::Value::array();
};

std::string sanitize_label_value(const std::string& v);
// The extended-resource name for a set of discovered devices (see partition_resource_name).
std::string advertised_resource(const NodeAgentConfig& cfg, const std::vector<GpuInfo>& gpus);
std::string product_label(const GpuInfo& g);

// Pure rendering of the Node patches (unit-tested).
json::Value node_labels_patch(const NodeAgentConfig& cfg, const std::vector<GpuInfo>& gpus, int healthy,
                              const DiagOutcome& diag);
json::Value node_status_patch(const NodeAgentConfig& cfg, const std::vector<GpuInfo>& gpus, int healthy,
                              const std::string& unhealthy_reason);

class NodeAgent {
 public:
  NodeAgent(kube::KubeClient& client, std::unique_ptr<Backend> backend, NodeAgentConfig cfg);
  ~NodeAgent();
  // Discovery (+ optional diagnostics); throws if no GPU is found.
  void init();
  // Apply labels + status now.
  void publish();
  void start();  // telemetry thread + heartbeat thread + Node watch
  // True when `node` already carries what publish() would write (labels + capacity).
  bool node_up_to_date(const json::Value& node) const;
  uint64_t publishes() const { return publishes_.load(); }
  void stop();
  json::Value describe() const;  // for GET /gpus
  const std::vector<GpuInfo>& gpus() const { return gpus_; }
  TelemetryPoller* poller() { return poller_.get(); }
  DevicePlugin* device_plugin() { return plugin_.get(); }
  // Per-GPU health: telemetry state machine AND (when run) the HIP diagnostics.
  std::vector<bool> healthy_flags() const;

 private:
  int healthy_count(std::string* reason) const;
  kube::KubeClient& client_;
  std::unique_ptr<Backend> backend_;
  NodeAgentConfig cfg_;
  std::vector<GpuInfo> gpus_;
  DiagOutcome diag_;
  std::unique_ptr<TelemetryPoller> poller_;
  std::unique_ptr<DevicePlugin> plugin_;
  std::mutex publish_mu_;
  CancelToken stop_;
  std::thread heartbeat_;
  std::thread node_watch_;
  std::atomic<bool> node_present_{true};
  std::atomic<uint64_t> publishes_{0};
};

}  // namespace bgc::gpu

// MI355X node agent (north-star N3): advertises each healthy MI355X as an `amd.com/gpu`
// extended resource and publishes topology labels so RCCL TP/DP/PP pods can be
// co-scheduled on one xGMI island.
//
//   labels       amd.com/gpu.present=true, .family=gfx950, .product=MI355X, .count=8,
//                .vram-gb=288, .xgmi-hive-id=<hex>, .compute-partition=SPX,
//                .memory-partition=NPS1, .cu-count=256, .healthy-count=8, .diag=passed
//   annotation   amd.com/gpu.topology = JSON [{index,uuid,bdf,hive,node,numa,render,
//                links:[{peer,type,hops,weight,bw}]}] (the measured amdsmi link map)
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
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "core/env_config.h"
#include "core/json.h"
#include "gpu/device.h"
#include "gpu/device_plugin.h"
#include "gpu/diag.h"
#include "gpu/diag_runner.h"
#include "gpu/telemetry.h"
#include "kube/client.h"
#include "kube/events.h"

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
  // a telemetry poll stuck this long marks every GPU unhealthy until one completes (0 = off)
  uint64_t telemetry_stall_ms = 30000;
  // a shutdown still running after this long exits anyway (under the kubelet's 30 s grace)
  uint64_t shutdown_timeout_secs = 20;
  std::string resource_name = "amd.com/gpu";
  // When every GPU runs a sub-device compute partition (DPX/QPX/CPX: one logical device
  // per partition), the devices are advertised under this name instead — the key the
  // synchronizer writes for the sheet's partition column (reference: the MIG column,
  // src/synchronizer.rs:276).  Empty = always `resource_name`.
  std::string partition_resource_name = "amd.com/gpu-partition";
  std::string label_prefix = "amd.com/gpu";
  int max_gpus = 0;                    // 0 = all discovered
  // HIP diagnostics (gpu/diag.h): HBM pattern + bandwidth, per-CU MFMA tiles + rate,
  // per-XCC balance and an MFMA GEMM checked against a host fp32 product.  They run
  // before the first advertisement and then every `diag_interval_secs` on GPUs that no
  // container holds (kubelet pod-resources API, else amdsmi's process list); a GPU that
  // fails a check or a floor is advertised Unhealthy until a later run passes.
  //
  // Every GPU is diagnosed on its own thread and the burn-in is one node-level phase
  // (gpu/diag_runner.h).  A periodic pass first fences its GPUs in the device plugin
  // (listed Unhealthy, refused by Allocate), waits `diag_fence_settle_ms` for an
  // in-flight admission to land, re-checks that they are still free and only then runs.
  bool run_diag = false;
  // GPUs that a container (pod-resources) or a process (amdsmi) holds when the agent
  // starts: "skip" leaves them without a verdict until a periodic pass finds them free;
  // "diagnose" runs the start-up pass on them anyway (a fresh node, or a test whose own
  // process holds the GPU)
  std::string diag_start_busy = "skip";
  uint64_t diag_hbm_bytes = 1ULL << 30;  // bandwidth phases (two buffers)
  uint64_t diag_interval_secs = 0;     // 0 = only at start
  // Address-pattern walk of this share of each GPU's free VRAM (0 = off), in chunks, with
  // a time budget after which the second (inverse) pass is skipped.
  double diag_hbm_walk_fraction = 0.9;
  uint64_t diag_hbm_walk_chunk_mb = 4096;
  uint64_t diag_hbm_walk_budget_ms = 20000;
  uint64_t diag_fence_settle_ms = 2000;
  // Burn-in: sustained MFMA load for this long while power, clocks, temperatures and
  // throttle residency are sampled (catches cooling/power-delivery faults the short
  // checks do not); 0 = off.
  uint64_t diag_burn_ms = 0;
  // its matrix-core path.  "fp4" (MX block-scaled) drives an MI355X to its power cap:
  // 1.30 kW mean, power-limited 71 % of the time, against 1.08-1.17 kW for "bf16" and
  // 1.21 kW for "fp8" (profiles/mx_lowp_r3/burn_dtype.json), so it is the hardest
  // power-delivery and cooling stress.  The bf16 rate floor scales with the dtype.
  std::string diag_burn_dtype = "fp4";
  // PCIe check: pinned host<->device copies of this size (0 = off) with the link's
  // width/speed read while they run.
  uint64_t diag_pcie_bytes = 256ULL << 20;
  // GEMM soak: `diag_soak_launches` back-to-back LDS-tiled MFMA GEMMs of size^3 (bf16),
  // checked by exact checksums (0 launches = off).
  int diag_soak_size = 8192;
  int diag_soak_launches = 20;
  // MX block-scaled fp8 / fp4 matrix-core tiles (with and without E8M0 scales) and rates
  bool diag_lowp = true;
  DiagFloors diag_floors = DiagFloors::mi355x_defaults();
  std::string pod_resources_socket = "/var/lib/kubelet/pod-resources/kubelet.sock";
  HealthPolicy health;
  int slow_every = 10;                 // polls between VRAM/ECC-total reads
  int ras_every = 60;                  // polls between bad-page / per-block ECC / link reads
  bool create_node = false;            // test clusters without a kubelet
  // Events on the Node (kubectl describe node): GPUUnhealthy / GPUHealthy transitions and
  // GPUDiagnosticsFailed, aggregated and rate limited (kube/events.h).
  bool events = true;
  // Kubelet device plugin (gpu/device_plugin.h).  When on, the kubelet owns the
  // amd.com/gpu capacity/allocatable counts, so the Node status patch carries only the
  // AMDGPUHealthy condition; labels and topology are published as before.
  bool device_plugin = false;
  std::string device_plugin_dir = "/var/lib/kubelet/device-plugins";
  std::string device_plugin_socket = "bgc-amd-gpu.sock";
  bool device_plugin_cdi = false;        // answer Allocate with CDI device names (DevicePluginConfig::cdi)
  std::string cdi_dir = "/var/run/cdi";
  std::string dev_root = "/dev";
  std::string sysfs_root = "/sys";
  // Coexistence with another advertiser of the same GPUs (an MI355X node commonly runs
  // AMD's GPU Operator: its device plugin registers amd.com/gpu and its labeller owns
  // amd.com/gpu.* labels).  At start and on every heartbeat the agent looks for
  //   * another live device plugin in device_plugin_dir serving resource_name
  //     (foreign_plugins_for), and
  //   * another field manager on the Node owning status.capacity/allocatable[resource_name],
  //     or owning label_prefix.* labels as a labelling controller: a server-side apply
  //     (not kubectl's) or one of known_labellers (foreign_field_owners).  A one-off
  //     `kubectl label` by an admin is reported but is no conflict;
  // on a finding it logs an error, records a Warning Event (GPUAdvertiserConflict) and
  // stands down: no device-plugin registration, no label or status writes.  A plugin
  // stopped for a conflict found while advertising starts again once a heartbeat finds
  // the conflict gone.  take_over (CONF_TAKE_OVER) advertises anyway (Event
  // GPUAdvertiserTakeOver).
  bool advertiser_check = true;
  bool take_over = false;
  // Field managers that label GPU nodes (CONF_KNOWN_LABELLERS, comma list): AMD's node
  // labeller, node-feature-discovery.
  std::vector<std::string> known_labellers = {"amdgpu-node-labeller", "amd-gpu-node-labeller", "node-labeller",
                                              "nfd-master", "nfd-worker"};
  static NodeAgentConfig from_env(const EnvConfig& env);
};

struct DiagOutcome {
  bool ran = false;
  bool passed = true;
  json::Value per_gpu = json::Value::array();  // judged results, one per GPU (null = not run)
  uint64_t runs = 0;
  uint64_t skipped_in_use = 0;
  double last_pass_ms = 0;             // wall time of the last pass
  uint64_t last_diagnosed = 0;         // GPUs the last pass ran on
  json::Value node_burn;               // node-level burn summary of the last pass (null = none)
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
// Field managers of `node` other than this agent that own what it advertises:
// [{"kind":"labels"|"capacity","manager":..,"operation":..,"fields":[..],"conflict":bool}].
// The kubelet's capacity/allocatable entries are its device-plugin bookkeeping and count
// only when the agent itself advertises through the Node status (no device plugin of its
// own).  Label owners are a conflict only as labelling controllers (label_owner_conflicts).
json::Value foreign_field_owners(const NodeAgentConfig& cfg, const json::Value& node);
// A foreign owner of label_prefix.* labels is another labeller unless it is kubectl (an
// admin's one-off `kubectl label/edit/patch`): most labelling controllers write with Update
// under a manager named after their binary, so neither the operation nor a list of known
// names can tell them apart.  known_labellers are a conflict even under a kubectl-prefixed
// name.
bool label_owner_conflicts(const NodeAgentConfig& cfg, const std::string& manager, const std::string& operation);

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
  // One diagnostics pass over every GPU not held by a container; returns true when any
  // GPU's verdict changed (and then re-publishes health).  `force` ignores allocation.
  bool run_diagnostics(bool at_start = false);
  DiagOutcome diag_outcome() const;
  // Another advertiser found by the last check (see NodeAgentConfig::advertiser_check).
  bool standing_down() const { return standing_down_.load(); }
  json::Value advertiser_conflicts() const;
  // Runs the coexistence check now; returns true when the agent stands down.
  bool check_advertisers();

 private:
  int healthy_count(std::string* reason) const;
  DiagPlan diag_plan() const;
  void setup_diag();  // engine + HIP device ids (by BDF); idempotent
  void record_diag_gauges(size_t i, const json::Value& judged);
  std::vector<bool> in_use() const;
  std::unique_ptr<DiagEngine> engine_;
  std::vector<int> hip_devs_;          // HIP device id per GPU (diag_runner.h hip_devices_for)
  std::atomic<uint64_t> fence_races_{0};  // GPUs released because an allocation raced the fence
  // start-up timeline (ms since the agent was constructed)
  std::chrono::steady_clock::time_point t_created_ = std::chrono::steady_clock::now();
  double discover_ms_ = 0, startup_diag_ms_ = 0;
  std::atomic<double> first_advertise_ms_{0};
  void mark_advertised();
  void on_health_changed();
  kube::KubeClient& client_;
  std::unique_ptr<Backend> backend_;
  NodeAgentConfig cfg_;
  std::vector<GpuInfo> gpus_;
  mutable std::mutex diag_mu_;  // guards diag_ (the diag thread updates it)
  DiagOutcome diag_;
  std::thread diag_thread_;
  std::unique_ptr<TelemetryPoller> poller_;
  std::unique_ptr<DevicePlugin> plugin_;
  bool diag_in_process_ = false;
  std::string pcie_lock_path_;
  std::mutex publish_mu_;
  CancelToken stop_;
  std::thread heartbeat_;
  std::thread node_watch_;
  std::atomic<bool> node_present_{true};
  std::atomic<uint64_t> publishes_{0};
  std::unique_ptr<kube::EventRecorder> events_;
  std::atomic<bool> standing_down_{false};
  std::atomic<bool> plugin_started_{false};
  std::atomic<bool> plugin_stopped_{false};  // stopped for a conflict found while advertising
  // Serialises the plugin's start/stop transitions with NodeAgent::stop(): once stop() has
  // taken it and cancelled stop_, no heartbeat restarts (re-registers) the plugin.
  std::mutex plugin_mu_;
  mutable std::mutex conflict_mu_;
  json::Value conflicts_ = json::Value::array();
  std::string conflict_sig_;  // last conflict set reported (one Event per change)
  void start_plugin();
  std::mutex event_mu_;
  std::vector<int> event_state_;  // per GPU: -1 not reported yet, 1 healthy, 0 unhealthy
  void emit_health_events();
  void node_event(const std::string& type, const std::string& reason, const std::string& message);
  std::string gpu_reason(size_t i) const;  // why GPU i is unhealthy ("" when healthy)
};

}  // namespace bgc::gpu

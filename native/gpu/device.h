// MI355X device discovery + telemetry backends (north-star components N1/N2; the
// reference has no GPU code at all — its only GPU touch-point is the quota key
// `requests.nvidia.com/gpu`, reference src/synchronizer.rs:268).
//
// Backends:
//   * amdsmi : libamd_smi.so (ROCm 7.2) resolved with dlopen at runtime, so binaries and
//              the Python module load on hosts without a GPU driver.
//   * mock   : JSON fixture describing N devices (CI / multi-node tests without GPUs).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "core/json.h"

namespace bgc::gpu {

// Connection from one GPU to another discovered GPU (amdsmi_topo_get_link_type,
// amdsmi_topo_get_link_weight, amdsmi_get_minmax_bandwidth_between_processors).
struct PeerLink {
  int peer = -1;               // GpuInfo::index of the other end
  std::string type;            // "xgmi" | "pcie" | "internal" | "n/a" | "unknown"
  uint64_t hops = 0;
  uint64_t weight = 0;         // KFD io-link weight (lower = closer)
  uint64_t min_bw_mbps = 0;    // theoretical, 1-hop xGMI only (0 = unknown)
  uint64_t max_bw_mbps = 0;
};

// One physical xGMI/PCIe link of a GPU (amdsmi_get_link_metrics).  The peer is named by
// BDF, so this also describes links to GPUs that are not visible to this process.
struct PhysLink {
  std::string peer_bdf;
  std::string type;
  uint32_t bit_rate_gbps = 0;       // current link speed (0 = down)
  uint32_t max_bandwidth_gbps = 0;
  uint64_t read_kb = 0, write_kb = 0;  // cumulative traffic
};

struct EccBlock {
  std::string block;  // umc, gfx, sdma, xgmi_wafl, ...
  uint64_t correctable = 0, uncorrectable = 0, deferred = 0;
};

struct GpuInfo {
  int index = 0;             // enumeration order (== HIP device id for amdsmi)
  std::string uuid;
  std::string bdf;           // 0000:05:00.0
  std::string market_name;   // "AMD Instinct MI355X"
  std::string vendor_name;
  std::string gfx_target;    // "gfx950"
  std::string serial;
  uint64_t vram_total_mb = 0;
  uint64_t vram_max_bandwidth_gbps = 0;
  uint32_t num_cus = 0;
  uint64_t xgmi_hive_id = 0;
  uint64_t xgmi_node_id = 0;
  uint32_t xgmi_lanes = 0;
  int numa_node = -1;
  std::string compute_partition;  // SPX/DPX/QPX/CPX
  std::string memory_partition;   // NPS1/NPS2
  uint32_t power_cap_w = 0;
  int hip_id = -1;
  // DRM minors of this logical device (amdsmi_get_gpu_enumeration_info).  Compute
  // partitions of one GPU share a BDF but each has its own render node; -1 = unknown.
  int drm_render = -1;
  int drm_card = -1;
  uint32_t bad_page_threshold = 0;   // driver's retirement limit (0 = unknown / no root)
  // PCIe link capability (amdsmi_get_pcie_info static part); -1 = unknown
  int pcie_max_width = -1;       // lanes
  int pcie_max_speed_mts = -1;   // per-lane rate, MT/s (Gen5 = 32000)
  int pcie_max_gen = -1;
  // Software/firmware identity (amdsmi_get_gpu_driver_info, amdsmi_get_gpu_vbios_info):
  // published as node labels so a driver or VBIOS rollout can be tracked per node.
  std::string driver_name;      // "amdgpu"
  std::string driver_version;   // "6.16.6" (empty = unknown)
  std::string vbios_version;
  std::string vbios_part_number;
  std::vector<PeerLink> links;       // to every other discovered GPU
  std::vector<PhysLink> phys_links;  // physical links at discovery time
};

struct Telemetry {
  int index = 0;
  int64_t ts_ns = 0;
  bool ok = false;
  std::string error;
  double gfx_activity_pct = 0;
  double umc_activity_pct = 0;
  double power_w = 0;
  double temp_edge_c = 0;
  double temp_hotspot_c = 0;
  double temp_mem_c = 0;
  uint64_t vram_used_mb = 0;
  uint64_t vram_total_mb = 0;
  uint32_t gfxclk_mhz = 0;
  uint32_t uclk_mhz = 0;
  bool throttle_valid = false;  // false when the firmware reports the all-ones sentinel
  uint64_t throttle_status = 0;
  // Violation (throttle residency) accumulators from gpu_metrics; the poller turns the
  // deltas between two samples into percentages.  kNoAcc = not reported.
  uint64_t acc_counter = kNoAcc;
  uint64_t acc_ppt = kNoAcc;       // package power tracking
  uint64_t acc_thermal = kNoAcc;   // max of socket / HBM / VR / PROCHOT residency
  double violation_ppt_pct = -1;     // over the last poll interval (-1 = unknown)
  double violation_thermal_pct = -1;
  uint64_t ecc_correctable = 0;
  uint64_t ecc_uncorrectable = 0;
  uint64_t ecc_deferred = 0;
  int xgmi_links_up = -1;     // -1 = unknown
  int xgmi_links_total = -1;
  // PCIe link state (Slow level; amdsmi_get_pcie_info metric part); -1 = unknown.  The
  // error counters are cumulative since boot: the poller watches their deltas.
  int pcie_width = -1;
  int pcie_speed_mts = -1;
  int64_t pcie_replays = -1;
  int64_t pcie_recoveries = -1;   // L0 -> recovery transitions
  int64_t pcie_nak_sent = -1;
  int64_t pcie_nak_received = -1;
  // RAS level only (SampleLevel::Ras); `ras_ok` says whether they were read.
  bool ras_ok = false;
  uint64_t retired_pages = 0;       // reserved + pending
  uint64_t unreservable_pages = 0;  // bad pages the driver could not retire
  std::vector<EccBlock> ecc_blocks;
  std::vector<PhysLink> links;
  double poll_us = 0;         // cost of this sample

  static constexpr uint64_t kNoAcc = ~0ULL;
};

// What one sample() reads.  Costs per device on MI355X / ROCm 7.2
// (profiles/archive/amdsmi_cost_r1.json, profiles/archive/amdsmi_cost_r2.json):
//   Fast : the gpu_metrics blob (activity, power, temps, clocks, throttle, violation
//          accumulators, xGMI link status)                              ~280 us
//   Slow : + VRAM usage and total ECC counts                           ~+750 us
//   Ras  : + retired/bad pages, per-block ECC, xGMI link metrics        measured r2
// The poller reads Fast every interval, Slow every `slow_every` and Ras every
// `ras_every` polls, caching the slower fields in between.
enum class SampleLevel : int { Fast = 0, Slow = 1, Ras = 2 };

class Backend {
 public:
  virtual ~Backend() = default;
  virtual std::string name() const = 0;
  virtual std::vector<GpuInfo> discover() = 0;
  virtual Telemetry sample(int index, SampleLevel level = SampleLevel::Ras) = 0;
  // Compute processes currently holding the device (-1 = unknown).
  virtual int busy_processes(int index) { (void)index; return -1; }
  // Every process the driver lists on the device: [{pid, name, vram_bytes, gtt_bytes,
  // gfx_ns, holds}] (holds = counted by busy_processes); empty when unknown.
  virtual json::Value processes(int index) { (void)index; return json::Value::array(); }
  // Mock backends only: a scripted diagnostics engine (diag_runner.h) instead of the HIP
  // kernels; null = run the real diagnostics.
  virtual json::Value diag_script() { return json::Value(); }
};

const char* link_type_name(int amdsmi_link_type);

// Throws std::runtime_error when libamd_smi is missing or amdsmi_init fails.
std::unique_ptr<Backend> make_amdsmi_backend();
// fixture: {"gpus":[{<GpuInfo fields>, "telemetry": {<Telemetry fields>}}]}
std::unique_ptr<Backend> make_mock_backend(const json::Value& fixture);
// kind: "amdsmi" | "mock" | "auto" (amdsmi, else mock fixture when given).
std::unique_ptr<Backend> make_backend(const std::string& kind, const std::string& mock_fixture_path);

// Default 8x MI355X hive used by tests and the mock node-agent (288 GB HBM3E each,
// one xGMI hive, 256 CUs, gfx950).
json::Value default_mi355x_fixture(int n_gpus = 8, uint64_t hive_id = 0x1a2b3c4d5e6f7788ULL);

json::Value to_json(const GpuInfo& g);
json::Value to_json(const Telemetry& t);
json::Value to_json(const PeerLink& l);
json::Value to_json(const PhysLink& l);
GpuInfo gpu_info_from_json(const json::Value& v);
PeerLink peer_link_from_json(const json::Value& v);
// Health-relevant fields only (tests drive the state machine with these).
Telemetry telemetry_from_json(const json::Value& v);
PhysLink phys_link_from_json(const json::Value& v);

}  // namespace bgc::gpu

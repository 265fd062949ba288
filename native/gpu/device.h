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
  uint64_t throttle_status = 0;
  uint64_t ecc_correctable = 0;
  uint64_t ecc_uncorrectable = 0;
  int xgmi_links_up = -1;     // -1 = unknown
  int xgmi_links_total = -1;
  double poll_us = 0;         // cost of this sample
};

class Backend {
 public:
  virtual ~Backend() = default;
  virtual std::string name() const = 0;
  virtual std::vector<GpuInfo> discover() = 0;
  // `full` also reads the slow counters (ECC totals ~670 us, VRAM usage ~80 us per
  // device on MI355X/ROCm 7.2, vs ~280 us for the gpu_metrics blob); when false those
  // fields are left zero and the caller keeps its cached values.
  virtual Telemetry sample(int index, bool full = true) = 0;
};

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
GpuInfo gpu_info_from_json(const json::Value& v);

}  // namespace bgc::gpu

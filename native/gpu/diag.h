// Loader for libbgc_gpu_diag.so (HIP/CDNA4 health kernels, native/gpu/hip/).
#pragma once

#include <cstdint>
#include <string>

#include "core/json.h"
#include "gpu/hip/gpu_diag.h"

namespace bgc::gpu {

// Performance floors that turn the diagnostics into a health gate: a GPU whose HBM or
// matrix cores run well below what an MI355X delivers is not advertised, even when every
// pattern and tile checks out.  Defaults sit ~25 % under the rates measured on MI355X at
// the node agent's default sizes (profiles/archive/diag_floors_r2.json); 0 disables a floor.
struct DiagFloors {
  double min_read_gbps = 0;
  double min_copy_gbps = 0;
  double min_write_gbps = 0;
  double min_mfma_tflops = 0;
  double min_xcc_balance = 0;  // slowest XCC mean wave time / fastest, inverted (0..1]
  // MX block-scaled low-precision matrix cores (`lowp` section): any wrong tile fails;
  // rate floors for the dense fp8 and fp4 phases.
  double min_fp8_tflops = 0;
  double min_fp4_tflops = 0;
  int min_xccs = 0;            // XCCs that must have run MFMA work
  // Burn-in (sustained MFMA load, `burn` section): rate floor, the rate may not sag
  // below this fraction of its first launch, and the thermal limits under load.
  double min_burn_tflops = 0;
  double min_burn_sustain = 0;   // tflops_last / tflops_max
  double max_burn_hotspot_c = 0;
  double max_burn_thermal_violation_pct = 0;
  // PCIe (`pcie` section): host<->device DMA rates, and the link must run at its full
  // width (and at least this fraction of its top speed) while the copies run.
  double min_pcie_h2d_gbps = 0;
  double min_pcie_d2h_gbps = 0;
  bool require_full_pcie_width = false;
  double min_pcie_speed_fraction = 0;
  // GEMM soak (`soak` section): every checksum must match; rate floor on the mean.
  double min_soak_tflops = 0;
  // HBM walk (`hbm_walk` section): any mismatch fails; the walk must cover at least this
  // share of the free VRAM (a failed allocation on an idle, fenced GPU means something
  // else holds its memory).
  double min_hbm_walk_coverage = 0;
  // Node-level burn (diag_runner.h): under the shared load every GPU must reach this
  // fraction of the node's fastest GPU, and the summed draw must stay under the limit.
  double min_node_burn_balance = 0;
  double max_node_power_w = 0;
  static DiagFloors mi355x_defaults();
};

// Burn dtype names ("bf16", "fp8", "fp4") <-> BGC_BURN_*; the name throws on anything else.
int burn_dtype_code(const std::string& name);
const char* burn_dtype_name(int code);
// Dense-rate ratio of a burn dtype to bf16 on MI355X, as the burn kernels measure it (fp8
// 2.0x, fp4 3.5x; profiles/mx_lowp_r3/): the bf16 burn floor scales by it.
double burn_dtype_rate_ratio(int code);

// Pure verdict over one GPU's results ({"hbm":…, "mfma":…, "gemm":…}): adds "passed" and
// "failures" (one string per violated check) to a copy of `result`.
json::Value judge_diag(const json::Value& result, const DiagFloors& floors);

class Diag {
 public:
  // Searches $BGC_GPU_DIAG_LIB, then <exe dir>/../bacchus_gpu_controller_amd/, then the
  // dynamic linker path. Throws std::runtime_error if not found.
  static Diag& instance(const std::string& explicit_path = "");
  int device_count();
  std::string device_arch(int device);
  json::Value hbm(int device, uint64_t bytes, int iters, uint32_t seed);
  json::Value mfma(int device, int waves_per_cu, int throughput_iters, uint32_t seed);
  // MX block-scaled fp8 / fp4 matrix-core tiles and rates (see bgc_diag_mfma_lowp).
  json::Value mfma_lowp(int device, int waves_per_cu, int throughput_iters, uint32_t seed);
  // MFMA GEMM on the device vs a host fp32 product of the same bf16 operands
  // (deterministic pseudo-random values in [-1, 1]).  Returns max error and the bound.
  json::Value gemm_check(int device, int m, int n, int k, uint32_t seed);
  // Sustained MFMA load for duration_ms (see bgc_diag_burn_dtype; dtype BGC_BURN_*).
  json::Value burn(int device, int duration_ms, int waves_per_cu, uint32_t seed, int dtype = BGC_BURN_BF16);
  // Pinned host <-> device copies (see bgc_diag_pcie).
  json::Value pcie(int device, uint64_t bytes, int iters, uint32_t seed);
  // LDS-tiled MFMA GEMM run back to back, checked by exact checksums (bgc_diag_gemm_soak).
  json::Value gemm_soak(int device, int m, int n, int k, int launches, uint32_t seed);
  // Raw GEMM: A/B as bf16 bit patterns, C fp32 (row-major).
  void gemm(int device, int m, int n, int k, const uint16_t* a, const uint16_t* b, float* c);
  // The soak's LDS-tiled GEMM on caller operands (Bt = B transposed, [n][k]).
  void gemm_tiled(int device, int m, int n, int k, const uint16_t* a, const uint16_t* bt, float* c);
  // MX fp8 (fmt 0) / fp4 (fmt 4) block-scaled GEMM on caller codes and E8M0 scales
  void mx_gemm(int device, int fmt, int m, int n, int k, const uint8_t* a, const uint8_t* a_scales, const uint8_t* bt,
               const uint8_t* bt_scales, float* c);
  // Address-pattern walk of `fraction` of the free VRAM (see bgc_diag_hbm_walk).
  json::Value hbm_walk(int device, double fraction, uint64_t chunk_bytes, int budget_ms, uint32_t seed);
  // PCI bus id of a HIP device, lower-case ("0000:05:00.0").
  std::string device_bdf(int device);
  const std::string& path() const { return path_; }

 private:
  explicit Diag(const std::string& path);
  std::string path_;
  void* lib_ = nullptr;
  int (*device_count_)() = nullptr;
  int (*hbm_)(int, uint64_t, int, uint32_t, bgc_hbm_result*) = nullptr;
  int (*mfma_)(int, int, int, uint32_t, bgc_mfma_result*) = nullptr;
  int (*lowp_)(int, int, int, uint32_t, bgc_lowp_result*) = nullptr;
  int (*arch_)(int, char*, size_t) = nullptr;
  int (*gemm_)(int, int, int, int, const uint16_t*, const uint16_t*, float*) = nullptr;
  int (*burn_)(int, int, int, uint32_t, int, bgc_burn_result*) = nullptr;
  int (*pcie_)(int, uint64_t, int, uint32_t, bgc_pcie_result*) = nullptr;
  int (*soak_)(int, int, int, int, int, uint32_t, bgc_soak_result*) = nullptr;
  int (*tiled_)(int, int, int, int, const uint16_t*, const uint16_t*, float*) = nullptr;
  int (*mx_gemm_)(int, int, int, int, int, const uint8_t*, const uint8_t*, const uint8_t*, const uint8_t*,
                  float*) = nullptr;
  int (*walk_)(int, double, uint64_t, int, uint32_t, bgc_hbm_walk_result*) = nullptr;
  int (*bdf_)(int, char*, size_t) = nullptr;
  const char* (*last_error_)() = nullptr;
};

}  // namespace bgc::gpu

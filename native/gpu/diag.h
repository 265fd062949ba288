// Loader for libbgc_gpu_diag.so (HIP/CDNA4 health kernels, native/gpu/hip/).
#pragma once

#include <string>

#include "core/json.h"
#include "gpu/hip/gpu_diag.h"

namespace bgc::gpu {

class Diag {
 public:
  // Searches $BGC_GPU_DIAG_LIB, then <exe dir>/../bacchus_gpu_controller_amd/, then the
  // dynamic linker path. Throws std::runtime_error if not found.
  static Diag& instance(const std::string& explicit_path = "");
  int device_count();
  std::string device_arch(int device);
  json::Value hbm(int device, uint64_t bytes, int iters, uint32_t seed);
  json::Value mfma(int device, int waves_per_cu, int throughput_iters, uint32_t seed);
  const std::string& path() const { return path_; }

 private:
  explicit Diag(const std::string& path);
  std::string path_;
  void* lib_ = nullptr;
  int (*device_count_)() = nullptr;
  int (*hbm_)(int, uint64_t, int, uint32_t, bgc_hbm_result*) = nullptr;
  int (*mfma_)(int, int, int, uint32_t, bgc_mfma_result*) = nullptr;
  int (*arch_)(int, char*, size_t) = nullptr;
  const char* (*last_error_)() = nullptr;
};

}  // namespace bgc::gpu

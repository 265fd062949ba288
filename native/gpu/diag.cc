#include "gpu/diag.h"

#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <mutex>
#include <stdexcept>

namespace bgc::gpu {

namespace {

std::string exe_dir() {
  char buf[4096];
  ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p(buf);
  return p.substr(0, p.rfind('/'));
}

std::string so_dir() {
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&exe_dir), &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    size_t s = p.rfind('/');
    if (s != std::string::npos) return p.substr(0, s);
  }
  return ".";
}

}  // namespace

Diag::Diag(const std::string& path) : path_(path) {
  lib_ = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!lib_) throw std::runtime_error("cannot load " + path + ": " + dlerror());
  device_count_ = reinterpret_cast<int (*)()>(dlsym(lib_, "bgc_diag_device_count"));
  hbm_ = reinterpret_cast<int (*)(int, uint64_t, int, uint32_t, bgc_hbm_result*)>(dlsym(lib_, "bgc_diag_hbm"));
  mfma_ = reinterpret_cast<int (*)(int, int, int, uint32_t, bgc_mfma_result*)>(dlsym(lib_, "bgc_diag_mfma"));
  lowp_ = reinterpret_cast<int (*)(int, int, int, uint32_t, bgc_lowp_result*)>(dlsym(lib_, "bgc_diag_mfma_lowp"));
  arch_ = reinterpret_cast<int (*)(int, char*, size_t)>(dlsym(lib_, "bgc_diag_device_arch"));
  gemm_ = reinterpret_cast<int (*)(int, int, int, int, const uint16_t*, const uint16_t*, float*)>(
      dlsym(lib_, "bgc_diag_gemm"));
  burn_ = reinterpret_cast<int (*)(int, int, int, uint32_t, int, bgc_burn_result*)>(dlsym(lib_, "bgc_diag_burn_dtype"));
  pcie_ = reinterpret_cast<int (*)(int, uint64_t, int, uint32_t, bgc_pcie_result*)>(dlsym(lib_, "bgc_diag_pcie"));
  soak_ = reinterpret_cast<int (*)(int, int, int, int, int, uint32_t, bgc_soak_result*)>(dlsym(lib_, "bgc_diag_gemm_soak"));
  tiled_ = reinterpret_cast<int (*)(int, int, int, int, const uint16_t*, const uint16_t*, float*)>(
      dlsym(lib_, "bgc_diag_gemm_tiled"));
  mx_gemm_ = reinterpret_cast<int (*)(int, int, int, int, int, const uint8_t*, const uint8_t*, const uint8_t*,
                                      const uint8_t*, float*)>(dlsym(lib_, "bgc_diag_mx_gemm"));
  walk_ = reinterpret_cast<int (*)(int, double, uint64_t, int, uint32_t, bgc_hbm_walk_result*)>(
      dlsym(lib_, "bgc_diag_hbm_walk"));
  bdf_ = reinterpret_cast<int (*)(int, char*, size_t)>(dlsym(lib_, "bgc_diag_device_bdf"));
  last_error_ = reinterpret_cast<const char* (*)()>(dlsym(lib_, "bgc_diag_last_error"));
  auto abi = reinterpret_cast<int (*)()>(dlsym(lib_, "bgc_diag_abi_version"));
  if (!device_count_ || !hbm_ || !mfma_ || !lowp_ || !arch_ || !gemm_ || !burn_ || !pcie_ || !soak_ || !tiled_ ||
      !mx_gemm_ || !walk_ || !bdf_ || !last_error_ || !abi ||
      abi() != BGC_DIAG_ABI_VERSION) {
    throw std::runtime_error(path + " is not a compatible bgc diag library");
  }
}

Diag& Diag::instance(const std::string& explicit_path) {
  static std::mutex mu;
  static Diag* d = nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (d) return *d;
  std::vector<std::string> candidates;
  if (!explicit_path.empty()) candidates.push_back(explicit_path);
  if (const char* e = std::getenv("BGC_GPU_DIAG_LIB")) candidates.emplace_back(e);
  candidates.push_back(so_dir() + "/libbgc_gpu_diag.so");
  candidates.push_back(exe_dir() + "/../bacchus_gpu_controller_amd/libbgc_gpu_diag.so");
  candidates.push_back("libbgc_gpu_diag.so");
  std::string errors;
  for (const auto& c : candidates) {
    if (c.find('/') != std::string::npos && access(c.c_str(), R_OK) != 0) continue;
    try {
      d = new Diag(c);
      return *d;
    } catch (const std::exception& e) {
      errors += std::string(e.what()) + "; ";
    }
  }
  throw std::runtime_error("libbgc_gpu_diag.so not found: " + errors);
}

int Diag::device_count() { return device_count_(); }

std::string Diag::device_arch(int device) {
  char buf[128] = {0};
  if (arch_(device, buf, sizeof(buf)) != 0) throw std::runtime_error(last_error_());
  return buf;
}

json::Value Diag::hbm(int device, uint64_t bytes, int iters, uint32_t seed) {
  bgc_hbm_result r{};
  if (hbm_(device, bytes, iters, seed, &r) != 0) throw std::runtime_error(std::string("hbm diag: ") + last_error_());
  json::Value v = json::Value::object();
  v["device"] = device;
  v["bytes"] = static_cast<unsigned long long>(r.bytes);
  v["iters"] = r.iters;
  v["write_gbps"] = r.write_gbps;
  v["read_gbps"] = r.read_gbps;
  v["copy_gbps"] = r.copy_gbps;
  v["mismatches"] = static_cast<unsigned long long>(r.mismatches);
  v["first_bad_word"] = r.first_bad_word == ~0ULL ? json::Value() : json::Value(static_cast<unsigned long long>(r.first_bad_word));
  v["elapsed_ms"] = r.elapsed_ms;
  v["passed"] = r.mismatches == 0;
  return v;
}

json::Value Diag::mfma(int device, int waves_per_cu, int throughput_iters, uint32_t seed) {
  bgc_mfma_result r{};
  if (mfma_(device, waves_per_cu, throughput_iters, seed, &r) != 0) {
    throw std::runtime_error(std::string("mfma diag: ") + last_error_());
  }
  json::Value v = json::Value::object();
  v["device"] = device;
  v["tiles_checked"] = static_cast<unsigned long long>(r.tiles_checked);
  v["mismatches"] = static_cast<unsigned long long>(r.mismatches);
  v["cus_seen"] = r.cus_seen;
  v["xccs_seen"] = r.xccs_seen;
  v["bad_cus"] = r.bad_cus;
  json::Value bad = json::Value::array();
  for (int i = 0; i < r.bad_cus && i < 64; ++i) bad.push_back(r.bad_cu_keys[i]);
  v["bad_cu_keys"] = bad;
  v["tflops"] = r.tflops;
  v["throughput_ok"] = r.throughput_ok != 0;
  json::Value xw = json::Value::array(), xus = json::Value::array();
  for (int x = 0; x < 8; ++x) {
    xw.push_back(r.xcc_waves[x]);
    xus.push_back(r.xcc_wave_us[x]);
  }
  v["xcc_waves"] = xw;
  v["xcc_wave_us"] = xus;
  v["xcc_balance"] = r.xcc_balance;
  v["elapsed_ms"] = r.elapsed_ms;
  v["passed"] = r.mismatches == 0 && r.throughput_ok != 0;
  return v;
}

json::Value Diag::mfma_lowp(int device, int waves_per_cu, int throughput_iters, uint32_t seed) {
  bgc_lowp_result r{};
  if (lowp_(device, waves_per_cu, throughput_iters, seed, &r) != 0) {
    throw std::runtime_error(std::string("low-precision mfma diag: ") + last_error_());
  }
  json::Value bad = json::Value::array();
  for (int i = 0; i < r.bad_cus && i < 64; ++i) bad.push_back(r.bad_cu_keys[i]);
  const uint64_t mism = r.fp8_mismatches + r.fp8_scaled_mismatches + r.fp4_mismatches + r.fp4_scaled_mismatches;
  return json::Value::object({{"device", device},
                              {"tiles_checked", static_cast<unsigned long long>(r.tiles_checked)},
                              {"fp8_mismatches", static_cast<unsigned long long>(r.fp8_mismatches)},
                              {"fp8_scaled_mismatches", static_cast<unsigned long long>(r.fp8_scaled_mismatches)},
                              {"fp4_mismatches", static_cast<unsigned long long>(r.fp4_mismatches)},
                              {"fp4_scaled_mismatches", static_cast<unsigned long long>(r.fp4_scaled_mismatches)},
                              {"mismatches", static_cast<unsigned long long>(mism)},
                              {"cus_seen", r.cus_seen},
                              {"bad_cus", r.bad_cus},
                              {"bad_cu_keys", bad},
                              {"fp8_tflops", r.fp8_tflops},
                              {"fp4_tflops", r.fp4_tflops},
                              {"throughput_ok", r.throughput_ok != 0},
                              {"elapsed_ms", r.elapsed_ms},
                              {"passed", mism == 0 && r.throughput_ok != 0}});
}

json::Value Diag::burn(int device, int duration_ms, int waves_per_cu, uint32_t seed, int dtype) {
  bgc_burn_result r{};
  if (burn_(device, duration_ms, waves_per_cu, seed, dtype, &r) != 0) {
    throw std::runtime_error(std::string("burn: ") + last_error_());
  }
  return json::Value::object({{"dtype", burn_dtype_name(dtype)}, {"launches", r.launches}, {"elapsed_ms", r.elapsed_ms}, {"tflops_mean", r.tflops_mean},
                              {"tflops_min", r.tflops_min}, {"tflops_first", r.tflops_first},
                              {"tflops_last", r.tflops_last}, {"tflops_max", r.tflops_max},
                              // the last launch against the best: < 1 when the GPU throttled
                              {"sustain", r.tflops_max > 0 ? r.tflops_last / r.tflops_max : 0.0},
                              {"mismatches", static_cast<unsigned long long>(r.mismatches)}});
}

json::Value Diag::pcie(int device, uint64_t bytes, int iters, uint32_t seed) {
  bgc_pcie_result r{};
  if (pcie_(device, bytes, iters, seed, &r) != 0) throw std::runtime_error(std::string("pcie diag: ") + last_error_());
  return json::Value::object({{"device", device}, {"bytes", static_cast<unsigned long long>(r.bytes)},
                              {"iters", r.iters}, {"h2d_gbps", r.h2d_gbps}, {"d2h_gbps", r.d2h_gbps},
                              {"bidir_gbps", r.bidir_gbps}, {"mismatches", static_cast<unsigned long long>(r.mismatches)},
                              {"elapsed_ms", r.elapsed_ms}, {"passed", r.mismatches == 0}});
}

json::Value Diag::gemm_soak(int device, int m, int n, int k, int launches, uint32_t seed) {
  bgc_soak_result r{};
  if (soak_(device, m, n, k, launches, seed, &r) != 0) throw std::runtime_error(std::string("gemm soak: ") + last_error_());
  return json::Value::object({{"device", device}, {"m", r.m}, {"n", r.n}, {"k", r.k}, {"launches", r.launches},
                              {"tile", r.tile}, {"kernel", r.kernel == 2 ? "pingpong" : "2buf"},
                              {"elapsed_ms", r.elapsed_ms}, {"tflops_mean", r.tflops_mean},
                              {"tflops_best", r.tflops_best},
                              {"row_mismatches", static_cast<unsigned long long>(r.row_mismatches)},
                              {"col_mismatches", static_cast<unsigned long long>(r.col_mismatches)},
                              {"passed", r.row_mismatches == 0 && r.col_mismatches == 0}});
}

void Diag::gemm(int device, int m, int n, int k, const uint16_t* a, const uint16_t* b, float* c) {
  if (gemm_(device, m, n, k, a, b, c) != 0) throw std::runtime_error(std::string("gemm diag: ") + last_error_());
}

void Diag::gemm_tiled(int device, int m, int n, int k, const uint16_t* a, const uint16_t* bt, float* c) {
  if (tiled_(device, m, n, k, a, bt, c) != 0) throw std::runtime_error(std::string("tiled gemm: ") + last_error_());
}

void Diag::mx_gemm(int device, int fmt, int m, int n, int k, const uint8_t* a, const uint8_t* a_scales,
                   const uint8_t* bt, const uint8_t* bt_scales, float* c) {
  if (mx_gemm_(device, fmt, m, n, k, a, a_scales, bt, bt_scales, c) != 0) {
    throw std::runtime_error(std::string("mx gemm: ") + last_error_());
  }
}

json::Value Diag::hbm_walk(int device, double fraction, uint64_t chunk_bytes, int budget_ms, uint32_t seed) {
  bgc_hbm_walk_result r{};
  if (walk_(device, fraction, chunk_bytes, budget_ms, seed, &r) != 0) {
    throw std::runtime_error(std::string("hbm walk: ") + last_error_());
  }
  char addr[32], flips[32];
  std::snprintf(addr, sizeof(addr), "0x%llx", static_cast<unsigned long long>(r.first_bad_addr));
  std::snprintf(flips, sizeof(flips), "0x%016llx", static_cast<unsigned long long>(r.first_bad_xor));
  const double cov = r.free_bytes ? static_cast<double>(r.bytes_covered) / static_cast<double>(r.free_bytes) : 0.0;
  return json::Value::object({{"device", device},
                              {"free_bytes", static_cast<unsigned long long>(r.free_bytes)},
                              {"total_bytes", static_cast<unsigned long long>(r.total_bytes)},
                              {"target_bytes", static_cast<unsigned long long>(r.target_bytes)},
                              {"bytes_covered", static_cast<unsigned long long>(r.bytes_covered)},
                              {"coverage_of_free", cov},
                              {"chunks", r.chunks},
                              {"passes", r.passes},
                              {"mismatches", static_cast<unsigned long long>(r.mismatches)},
                              {"first_bad_addr", r.mismatches ? json::Value(std::string(addr)) : json::Value()},
                              {"first_bad_bits", r.mismatches ? json::Value(std::string(flips)) : json::Value()},
                              {"write_gbps", r.write_gbps},
                              {"read_gbps", r.read_gbps},
                              {"alloc_ms", r.alloc_ms},
                              {"elapsed_ms", r.elapsed_ms},
                              {"budget_hit", r.budget_hit != 0},
                              {"passed", r.mismatches == 0 && r.passes == 2}});
}

std::string Diag::device_bdf(int device) {
  char buf[64] = {0};
  if (bdf_(device, buf, sizeof(buf)) != 0) throw std::runtime_error(std::string("device bdf: ") + last_error_());
  return buf;
}

namespace {

uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// bf16 bit pattern of a pseudo-random value in [-1, 1] (round-to-nearest-even), and the
// exact float it encodes.
uint16_t rand_bf16(uint32_t seed, uint32_t i, float* exact) {
  float f = static_cast<float>(mix(seed ^ mix(i * 0x9e3779b9U))) / 4294967295.0f * 2.0f - 1.0f;
  uint32_t bits;
  std::memcpy(&bits, &f, 4);
  bits += 0x7fff + ((bits >> 16) & 1);
  uint16_t h = static_cast<uint16_t>(bits >> 16);
  uint32_t back = static_cast<uint32_t>(h) << 16;
  std::memcpy(exact, &back, 4);
  return h;
}

}  // namespace

json::Value Diag::gemm_check(int device, int m, int n, int k, uint32_t seed) {
  std::vector<uint16_t> a(static_cast<size_t>(m) * k), b(static_cast<size_t>(k) * n);
  std::vector<float> af(a.size()), bf(b.size()), c(static_cast<size_t>(m) * n);
  for (size_t i = 0; i < a.size(); ++i) a[i] = rand_bf16(seed, static_cast<uint32_t>(i), &af[i]);
  for (size_t i = 0; i < b.size(); ++i) b[i] = rand_bf16(seed ^ 0xB0B0B0B0U, static_cast<uint32_t>(i), &bf[i]);
  gemm(device, m, n, k, a.data(), b.data(), c.data());
  // fp32 MFMA accumulation of exact bf16 products: |err| <= K * 2^-24 * sum|a||b| (plus
  // slack); measured against a double-precision host product.
  double max_err = 0, max_ratio = 0;
  uint64_t bad = 0;
  for (int i = 0; i < m; ++i) {
    for (int j = 0; j < n; ++j) {
      double ref = 0, mag = 0;
      for (int kk = 0; kk < k; ++kk) {
        const double p = static_cast<double>(af[static_cast<size_t>(i) * k + kk]) * bf[static_cast<size_t>(kk) * n + j];
        ref += p;
        mag += std::fabs(p);
      }
      const double err = std::fabs(static_cast<double>(c[static_cast<size_t>(i) * n + j]) - ref);
      const double bound = 4.0 * k * 5.96e-8 * mag + 1e-6;
      max_err = std::max(max_err, err);
      max_ratio = std::max(max_ratio, err / bound);
      if (err > bound || !std::isfinite(c[static_cast<size_t>(i) * n + j])) ++bad;
    }
  }
  return json::Value::object({{"m", m}, {"n", n}, {"k", k}, {"max_abs_err", max_err},
                              {"max_err_over_bound", max_ratio}, {"bad_elements", static_cast<unsigned long long>(bad)},
                              {"passed", bad == 0}});
}

int burn_dtype_code(const std::string& name) {
  if (name == "bf16") return BGC_BURN_BF16;
  if (name == "fp8") return BGC_BURN_FP8;
  if (name == "fp4") return BGC_BURN_FP4;
  throw std::runtime_error("burn dtype must be bf16, fp8 or fp4, not '" + name + "'");
}

const char* burn_dtype_name(int code) {
  return code == BGC_BURN_FP8 ? "fp8" : code == BGC_BURN_FP4 ? "fp4" : "bf16";
}

double burn_dtype_rate_ratio(int code) {
  // sustained on MI355X: bf16 2.40, MX fp8 4.79, MX fp4 8.47 PF/s (profiles/mx_lowp_r3/)
  return code == BGC_BURN_FP8 ? 2.0 : code == BGC_BURN_FP4 ? 3.5 : 1.0;
}

DiagFloors DiagFloors::mi355x_defaults() {
  DiagFloors f;
  // MI355X, ROCm 7.2, 1 GiB buffers / 16 waves per CU x 2048 MFMA iterations
  // (profiles/archive/diag_floors_r2.json): read 6.33-6.57 TB/s, copy 5.36-5.42, write 5.11-5.25,
  // MFMA bf16 1.92-2.06 PF/s, XCC balance 0.96.  At 256 MiB (Infinity-Cache-sized, the
  // smallest sensible buffer) read is still 5.56 TB/s, so these floors hold down to it.
  f.min_read_gbps = 4750;
  f.min_copy_gbps = 4000;
  f.min_write_gbps = 3800;
  f.min_mfma_tflops = 1500;
  f.min_xcc_balance = 0.85;
  f.min_xccs = 8;
  // MX fp8 / fp4 (v_mfma_scale_f32_16x16x128_f8f6f4, 32 waves per CU x 4096 iterations,
  // profiles/mx_lowp_r3/): 4.1-4.7 PF/s fp8 and 7.3-8.1 PF/s fp4 depending on how warm
  // the clocks are, against ~5 and ~10 PF/s dense peaks
  f.min_fp8_tflops = 3000;
  f.min_fp4_tflops = 5000;
  // burn-in: measured on MI355X in profiles/archive/diag_burn_r2.json (sustained bf16 MFMA at
  // 97 % of the 2.5 PF/s dense peak once clocks settle)
  f.min_burn_tflops = 1800;  // measured 2409-2421 PF/s mean over 10 s at 1.17-1.22 kW, 2.34-2.39 GHz
  f.min_burn_sustain = 0.80;
  f.max_burn_hotspot_c = 100;
  f.max_burn_thermal_violation_pct = 20;
  // PCIe Gen5 x16 host link (profiles/archive/pcie_r2/probe.json): 57.1 GB/s host-to-device and
  // 56.7 GB/s device-to-host with 64 MiB - 1 GiB pinned copies, 97 GB/s both ways at
  // once; a Gen4-trained or x8 link delivers half of that.
  f.min_pcie_h2d_gbps = 45;
  f.min_pcie_d2h_gbps = 45;
  f.require_full_pcie_width = true;
  f.min_pcie_speed_fraction = 0.5;
  // GEMM soak (8-phase ping-pong bf16 MFMA, 256x256 tiles): 1463-1587 TF/s at 8192^3
  // and 1348-1444 at 4096^3 on MI355X (profiles/gemm_soak_r3/); the floor stays where
  // round 2's double-buffered kernel (1253-1361 TF/s) also passes, for BGC_SOAK_KERNEL=2buf
  f.min_soak_tflops = 950;
  // HBM walk: 0.9 of free VRAM is requested; 0.8 leaves room for allocator granularity
  f.min_hbm_walk_coverage = 0.8;
  // node-level burn: one GPU 15 % behind the node's fastest under the shared load is a
  // cooling or power-delivery outlier (healthy MI355X burns agree within ~1 %,
  // profiles/archive/diag_burn_r2.json); the node power limit is site-specific (0 = off)
  f.min_node_burn_balance = 0.85;
  f.max_node_power_w = 0;
  return f;
}

json::Value judge_diag(const json::Value& result, const DiagFloors& fl) {
  json::Value out = result;
  json::Value failures = json::Value::array();
  auto num = [](const json::Value& v, const char* k) { return v.get(k).is_number() ? v.get(k).as_double() : 0.0; };
  auto floor_check = [&](const json::Value& v, const char* key, double floor, const char* what) {
    if (floor <= 0) return;
    const double got = num(v, key);
    if (got < floor) {
      char buf[160];
      std::snprintf(buf, sizeof(buf), "%s %.0f below floor %.0f", what, got, floor);
      failures.push_back(std::string(buf));
    }
  };
  const json::Value& hbm = result.get("hbm");
  if (hbm.is_object()) {
    if (num(hbm, "mismatches") > 0) failures.push_back("HBM pattern mismatches: " + std::to_string(static_cast<uint64_t>(num(hbm, "mismatches"))));
    floor_check(hbm, "read_gbps", fl.min_read_gbps, "HBM read GB/s");
    floor_check(hbm, "copy_gbps", fl.min_copy_gbps, "HBM copy GB/s");
    floor_check(hbm, "write_gbps", fl.min_write_gbps, "HBM write GB/s");
  }
  const json::Value& hw = result.get("hbm_walk");
  if (hw.is_object()) {
    if (num(hw, "mismatches") > 0) {
      std::string msg = "HBM walk mismatches: " + std::to_string(static_cast<uint64_t>(num(hw, "mismatches")));
      if (hw.get("first_bad_addr").is_string()) {
        msg += " (first at " + hw.get_string("first_bad_addr") + ", bits " + hw.get_string("first_bad_bits") + ")";
      }
      failures.push_back(msg);
    }
    if (fl.min_hbm_walk_coverage > 0 && num(hw, "coverage_of_free") < fl.min_hbm_walk_coverage) {
      char buf[160];
      std::snprintf(buf, sizeof(buf), "HBM walk covered %.2f of free VRAM (floor %.2f)", num(hw, "coverage_of_free"),
                    fl.min_hbm_walk_coverage);
      failures.push_back(std::string(buf));
    }
  }
  const json::Value& mf = result.get("mfma");
  if (mf.is_object()) {
    if (num(mf, "mismatches") > 0) failures.push_back("MFMA tile mismatches on " + std::to_string(static_cast<int>(num(mf, "bad_cus"))) + " CU(s)");
    if (mf.get("throughput_ok").is_bool() && !mf.get("throughput_ok").as_bool()) failures.push_back("MFMA throughput accumulators wrong");
    floor_check(mf, "tflops", fl.min_mfma_tflops, "MFMA bf16 TFLOP/s");
    if (fl.min_xcc_balance > 0 && num(mf, "xcc_balance") < fl.min_xcc_balance) {
      char buf[160];
      std::snprintf(buf, sizeof(buf), "XCC balance %.2f below floor %.2f", num(mf, "xcc_balance"), fl.min_xcc_balance);
      failures.push_back(std::string(buf));
    }
    if (fl.min_xccs > 0 && num(mf, "xccs_seen") < fl.min_xccs) {
      failures.push_back("only " + std::to_string(static_cast<int>(num(mf, "xccs_seen"))) + " XCCs ran MFMA work");
    }
  }
  const json::Value& lp = result.get("lowp");
  if (lp.is_object()) {
    if (num(lp, "mismatches") > 0) {
      char buf[200];
      std::snprintf(buf, sizeof(buf), "MX fp8/fp4 MFMA tile mismatches on %d CU(s): fp8 %.0f, fp8 scaled %.0f, fp4 %.0f, fp4 scaled %.0f",
                    static_cast<int>(num(lp, "bad_cus")), num(lp, "fp8_mismatches"), num(lp, "fp8_scaled_mismatches"),
                    num(lp, "fp4_mismatches"), num(lp, "fp4_scaled_mismatches"));
      failures.push_back(std::string(buf));
    }
    if (lp.get("throughput_ok").is_bool() && !lp.get("throughput_ok").as_bool()) {
      failures.push_back("MX fp8/fp4 MFMA throughput accumulators wrong");
    }
    floor_check(lp, "fp8_tflops", fl.min_fp8_tflops, "MX fp8 MFMA TFLOP/s");
    floor_check(lp, "fp4_tflops", fl.min_fp4_tflops, "MX fp4 MFMA TFLOP/s");
  }
  const json::Value& burn = result.get("burn");
  if (burn.is_object()) {
    if (num(burn, "mismatches") > 0) failures.push_back("burn-in MFMA accumulators wrong");
    // the floor is for bf16; an fp8 / fp4 burn is held to it scaled by that path's rate
    const std::string dt = burn.get("dtype").is_string() ? burn.get_string("dtype") : "bf16";
    const int code = dt == "fp8" ? BGC_BURN_FP8 : dt == "fp4" ? BGC_BURN_FP4 : BGC_BURN_BF16;
    const std::string what = "burn-in MFMA " + (code == BGC_BURN_BF16 ? std::string() : "MX " + dt + " ") + "TFLOP/s";
    floor_check(burn, "tflops_mean", fl.min_burn_tflops * burn_dtype_rate_ratio(code), what.c_str());
    if (fl.min_burn_sustain > 0 && num(burn, "sustain") < fl.min_burn_sustain) {
      char buf[160];
      std::snprintf(buf, sizeof(buf), "MFMA rate sagged to %.2f of its start under sustained load (floor %.2f)",
                    num(burn, "sustain"), fl.min_burn_sustain);
      failures.push_back(std::string(buf));
    }
    if (fl.max_burn_hotspot_c > 0 && num(burn, "max_hotspot_c") > fl.max_burn_hotspot_c) {
      char buf[160];
      std::snprintf(buf, sizeof(buf), "hotspot %.0f C under sustained load (limit %.0f)", num(burn, "max_hotspot_c"),
                    fl.max_burn_hotspot_c);
      failures.push_back(std::string(buf));
    }
    if (fl.max_burn_thermal_violation_pct > 0 &&
        num(burn, "thermal_violation_pct") > fl.max_burn_thermal_violation_pct) {
      char buf[160];
      std::snprintf(buf, sizeof(buf), "thermal throttling %.0f%% of the burn (limit %.0f%%)",
                    num(burn, "thermal_violation_pct"), fl.max_burn_thermal_violation_pct);
      failures.push_back(std::string(buf));
    }
  }
  const json::Value& pc = result.get("pcie");
  if (pc.is_object()) {
    if (num(pc, "mismatches") > 0) failures.push_back("PCIe round-trip mismatches: " + std::to_string(static_cast<uint64_t>(num(pc, "mismatches"))));
    floor_check(pc, "h2d_gbps", fl.min_pcie_h2d_gbps, "PCIe host-to-device GB/s");
    floor_check(pc, "d2h_gbps", fl.min_pcie_d2h_gbps, "PCIe device-to-host GB/s");
    // link state read right after the copies (amdsmi; absent when unknown)
    const double w = num(pc, "link_width"), mw = num(pc, "max_width");
    if (fl.require_full_pcie_width && w > 0 && mw > 0 && w < mw) {
      failures.push_back("PCIe link x" + std::to_string(static_cast<int>(w)) + " of x" + std::to_string(static_cast<int>(mw)));
    }
    const double sp = num(pc, "link_speed_mts"), msp = num(pc, "max_speed_mts");
    if (fl.min_pcie_speed_fraction > 0 && sp > 0 && msp > 0 && sp < fl.min_pcie_speed_fraction * msp) {
      char buf[160];
      std::snprintf(buf, sizeof(buf), "PCIe link at %.0f of %.0f MT/s under load", sp, msp);
      failures.push_back(std::string(buf));
    }
  }
  const json::Value& sk = result.get("soak");
  if (sk.is_object()) {
    const double bad = num(sk, "row_mismatches") + num(sk, "col_mismatches");
    if (bad > 0) {
      failures.push_back("GEMM soak checksums wrong: " + std::to_string(static_cast<uint64_t>(num(sk, "row_mismatches"))) +
                         " rows, " + std::to_string(static_cast<uint64_t>(num(sk, "col_mismatches"))) + " columns");
    }
    floor_check(sk, "tflops_mean", fl.min_soak_tflops, "GEMM soak TFLOP/s");
  }
  const json::Value& gm = result.get("gemm");
  if (gm.is_object() && gm.get("passed").is_bool() && !gm.get("passed").as_bool()) {
    failures.push_back("MFMA GEMM differs from the host fp32 product");
  }
  if (result.get("error").is_string()) failures.push_back(result.get_string("error"));
  // a section that failed to run (a HIP fault, a worker that timed out) carries the cause
  // as {"error": ...}: that is a failure in its own right, whatever the floors say
  static const char* const kSections[] = {"hbm", "hbm_walk", "mfma", "lowp", "burn", "pcie", "soak", "gemm"};
  for (const char* sect : kSections) {
    const json::Value& v = result.get(sect);
    if (v.is_object() && v.get("error").is_string()) failures.push_back(std::string(sect) + ": " + v.get_string("error"));
  }
  out["failures"] = failures;
  out["passed"] = failures.items().empty();
  return out;
}

}  // namespace bgc::gpu

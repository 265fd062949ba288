#include "gpu/diag.h"

#include <dlfcn.h>
#include <unistd.h>

#include <cstdlib>
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
  arch_ = reinterpret_cast<int (*)(int, char*, size_t)>(dlsym(lib_, "bgc_diag_device_arch"));
  last_error_ = reinterpret_cast<const char* (*)()>(dlsym(lib_, "bgc_diag_last_error"));
  auto abi = reinterpret_cast<int (*)()>(dlsym(lib_, "bgc_diag_abi_version"));
  if (!device_count_ || !hbm_ || !mfma_ || !arch_ || !last_error_ || !abi || abi() != BGC_DIAG_ABI_VERSION) {
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
  v["elapsed_ms"] = r.elapsed_ms;
  v["passed"] = r.mismatches == 0 && r.throughput_ok != 0;
  return v;
}

}  // namespace bgc::gpu

#include "gpu/device.h"

#include <amd_smi/amdsmi.h>
#include <dlfcn.h>
#include <sys/stat.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>

#include "core/log.h"
#include "core/metrics.h"
#include "core/net.h"

namespace bgc::gpu {

using json::Value;

// ---------------------------------------------------------------------------
// JSON conversions

Value to_json(const GpuInfo& g) {
  Value v = Value::object();
  v["index"] = g.index;
  v["uuid"] = g.uuid;
  v["bdf"] = g.bdf;
  v["market_name"] = g.market_name;
  v["vendor_name"] = g.vendor_name;
  v["gfx_target"] = g.gfx_target;
  v["serial"] = g.serial;
  v["vram_total_mb"] = static_cast<unsigned long long>(g.vram_total_mb);
  v["vram_max_bandwidth_gbps"] = static_cast<unsigned long long>(g.vram_max_bandwidth_gbps);
  v["num_cus"] = g.num_cus;
  char hive[32];
  std::snprintf(hive, sizeof(hive), "%016llx", static_cast<unsigned long long>(g.xgmi_hive_id));
  v["xgmi_hive_id"] = std::string(hive);
  v["xgmi_node_id"] = static_cast<unsigned long long>(g.xgmi_node_id);
  v["xgmi_lanes"] = g.xgmi_lanes;
  v["numa_node"] = g.numa_node;
  v["compute_partition"] = g.compute_partition;
  v["memory_partition"] = g.memory_partition;
  v["power_cap_w"] = g.power_cap_w;
  v["hip_id"] = g.hip_id;
  return v;
}

Value to_json(const Telemetry& t) {
  Value v = Value::object();
  v["index"] = t.index;
  v["ok"] = t.ok;
  if (!t.error.empty()) v["error"] = t.error;
  v["gfx_activity_pct"] = t.gfx_activity_pct;
  v["umc_activity_pct"] = t.umc_activity_pct;
  v["power_w"] = t.power_w;
  v["temp_edge_c"] = t.temp_edge_c;
  v["temp_hotspot_c"] = t.temp_hotspot_c;
  v["temp_mem_c"] = t.temp_mem_c;
  v["vram_used_mb"] = static_cast<unsigned long long>(t.vram_used_mb);
  v["vram_total_mb"] = static_cast<unsigned long long>(t.vram_total_mb);
  v["gfxclk_mhz"] = t.gfxclk_mhz;
  v["uclk_mhz"] = t.uclk_mhz;
  v["throttle_status"] = static_cast<unsigned long long>(t.throttle_status);
  v["ecc_correctable"] = static_cast<unsigned long long>(t.ecc_correctable);
  v["ecc_uncorrectable"] = static_cast<unsigned long long>(t.ecc_uncorrectable);
  v["xgmi_links_up"] = t.xgmi_links_up;
  v["xgmi_links_total"] = t.xgmi_links_total;
  v["poll_us"] = t.poll_us;
  return v;
}

static uint64_t parse_hive(const Value& v) {
  if (v.is_string()) return std::stoull(v.as_string(), nullptr, 16);
  if (v.is_int()) return v.as_uint();
  return 0;
}

GpuInfo gpu_info_from_json(const Value& v) {
  GpuInfo g;
  g.index = v.get("index").is_int() ? static_cast<int>(v.get("index").as_int()) : 0;
  g.uuid = v.get_string("uuid");
  g.bdf = v.get_string("bdf");
  g.market_name = v.get_string("market_name", "AMD Instinct MI355X");
  g.vendor_name = v.get_string("vendor_name", "Advanced Micro Devices Inc. [AMD/ATI]");
  g.gfx_target = v.get_string("gfx_target", "gfx950");
  g.serial = v.get_string("serial");
  if (v.get("vram_total_mb").is_int()) g.vram_total_mb = v.get("vram_total_mb").as_uint();
  if (v.get("vram_max_bandwidth_gbps").is_int()) g.vram_max_bandwidth_gbps = v.get("vram_max_bandwidth_gbps").as_uint();
  if (v.get("num_cus").is_int()) g.num_cus = static_cast<uint32_t>(v.get("num_cus").as_int());
  g.xgmi_hive_id = parse_hive(v.get("xgmi_hive_id"));
  if (v.get("xgmi_node_id").is_int()) g.xgmi_node_id = v.get("xgmi_node_id").as_uint();
  if (v.get("xgmi_lanes").is_int()) g.xgmi_lanes = static_cast<uint32_t>(v.get("xgmi_lanes").as_int());
  if (v.get("numa_node").is_int()) g.numa_node = static_cast<int>(v.get("numa_node").as_int());
  g.compute_partition = v.get_string("compute_partition", "SPX");
  g.memory_partition = v.get_string("memory_partition", "NPS1");
  if (v.get("power_cap_w").is_int()) g.power_cap_w = static_cast<uint32_t>(v.get("power_cap_w").as_int());
  g.hip_id = v.get("hip_id").is_int() ? static_cast<int>(v.get("hip_id").as_int()) : g.index;
  return g;
}

Value default_mi355x_fixture(int n_gpus, uint64_t hive_id) {
  Value gpus = Value::array();
  char hive[32];
  std::snprintf(hive, sizeof(hive), "%016llx", static_cast<unsigned long long>(hive_id));
  for (int i = 0; i < n_gpus; ++i) {
    Value g = Value::object();
    char buf[64];
    g["index"] = i;
    std::snprintf(buf, sizeof(buf), "%08x-0000-1000-80a5-%012x", 0x75a10000 + i, 0x355 + i);
    g["uuid"] = std::string(buf);
    std::snprintf(buf, sizeof(buf), "0000:%02x:00.0", 0x05 + 0x10 * i);
    g["bdf"] = std::string(buf);
    g["market_name"] = "AMD Instinct MI355X";
    g["gfx_target"] = "gfx950";
    g["vram_total_mb"] = 294912;  // 288 GiB HBM3E
    g["vram_max_bandwidth_gbps"] = 8000;
    g["num_cus"] = 256;
    g["xgmi_hive_id"] = std::string(hive);
    g["xgmi_node_id"] = i;
    g["xgmi_lanes"] = 16;
    g["numa_node"] = i < n_gpus / 2 ? 0 : 1;
    g["compute_partition"] = "SPX";
    g["memory_partition"] = "NPS1";
    g["power_cap_w"] = 1400;
    Value t = Value::object();
    t["gfx_activity_pct"] = 0;
    t["umc_activity_pct"] = 0;
    t["power_w"] = 180.0 + i;
    t["temp_edge_c"] = 38.0;
    t["temp_hotspot_c"] = 45.0;
    t["temp_mem_c"] = 40.0;
    t["vram_used_mb"] = 300;
    t["gfxclk_mhz"] = 2400;
    t["uclk_mhz"] = 1900;
    t["xgmi_links_up"] = n_gpus - 1;
    t["xgmi_links_total"] = n_gpus - 1;
    g["telemetry"] = t;
    gpus.push_back(g);
  }
  Value f = Value::object();
  f["gpus"] = gpus;
  return f;
}

// ---------------------------------------------------------------------------
// Mock backend

namespace {

class MockBackend : public Backend {
 public:
  explicit MockBackend(const Value& fixture) : fixture_(fixture) {}
  // File-backed: the fixture is re-read when its mtime changes, so tests can flip a
  // device's telemetry (GPU flap / drain scenarios) while the agent runs.
  explicit MockBackend(std::string path) : path_(std::move(path)) { reload(); }
  void reload() {
    if (path_.empty()) return;
    std::lock_guard<std::mutex> rl(reload_mu_);  // per-GPU samplers call this concurrently
    struct stat st {};
    if (::stat(path_.c_str(), &st) != 0) return;
    if (st.st_mtim.tv_sec == mtime_.tv_sec && st.st_mtim.tv_nsec == mtime_.tv_nsec) return;
    try {
      Value v = json::parse(net::read_file(path_));
      std::lock_guard<std::mutex> lk(mu_);
      fixture_ = std::move(v);
      mtime_ = st.st_mtim;
    } catch (const std::exception& e) {
      LOG_WARN("gpu") << "mock fixture reload failed: " << e.what();
    }
  }
  std::string name() const override { return "mock"; }
  std::vector<GpuInfo> discover() override {
    reload();
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<GpuInfo> out;
    int i = 0;
    for (const auto& g : fixture_.get("gpus").items()) {
      GpuInfo info = gpu_info_from_json(g);
      if (!g.get("index").is_int()) info.index = i;
      out.push_back(info);
      ++i;
    }
    return out;
  }
  Telemetry sample(int index, bool full) override {
    (void)full;
    reload();
    std::lock_guard<std::mutex> lk(mu_);
    int64_t t0 = metrics::now_ns();
    Telemetry t;
    t.index = index;
    t.ts_ns = t0;
    const auto& gpus = fixture_.get("gpus").items();
    if (index < 0 || static_cast<size_t>(index) >= gpus.size()) {
      t.error = "no such device";
      return t;
    }
    const Value& g = gpus[static_cast<size_t>(index)];
    const Value& tv = g.get("telemetry");
    if (tv.get("error").is_string()) {
      t.error = tv.get_string("error");
      return t;
    }
    auto num = [&](const char* k, double d) { return tv.get(k).is_number() ? tv.get(k).as_double() : d; };
    t.ok = true;
    t.gfx_activity_pct = num("gfx_activity_pct", 0);
    t.umc_activity_pct = num("umc_activity_pct", 0);
    t.power_w = num("power_w", 0);
    t.temp_edge_c = num("temp_edge_c", 0);
    t.temp_hotspot_c = num("temp_hotspot_c", 0);
    t.temp_mem_c = num("temp_mem_c", 0);
    t.vram_used_mb = static_cast<uint64_t>(num("vram_used_mb", 0));
    t.vram_total_mb = g.get("vram_total_mb").is_int() ? g.get("vram_total_mb").as_uint() : 0;
    t.gfxclk_mhz = static_cast<uint32_t>(num("gfxclk_mhz", 0));
    t.uclk_mhz = static_cast<uint32_t>(num("uclk_mhz", 0));
    t.throttle_status = static_cast<uint64_t>(num("throttle_status", 0));
    t.ecc_correctable = static_cast<uint64_t>(num("ecc_correctable", 0));
    t.ecc_uncorrectable = static_cast<uint64_t>(num("ecc_uncorrectable", 0));
    t.xgmi_links_up = static_cast<int>(num("xgmi_links_up", -1));
    t.xgmi_links_total = static_cast<int>(num("xgmi_links_total", -1));
    t.poll_us = static_cast<double>(metrics::now_ns() - t0) / 1e3;
    return t;
  }

 private:
  Value fixture_;
  std::string path_;
  struct timespec mtime_ {};
  std::mutex reload_mu_;  // guards mtime_ and serializes file reads
  std::mutex mu_;         // guards fixture_
};

// ---------------------------------------------------------------------------
// amdsmi backend (dlopen)

struct AmdSmiApi {
  void* lib = nullptr;
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_shut_down) shut_down = nullptr;
  decltype(&amdsmi_get_socket_handles) get_socket_handles = nullptr;
  decltype(&amdsmi_get_processor_handles) get_processor_handles = nullptr;
  decltype(&amdsmi_get_gpu_device_uuid) get_uuid = nullptr;
  decltype(&amdsmi_get_gpu_device_bdf) get_bdf = nullptr;
  decltype(&amdsmi_get_gpu_asic_info) get_asic = nullptr;
  decltype(&amdsmi_get_gpu_vram_info) get_vram_info = nullptr;
  decltype(&amdsmi_get_xgmi_info) get_xgmi = nullptr;
  decltype(&amdsmi_topo_get_numa_node_number) get_numa = nullptr;
  decltype(&amdsmi_get_gpu_compute_partition) get_compute_partition = nullptr;
  decltype(&amdsmi_get_gpu_memory_partition) get_memory_partition = nullptr;
  decltype(&amdsmi_get_gpu_metrics_info) get_metrics = nullptr;
  decltype(&amdsmi_get_gpu_vram_usage) get_vram_usage = nullptr;
  decltype(&amdsmi_get_gpu_total_ecc_count) get_ecc = nullptr;
  decltype(&amdsmi_get_power_info) get_power = nullptr;
  decltype(&amdsmi_get_gpu_enumeration_info) get_enum = nullptr;
};

template <typename F>
void resolve(void* lib, F& fn, const char* sym, bool required) {
  fn = reinterpret_cast<F>(dlsym(lib, sym));
  if (!fn && required) throw std::runtime_error(std::string("libamd_smi missing symbol ") + sym);
}

class AmdSmiBackend : public Backend {
 public:
  AmdSmiBackend() {
    const char* candidates[] = {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"};
    for (const char* c : candidates) {
      api_.lib = dlopen(c, RTLD_NOW | RTLD_LOCAL);
      if (api_.lib) break;
    }
    if (!api_.lib) throw std::runtime_error(std::string("cannot load libamd_smi: ") + dlerror());
    resolve(api_.lib, api_.init, "amdsmi_init", true);
    resolve(api_.lib, api_.shut_down, "amdsmi_shut_down", true);
    resolve(api_.lib, api_.get_socket_handles, "amdsmi_get_socket_handles", true);
    resolve(api_.lib, api_.get_processor_handles, "amdsmi_get_processor_handles", true);
    resolve(api_.lib, api_.get_uuid, "amdsmi_get_gpu_device_uuid", false);
    resolve(api_.lib, api_.get_bdf, "amdsmi_get_gpu_device_bdf", false);
    resolve(api_.lib, api_.get_asic, "amdsmi_get_gpu_asic_info", false);
    resolve(api_.lib, api_.get_vram_info, "amdsmi_get_gpu_vram_info", false);
    resolve(api_.lib, api_.get_xgmi, "amdsmi_get_xgmi_info", false);
    resolve(api_.lib, api_.get_numa, "amdsmi_topo_get_numa_node_number", false);
    resolve(api_.lib, api_.get_compute_partition, "amdsmi_get_gpu_compute_partition", false);
    resolve(api_.lib, api_.get_memory_partition, "amdsmi_get_gpu_memory_partition", false);
    resolve(api_.lib, api_.get_metrics, "amdsmi_get_gpu_metrics_info", false);
    resolve(api_.lib, api_.get_vram_usage, "amdsmi_get_gpu_vram_usage", false);
    resolve(api_.lib, api_.get_ecc, "amdsmi_get_gpu_total_ecc_count", false);
    resolve(api_.lib, api_.get_power, "amdsmi_get_power_info", false);
    resolve(api_.lib, api_.get_enum, "amdsmi_get_gpu_enumeration_info", false);
    amdsmi_status_t st = api_.init(AMDSMI_INIT_AMD_GPUS);
    if (st != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("amdsmi_init failed: status " + std::to_string(st));
    initialized_ = true;
    uint32_t nsock = 0;
    if (api_.get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) throw std::runtime_error("amdsmi_get_socket_handles failed");
    std::vector<amdsmi_socket_handle> socks(nsock);
    api_.get_socket_handles(&nsock, socks.data());
    for (auto s : socks) {
      uint32_t n = 0;
      if (api_.get_processor_handles(s, &n, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> ps(n);
      api_.get_processor_handles(s, &n, ps.data());
      for (auto p : ps) handles_.push_back(p);
    }
  }
  ~AmdSmiBackend() override {
    if (initialized_) api_.shut_down();
    // keep the library mapped: amdsmi spawns helper state that outlives shut_down
  }
  std::string name() const override { return "amdsmi"; }

  std::vector<GpuInfo> discover() override {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<GpuInfo> out;
    for (size_t i = 0; i < handles_.size(); ++i) {
      auto h = handles_[i];
      GpuInfo g;
      g.index = static_cast<int>(i);
      g.hip_id = static_cast<int>(i);
      if (api_.get_uuid) {
        char buf[AMDSMI_GPU_UUID_SIZE] = {0};
        unsigned len = sizeof(buf);
        if (api_.get_uuid(h, &len, buf) == AMDSMI_STATUS_SUCCESS) g.uuid = buf;
      }
      if (api_.get_bdf) {
        amdsmi_bdf_t bdf{};
        if (api_.get_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
          char buf[32];
          std::snprintf(buf, sizeof(buf), "%04llx:%02x:%02x.%x", static_cast<unsigned long long>(bdf.domain_number),
                        static_cast<unsigned>(bdf.bus_number), static_cast<unsigned>(bdf.device_number),
                        static_cast<unsigned>(bdf.function_number));
          g.bdf = buf;
        }
      }
      if (api_.get_asic) {
        amdsmi_asic_info_t a{};
        if (api_.get_asic(h, &a) == AMDSMI_STATUS_SUCCESS) {
          g.market_name = a.market_name;
          g.vendor_name = a.vendor_name;
          g.serial = a.asic_serial;
          if (a.num_of_compute_units != 0xFFFFFFFFu) g.num_cus = a.num_of_compute_units;
          if (a.target_graphics_version != 0xFFFFFFFFFFFFFFFFULL) {
            char buf[32];
            std::snprintf(buf, sizeof(buf), "gfx%llx", static_cast<unsigned long long>(a.target_graphics_version));
            g.gfx_target = buf;
          }
        }
      }
      if (api_.get_vram_info) {
        amdsmi_vram_info_t v{};
        if (api_.get_vram_info(h, &v) == AMDSMI_STATUS_SUCCESS) {
          g.vram_total_mb = v.vram_size;
          g.vram_max_bandwidth_gbps = v.vram_max_bandwidth;
        }
      }
      if (api_.get_xgmi) {
        amdsmi_xgmi_info_t x{};
        if (api_.get_xgmi(h, &x) == AMDSMI_STATUS_SUCCESS) {
          g.xgmi_hive_id = x.xgmi_hive_id;
          g.xgmi_node_id = x.xgmi_node_id;
          g.xgmi_lanes = x.xgmi_lanes;
        }
      }
      if (api_.get_numa) {
        uint32_t numa = 0;
        if (api_.get_numa(h, &numa) == AMDSMI_STATUS_SUCCESS) g.numa_node = static_cast<int>(numa);
      }
      if (api_.get_compute_partition) {
        char buf[64] = {0};
        if (api_.get_compute_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS) g.compute_partition = buf;
      }
      if (api_.get_memory_partition) {
        char buf[64] = {0};
        if (api_.get_memory_partition(h, buf, sizeof(buf)) == AMDSMI_STATUS_SUCCESS) g.memory_partition = buf;
      }
      if (api_.get_power) {
        amdsmi_power_info_t p{};
        if (api_.get_power(h, &p) == AMDSMI_STATUS_SUCCESS) {
          // ROCm 7.2 reports the limit in microwatts on MI3xx/MI355X despite the header.
          uint64_t lim = p.power_limit;
          g.power_cap_w = static_cast<uint32_t>(lim > 100000 ? lim / 1000000 : lim);
        }
      }
      if (api_.get_enum) {
        amdsmi_enumeration_info_t e{};
        if (api_.get_enum(h, &e) == AMDSMI_STATUS_SUCCESS) g.hip_id = static_cast<int>(e.hip_id);
      }
      out.push_back(g);
    }
    return out;
  }

  Telemetry sample(int index, bool full) override {
    Telemetry t;
    t.index = index;
    int64_t t0 = metrics::now_ns();
    t.ts_ns = t0;
    if (index < 0 || static_cast<size_t>(index) >= handles_.size()) {
      t.error = "no such device";
      return t;
    }
    auto h = handles_[static_cast<size_t>(index)];
    if (!api_.get_metrics) {
      t.error = "amdsmi_get_gpu_metrics_info unavailable";
      return t;
    }
    amdsmi_gpu_metrics_t m;
    std::memset(&m, 0, sizeof(m));
    amdsmi_status_t st = api_.get_metrics(h, &m);
    if (st != AMDSMI_STATUS_SUCCESS) {
      t.error = "amdsmi_get_gpu_metrics_info status " + std::to_string(st);
      t.poll_us = static_cast<double>(metrics::now_ns() - t0) / 1e3;
      return t;
    }
    auto valid16 = [](uint16_t v) { return v != 0xFFFF; };
    t.ok = true;
    if (valid16(m.average_gfx_activity)) t.gfx_activity_pct = m.average_gfx_activity;
    if (valid16(m.average_umc_activity)) t.umc_activity_pct = m.average_umc_activity;
    if (valid16(m.current_socket_power)) t.power_w = m.current_socket_power;
    else if (valid16(m.average_socket_power)) t.power_w = m.average_socket_power;
    if (valid16(m.temperature_edge)) t.temp_edge_c = m.temperature_edge;
    if (valid16(m.temperature_hotspot)) t.temp_hotspot_c = m.temperature_hotspot;
    if (valid16(m.temperature_mem)) t.temp_mem_c = m.temperature_mem;
    if (valid16(m.current_gfxclk)) t.gfxclk_mhz = m.current_gfxclk;
    else if (valid16(m.current_gfxclks[0])) t.gfxclk_mhz = m.current_gfxclks[0];
    if (valid16(m.current_uclk)) t.uclk_mhz = m.current_uclk;
    t.throttle_status = m.indep_throttle_status != 0xFFFFFFFFFFFFFFFFULL ? m.indep_throttle_status : m.throttle_status;
    int up = 0, total = 0;
    for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
      uint16_t s = m.xgmi_link_status[l];
      if (s == 0xFFFF) continue;
      ++total;
      if (s) ++up;
    }
    if (total) {
      t.xgmi_links_up = up;
      t.xgmi_links_total = total;
    }
    if (full && api_.get_vram_usage) {
      amdsmi_vram_usage_t u{};
      if (api_.get_vram_usage(h, &u) == AMDSMI_STATUS_SUCCESS) {
        t.vram_used_mb = u.vram_used;
        t.vram_total_mb = u.vram_total;
      }
    }
    if (full && api_.get_ecc) {
      amdsmi_error_count_t e{};
      if (api_.get_ecc(h, &e) == AMDSMI_STATUS_SUCCESS) {
        t.ecc_correctable = e.correctable_count;
        t.ecc_uncorrectable = e.uncorrectable_count;
      }
    }
    t.poll_us = static_cast<double>(metrics::now_ns() - t0) / 1e3;
    return t;
  }

 private:
  AmdSmiApi api_;
  bool initialized_ = false;
  std::vector<amdsmi_processor_handle> handles_;
  std::mutex mu_;
};

}  // namespace

std::unique_ptr<Backend> make_amdsmi_backend() { return std::make_unique<AmdSmiBackend>(); }

std::unique_ptr<Backend> make_mock_backend(const Value& fixture) { return std::make_unique<MockBackend>(fixture); }

std::unique_ptr<Backend> make_backend(const std::string& kind, const std::string& mock_fixture_path) {
  auto load_mock = [&]() -> std::unique_ptr<Backend> {
    if (mock_fixture_path.empty()) return make_mock_backend(default_mi355x_fixture());
    return std::make_unique<MockBackend>(mock_fixture_path);
  };
  if (kind == "mock") return load_mock();
  if (kind == "amdsmi") return make_amdsmi_backend();
  try {
    auto b = make_amdsmi_backend();
    if (!b->discover().empty()) return b;
    LOG_WARN("gpu") << "amdsmi found no GPUs";
  } catch (const std::exception& e) {
    LOG_WARN("gpu") << "amdsmi unavailable (" << e.what() << ")";
  }
  if (!mock_fixture_path.empty()) return load_mock();
  throw std::runtime_error("no GPU backend available (amdsmi failed and no mock fixture configured)");
}

}  // namespace bgc::gpu

#include "gpu/device.h"

#include <amd_smi/amdsmi.h>
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <algorithm>
#include <cstring>
#include <chrono>
#include <map>
#include <mutex>
#include <thread>
#include <stdexcept>

#include "core/log.h"
#include "core/metrics.h"
#include "core/roctx.h"
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
  v["drm_render"] = g.drm_render;
  v["drm_card"] = g.drm_card;
  v["bad_page_threshold"] = g.bad_page_threshold;
  v["pcie_max_width"] = g.pcie_max_width;
  v["pcie_max_speed_mts"] = g.pcie_max_speed_mts;
  v["pcie_max_gen"] = g.pcie_max_gen;
  v["driver_name"] = g.driver_name;
  v["driver_version"] = g.driver_version;
  v["vbios_version"] = g.vbios_version;
  v["vbios_part_number"] = g.vbios_part_number;
  Value links = Value::array();
  for (const auto& l : g.links) links.push_back(to_json(l));
  v["links"] = links;
  Value phys = Value::array();
  for (const auto& l : g.phys_links) phys.push_back(to_json(l));
  v["phys_links"] = phys;
  return v;
}

Value to_json(const PeerLink& l) {
  return Value::object({{"peer", l.peer}, {"type", l.type}, {"hops", static_cast<unsigned long long>(l.hops)},
                        {"weight", static_cast<unsigned long long>(l.weight)},
                        {"min_bw_mbps", static_cast<unsigned long long>(l.min_bw_mbps)},
                        {"max_bw_mbps", static_cast<unsigned long long>(l.max_bw_mbps)}});
}

Value to_json(const PhysLink& l) {
  return Value::object({{"peer_bdf", l.peer_bdf}, {"type", l.type}, {"bit_rate_gbps", l.bit_rate_gbps},
                        {"max_bandwidth_gbps", l.max_bandwidth_gbps},
                        {"read_kb", static_cast<unsigned long long>(l.read_kb)},
                        {"write_kb", static_cast<unsigned long long>(l.write_kb)}});
}

static uint64_t u64_or(const Value& v, const char* k, uint64_t d) { return v.get(k).is_int() ? v.get(k).as_uint() : d; }

PeerLink peer_link_from_json(const Value& v) {
  PeerLink l;
  l.peer = v.get("peer").is_int() ? static_cast<int>(v.get("peer").as_int()) : -1;
  l.type = v.get_string("type", "unknown");
  l.hops = u64_or(v, "hops", 0);
  l.weight = u64_or(v, "weight", 0);
  l.min_bw_mbps = u64_or(v, "min_bw_mbps", 0);
  l.max_bw_mbps = u64_or(v, "max_bw_mbps", 0);
  return l;
}

PhysLink phys_link_from_json(const Value& v) {
  PhysLink l;
  l.peer_bdf = v.get_string("peer_bdf");
  l.type = v.get_string("type", "xgmi");
  l.bit_rate_gbps = static_cast<uint32_t>(u64_or(v, "bit_rate_gbps", 0));
  l.max_bandwidth_gbps = static_cast<uint32_t>(u64_or(v, "max_bandwidth_gbps", 0));
  l.read_kb = u64_or(v, "read_kb", 0);
  l.write_kb = u64_or(v, "write_kb", 0);
  return l;
}

const char* link_type_name(int t) {
  switch (t) {
    case AMDSMI_LINK_TYPE_INTERNAL: return "internal";
    case AMDSMI_LINK_TYPE_PCIE: return "pcie";
    case AMDSMI_LINK_TYPE_XGMI: return "xgmi";
    case AMDSMI_LINK_TYPE_NOT_APPLICABLE: return "n/a";
    default: return "unknown";
  }
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
  v["throttle_status"] = t.throttle_valid ? Value(static_cast<unsigned long long>(t.throttle_status)) : Value();
  v["violation_ppt_pct"] = t.violation_ppt_pct < 0 ? Value() : Value(t.violation_ppt_pct);
  v["violation_thermal_pct"] = t.violation_thermal_pct < 0 ? Value() : Value(t.violation_thermal_pct);
  v["ecc_correctable"] = static_cast<unsigned long long>(t.ecc_correctable);
  v["ecc_uncorrectable"] = static_cast<unsigned long long>(t.ecc_uncorrectable);
  v["ecc_deferred"] = static_cast<unsigned long long>(t.ecc_deferred);
  v["xgmi_links_up"] = t.xgmi_links_up;
  v["xgmi_links_total"] = t.xgmi_links_total;
  if (t.pcie_width >= 0) v["pcie_width"] = t.pcie_width;
  if (t.pcie_speed_mts >= 0) v["pcie_speed_mts"] = t.pcie_speed_mts;
  if (t.pcie_replays >= 0) v["pcie_replays"] = t.pcie_replays;
  if (t.pcie_recoveries >= 0) v["pcie_recoveries"] = t.pcie_recoveries;
  if (t.pcie_nak_sent >= 0) v["pcie_nak_sent"] = t.pcie_nak_sent;
  if (t.pcie_nak_received >= 0) v["pcie_nak_received"] = t.pcie_nak_received;
  if (t.ras_ok) {
    v["retired_pages"] = static_cast<unsigned long long>(t.retired_pages);
    v["unreservable_pages"] = static_cast<unsigned long long>(t.unreservable_pages);
    Value blocks = Value::object();
    for (const auto& b : t.ecc_blocks) {
      blocks[b.block] = Value::object({{"ce", static_cast<unsigned long long>(b.correctable)},
                                       {"ue", static_cast<unsigned long long>(b.uncorrectable)},
                                       {"de", static_cast<unsigned long long>(b.deferred)}});
    }
    v["ecc_blocks"] = blocks;
    Value links = Value::array();
    for (const auto& l : t.links) links.push_back(to_json(l));
    v["links"] = links;
  }
  if (t.acc_counter != Telemetry::kNoAcc) v["acc_counter"] = static_cast<unsigned long long>(t.acc_counter);
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
  g.drm_render = v.get("drm_render").is_int() ? static_cast<int>(v.get("drm_render").as_int()) : -1;
  g.drm_card = v.get("drm_card").is_int() ? static_cast<int>(v.get("drm_card").as_int()) : -1;
  g.bad_page_threshold = static_cast<uint32_t>(u64_or(v, "bad_page_threshold", 0));
  auto int_or = [&](const char* k, int d) { return v.get(k).is_int() ? static_cast<int>(v.get(k).as_int()) : d; };
  g.pcie_max_width = int_or("pcie_max_width", -1);
  g.pcie_max_speed_mts = int_or("pcie_max_speed_mts", -1);
  g.pcie_max_gen = int_or("pcie_max_gen", -1);
  g.driver_name = v.get_string("driver_name");
  g.driver_version = v.get_string("driver_version");
  g.vbios_version = v.get_string("vbios_version");
  g.vbios_part_number = v.get_string("vbios_part_number");
  for (const auto& l : v.get("links").items()) g.links.push_back(peer_link_from_json(l));
  for (const auto& l : v.get("phys_links").items()) g.phys_links.push_back(phys_link_from_json(l));
  return g;
}

Telemetry telemetry_from_json(const Value& v) {
  Telemetry t;
  auto num = [&](const char* k, double d) { return v.get(k).is_number() ? v.get(k).as_double() : d; };
  t.index = static_cast<int>(num("index", 0));
  t.ok = v.get("ok").is_bool() ? v.get("ok").as_bool() : true;
  t.error = v.get_string("error");
  t.temp_hotspot_c = num("temp_hotspot_c", 40);
  t.temp_mem_c = num("temp_mem_c", 40);
  t.ecc_uncorrectable = static_cast<uint64_t>(num("ecc_uncorrectable", 0));
  t.xgmi_links_up = static_cast<int>(num("xgmi_links_up", -1));
  t.xgmi_links_total = static_cast<int>(num("xgmi_links_total", -1));
  t.violation_ppt_pct = num("violation_ppt_pct", -1);
  t.violation_thermal_pct = num("violation_thermal_pct", -1);
  if (v.get("acc_counter").is_number()) {
    t.acc_counter = static_cast<uint64_t>(num("acc_counter", 0));
    t.acc_ppt = v.get("acc_ppt").is_number() ? static_cast<uint64_t>(num("acc_ppt", 0)) : Telemetry::kNoAcc;
    t.acc_thermal = v.get("acc_thermal").is_number() ? static_cast<uint64_t>(num("acc_thermal", 0)) : Telemetry::kNoAcc;
  }
  t.pcie_width = static_cast<int>(num("pcie_width", -1));
  t.pcie_speed_mts = static_cast<int>(num("pcie_speed_mts", -1));
  t.pcie_replays = static_cast<int64_t>(num("pcie_replays", -1));
  t.pcie_recoveries = static_cast<int64_t>(num("pcie_recoveries", -1));
  if (v.get("retired_pages").is_number() || v.get("unreservable_pages").is_number()) {
    t.ras_ok = true;
    t.retired_pages = static_cast<uint64_t>(num("retired_pages", 0));
    t.unreservable_pages = static_cast<uint64_t>(num("unreservable_pages", 0));
  }
  return t;
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
    g["drm_card"] = 1 + i;
    g["drm_render"] = 128 + i;
    g["pcie_max_width"] = 16;
    g["pcie_max_speed_mts"] = 32000;  // Gen5
    g["pcie_max_gen"] = 5;
    g["driver_name"] = "amdgpu";
    g["driver_version"] = "6.16.6";
    g["vbios_version"] = "022.040.003.043.000001";
    g["vbios_part_number"] = "113-M3550101-100";
    // 8x MI355X UBB: a full xGMI mesh, one link to every peer (7 x ~153 GB/s per GPU).
    Value links = Value::array(), phys = Value::array();
    for (int j = 0; j < n_gpus; ++j) {
      if (j == i) continue;
      links.push_back(Value::object({{"peer", j}, {"type", "xgmi"}, {"hops", 1}, {"weight", 15},
                                     {"min_bw_mbps", 50000}, {"max_bw_mbps", 153600}}));
      std::snprintf(buf, sizeof(buf), "0000:%02x:00.0", 0x05 + 0x10 * j);
      phys.push_back(Value::object({{"peer_bdf", std::string(buf)}, {"type", "xgmi"}, {"bit_rate_gbps", 32},
                                    {"max_bandwidth_gbps", 1228}}));
    }
    g["links"] = links;
    g["phys_links"] = phys;
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
    t["pcie_width"] = 16;
    t["pcie_speed_mts"] = 32000;
    t["pcie_replays"] = 0;
    t["pcie_recoveries"] = 0;
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
  Telemetry sample(int index, SampleLevel level) override {
    reload();
    std::unique_lock<std::mutex> lk(mu_);
    // "sample_hang_ms": every reading blocks this long, as amdsmi does while the driver
    // resets a wedged GPU; rewriting the fixture without it ends the hang early.
    // "sample_hang_samples" (optional): only that many readings block, the rest return.
    bool hangs = fixture_.get("sample_hang_ms").is_number();
    if (hangs && fixture_.get("sample_hang_samples").is_int()) {
      hangs = hung_samples_ < fixture_.get("sample_hang_samples").as_int();
      if (hangs) ++hung_samples_;
    }
    for (int64_t hang_start = metrics::now_ns(); hangs;) {
      const Value& hang = fixture_.get("sample_hang_ms");
      if (!hang.is_number() || static_cast<double>(metrics::now_ns() - hang_start) / 1e6 >= hang.as_double()) break;
      lk.unlock();
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
      reload();
      lk.lock();
    }
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
    t.throttle_valid = tv.get("throttle_status").is_number();
    t.throttle_status = static_cast<uint64_t>(num("throttle_status", 0));
    // Violation accumulators: either given directly, or synthesised from a steady
    // "violation_*_pct" so a fixture can model sustained throttling without rewriting
    // the file every poll (the counter advances 1000 per sample).
    if (tv.get("acc_counter").is_number()) {
      t.acc_counter = static_cast<uint64_t>(num("acc_counter", 0));
      t.acc_ppt = static_cast<uint64_t>(num("acc_ppt", 0));
      t.acc_thermal = static_cast<uint64_t>(num("acc_thermal", 0));
    } else {
      uint64_t& seq = acc_seq_[index];
      seq += 1000;
      t.acc_counter = seq;
      t.acc_ppt = static_cast<uint64_t>(static_cast<double>(seq) * num("violation_ppt_pct", 0) / 100.0);
      t.acc_thermal = static_cast<uint64_t>(static_cast<double>(seq) * num("violation_thermal_pct", 0) / 100.0);
    }
    if (level >= SampleLevel::Slow) {
      t.ecc_correctable = static_cast<uint64_t>(num("ecc_correctable", 0));
      t.ecc_uncorrectable = static_cast<uint64_t>(num("ecc_uncorrectable", 0));
      t.ecc_deferred = static_cast<uint64_t>(num("ecc_deferred", 0));
      t.pcie_width = static_cast<int>(num("pcie_width", -1));
      t.pcie_speed_mts = static_cast<int>(num("pcie_speed_mts", -1));
      t.pcie_replays = static_cast<int64_t>(num("pcie_replays", -1));
      t.pcie_recoveries = static_cast<int64_t>(num("pcie_recoveries", -1));
      t.pcie_nak_sent = static_cast<int64_t>(num("pcie_nak_sent", -1));
      t.pcie_nak_received = static_cast<int64_t>(num("pcie_nak_received", -1));
    } else {
      t.vram_used_mb = 0;
    }
    t.xgmi_links_up = static_cast<int>(num("xgmi_links_up", -1));
    t.xgmi_links_total = static_cast<int>(num("xgmi_links_total", -1));
    if (level == SampleLevel::Ras) {
      t.ras_ok = true;
      t.retired_pages = static_cast<uint64_t>(num("retired_pages", 0));
      t.unreservable_pages = static_cast<uint64_t>(num("unreservable_pages", 0));
      for (const auto& b : tv.get("ecc_blocks").items()) {
        EccBlock e;
        e.block = b.get_string("block");
        e.correctable = u64_or(b, "ce", 0);
        e.uncorrectable = u64_or(b, "ue", 0);
        e.deferred = u64_or(b, "de", 0);
        t.ecc_blocks.push_back(std::move(e));
      }
      const Value& links = tv.get("links").is_array() ? tv.get("links") : g.get("phys_links");
      for (const auto& l : links.items()) t.links.push_back(phys_link_from_json(l));
    }
    if (const double d = num("sample_delay_us", 0); d > 0) {  // models amdsmi's per-call cost
      lk.unlock();
      std::this_thread::sleep_for(std::chrono::microseconds(static_cast<int64_t>(d)));
    }
    t.poll_us = static_cast<double>(metrics::now_ns() - t0) / 1e3;
    return t;
  }
  int busy_processes(int index) override {
    reload();
    std::lock_guard<std::mutex> lk(mu_);
    const auto& gpus = fixture_.get("gpus").items();
    if (index < 0 || static_cast<size_t>(index) >= gpus.size()) return -1;
    const Value& b = gpus[static_cast<size_t>(index)].get("telemetry").get("busy_processes");
    return b.is_int() ? static_cast<int>(b.as_int()) : 0;
  }
  Value diag_script() override {
    reload();
    std::lock_guard<std::mutex> lk(mu_);
    return fixture_.get("diag_script");
  }

 private:
  Value fixture_;
  std::string path_;
  struct timespec mtime_ {};
  std::mutex reload_mu_;  // guards mtime_ and serializes file reads
  std::mutex mu_;         // guards fixture_, acc_seq_ and hung_samples_
  std::map<int, uint64_t> acc_seq_;
  int64_t hung_samples_ = 0;
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
  decltype(&amdsmi_topo_get_link_type) topo_link_type = nullptr;
  decltype(&amdsmi_topo_get_link_weight) topo_link_weight = nullptr;
  decltype(&amdsmi_get_minmax_bandwidth_between_processors) minmax_bw = nullptr;
  decltype(&amdsmi_get_link_metrics) link_metrics = nullptr;
  decltype(&amdsmi_get_gpu_bad_page_info) bad_pages = nullptr;
  decltype(&amdsmi_get_gpu_bad_page_threshold) bad_page_threshold = nullptr;
  decltype(&amdsmi_get_gpu_ecc_enabled) ecc_enabled = nullptr;
  decltype(&amdsmi_get_gpu_ecc_count) ecc_count = nullptr;
  decltype(&amdsmi_get_gpu_process_list) process_list = nullptr;
  decltype(&amdsmi_get_pcie_info) pcie_info = nullptr;
  decltype(&amdsmi_get_gpu_driver_info) driver_info = nullptr;
  decltype(&amdsmi_get_gpu_vbios_info) vbios_info = nullptr;
};

struct BlockName {
  amdsmi_gpu_block_t block;
  const char* name;
};
constexpr BlockName kEccBlocks[] = {
    {AMDSMI_GPU_BLOCK_UMC, "umc"},       {AMDSMI_GPU_BLOCK_SDMA, "sdma"},   {AMDSMI_GPU_BLOCK_GFX, "gfx"},
    {AMDSMI_GPU_BLOCK_MMHUB, "mmhub"},   {AMDSMI_GPU_BLOCK_ATHUB, "athub"}, {AMDSMI_GPU_BLOCK_PCIE_BIF, "pcie_bif"},
    {AMDSMI_GPU_BLOCK_HDP, "hdp"},       {AMDSMI_GPU_BLOCK_XGMI_WAFL, "xgmi_wafl"}, {AMDSMI_GPU_BLOCK_DF, "df"},
    {AMDSMI_GPU_BLOCK_SMN, "smn"},       {AMDSMI_GPU_BLOCK_SEM, "sem"},     {AMDSMI_GPU_BLOCK_MP0, "mp0"},
    {AMDSMI_GPU_BLOCK_MP1, "mp1"},       {AMDSMI_GPU_BLOCK_FUSE, "fuse"},   {AMDSMI_GPU_BLOCK_MCA, "mca"},
    {AMDSMI_GPU_BLOCK_VCN, "vcn"},       {AMDSMI_GPU_BLOCK_JPEG, "jpeg"},   {AMDSMI_GPU_BLOCK_IH, "ih"},
    {AMDSMI_GPU_BLOCK_MPIO, "mpio"},
};

std::string bdf_string(const amdsmi_bdf_t& bdf) {
  char buf[32];
  std::snprintf(buf, sizeof(buf), "%04llx:%02x:%02x.%x", static_cast<unsigned long long>(bdf.domain_number),
                static_cast<unsigned>(bdf.bus_number), static_cast<unsigned>(bdf.device_number),
                static_cast<unsigned>(bdf.function_number));
  return buf;
}

// amdsmi string fields are fixed arrays that may lack a terminator when full
std::string cstr(const char* p, size_t cap) { return std::string(p, strnlen(p, cap)); }

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
    resolve(api_.lib, api_.topo_link_type, "amdsmi_topo_get_link_type", false);
    resolve(api_.lib, api_.topo_link_weight, "amdsmi_topo_get_link_weight", false);
    resolve(api_.lib, api_.minmax_bw, "amdsmi_get_minmax_bandwidth_between_processors", false);
    resolve(api_.lib, api_.link_metrics, "amdsmi_get_link_metrics", false);
    resolve(api_.lib, api_.bad_pages, "amdsmi_get_gpu_bad_page_info", false);
    resolve(api_.lib, api_.bad_page_threshold, "amdsmi_get_gpu_bad_page_threshold", false);
    resolve(api_.lib, api_.ecc_enabled, "amdsmi_get_gpu_ecc_enabled", false);
    resolve(api_.lib, api_.ecc_count, "amdsmi_get_gpu_ecc_count", false);
    resolve(api_.lib, api_.process_list, "amdsmi_get_gpu_process_list", false);
    resolve(api_.lib, api_.pcie_info, "amdsmi_get_pcie_info", false);
    resolve(api_.lib, api_.driver_info, "amdsmi_get_gpu_driver_info", false);
    resolve(api_.lib, api_.vbios_info, "amdsmi_get_gpu_vbios_info", false);
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
    for (size_t i = 0; i < handles_.size(); ++i) handle_mu_.push_back(std::make_unique<std::mutex>());
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
        if (api_.get_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) g.bdf = bdf_string(bdf);
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
        if (api_.get_enum(h, &e) == AMDSMI_STATUS_SUCCESS) {
          g.hip_id = static_cast<int>(e.hip_id);
          if (e.drm_render != 0xFFFFFFFFu && e.drm_render != 0) g.drm_render = static_cast<int>(e.drm_render);
          if (e.drm_card != 0xFFFFFFFFu) g.drm_card = static_cast<int>(e.drm_card);
        }
      }
      if (api_.bad_page_threshold) {
        uint32_t thr = 0;
        if (api_.bad_page_threshold(h, &thr) == AMDSMI_STATUS_SUCCESS && thr != 0xFFFFFFFFu) g.bad_page_threshold = thr;
      }
      if (api_.pcie_info) {
        amdsmi_pcie_info_t pi;
        std::memset(&pi, 0, sizeof(pi));
        if (api_.pcie_info(h, &pi) == AMDSMI_STATUS_SUCCESS) {
          const auto& ps = pi.pcie_static;
          if (ps.max_pcie_width != 0xFFFF && ps.max_pcie_width != 0) g.pcie_max_width = ps.max_pcie_width;
          if (ps.max_pcie_speed != 0xFFFFFFFFu && ps.max_pcie_speed != 0) {
            // documented as GT/s, reported as MT/s by some firmware: normalise to MT/s
            g.pcie_max_speed_mts = static_cast<int>(ps.max_pcie_speed < 1000 ? ps.max_pcie_speed * 1000 : ps.max_pcie_speed);
          }
          const uint32_t gen = ps.max_pcie_interface_version != 0xFFFFFFFFu && ps.max_pcie_interface_version != 0
                                   ? ps.max_pcie_interface_version
                                   : ps.pcie_interface_version;
          if (gen != 0xFFFFFFFFu && gen != 0) g.pcie_max_gen = static_cast<int>(gen);
        }
      }
      if (api_.driver_info) {
        amdsmi_driver_info_t d;
        std::memset(&d, 0, sizeof(d));
        if (api_.driver_info(h, &d) == AMDSMI_STATUS_SUCCESS) {
          g.driver_name = cstr(d.driver_name, sizeof(d.driver_name));
          g.driver_version = cstr(d.driver_version, sizeof(d.driver_version));
        }
      }
      if (api_.vbios_info) {
        amdsmi_vbios_info_t vb;
        std::memset(&vb, 0, sizeof(vb));
        if (api_.vbios_info(h, &vb) == AMDSMI_STATUS_SUCCESS) {
          g.vbios_version = cstr(vb.version, sizeof(vb.version));
          g.vbios_part_number = cstr(vb.part_number, sizeof(vb.part_number));
        }
      }
      g.phys_links = read_links(h);
      // Peer links: one amdsmi topology query per ordered pair (8 GPUs: 56 pairs, once
      // at discovery, never on the poll path).
      for (size_t j = 0; j < handles_.size(); ++j) {
        if (j == i) continue;
        PeerLink l;
        l.peer = static_cast<int>(j);
        if (api_.topo_link_type) {
          uint64_t hops = 0;
          amdsmi_link_type_t type = AMDSMI_LINK_TYPE_UNKNOWN;
          if (api_.topo_link_type(h, handles_[j], &hops, &type) == AMDSMI_STATUS_SUCCESS) {
            l.hops = hops;
            l.type = link_type_name(type);
          }
        }
        if (l.type.empty()) l.type = "unknown";
        if (api_.topo_link_weight) {
          uint64_t w = 0;
          if (api_.topo_link_weight(h, handles_[j], &w) == AMDSMI_STATUS_SUCCESS) l.weight = w;
        }
        if (api_.minmax_bw && l.type == "xgmi") {
          uint64_t lo = 0, hi = 0;
          if (api_.minmax_bw(h, handles_[j], &lo, &hi) == AMDSMI_STATUS_SUCCESS) {
            l.min_bw_mbps = lo;
            l.max_bw_mbps = hi;
          }
        }
        g.links.push_back(std::move(l));
      }
      out.push_back(g);
    }
    return out;
  }

  int busy_processes(int index) override {
    if (index < 0 || static_cast<size_t>(index) >= handles_.size() || !api_.process_list) return -1;
    // Processes other than this one that hold memory on the GPU or have run work on it.
    // A process that merely opened the device (a monitoring daemon's KFD context: no
    // VRAM, no GTT, no engine time; on the MI355X box one such host process is always
    // listed) is not a tenant.  A container's getpid() is not the host PID KFD reports,
    // so the agent keeps HIP out of its own process (gpu/diag_runner.h) rather than rely
    // on recognising itself here.
    std::lock_guard<std::mutex> hl(*handle_mu_[static_cast<size_t>(index)]);
    std::vector<amdsmi_proc_info_t> procs(64);
    uint32_t n = static_cast<uint32_t>(procs.size());
    amdsmi_status_t st = api_.process_list(handles_[static_cast<size_t>(index)], &n, procs.data());
    if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) return -1;
    const uint32_t self = static_cast<uint32_t>(::getpid());
    int others = 0;
    for (uint32_t k = 0; k < n && k < procs.size(); ++k) {
      const auto& p = procs[k];
      const bool holds = p.mem > 0 || p.memory_usage.vram_mem > 0 || p.memory_usage.gtt_mem > 0 || p.engine_usage.gfx > 0;
      others += p.pid != self && holds ? 1 : 0;
    }
    if (n > procs.size()) others += static_cast<int>(n - procs.size());
    return others;
  }

  Value processes(int index) override {
    Value out = Value::array();
    if (index < 0 || static_cast<size_t>(index) >= handles_.size() || !api_.process_list) return out;
    std::lock_guard<std::mutex> hl(*handle_mu_[static_cast<size_t>(index)]);
    std::vector<amdsmi_proc_info_t> procs(64);
    uint32_t n = static_cast<uint32_t>(procs.size());
    amdsmi_status_t st = api_.process_list(handles_[static_cast<size_t>(index)], &n, procs.data());
    if (st != AMDSMI_STATUS_SUCCESS && st != AMDSMI_STATUS_OUT_OF_RESOURCES) return out;
    for (uint32_t k = 0; k < n && k < procs.size(); ++k) {
      const auto& p = procs[k];
      const bool holds = p.mem > 0 || p.memory_usage.vram_mem > 0 || p.memory_usage.gtt_mem > 0 || p.engine_usage.gfx > 0;
      out.push_back(Value::object({{"pid", static_cast<unsigned long long>(p.pid)},
                                   {"name", std::string(p.name, strnlen(p.name, sizeof(p.name)))},
                                   {"vram_bytes", static_cast<unsigned long long>(p.memory_usage.vram_mem)},
                                   {"gtt_bytes", static_cast<unsigned long long>(p.memory_usage.gtt_mem)},
                                   {"gfx_ns", static_cast<unsigned long long>(p.engine_usage.gfx)},
                                   {"holds", holds}}));
    }
    return out;
  }

  std::vector<PhysLink> read_links(amdsmi_processor_handle h) {
    std::vector<PhysLink> out;
    if (!api_.link_metrics) return out;
    amdsmi_link_metrics_t lm;
    std::memset(&lm, 0, sizeof(lm));
    if (api_.link_metrics(h, &lm) != AMDSMI_STATUS_SUCCESS) return out;
    const uint32_t n = std::min<uint32_t>(lm.num_links, AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK);
    for (uint32_t k = 0; k < n; ++k) {
      const auto& x = lm.links[k];
      PhysLink l;
      l.peer_bdf = x.bdf.as_uint == ~0ULL ? "" : bdf_string(x.bdf);  // all-ones: peer not reported
      l.type = link_type_name(x.link_type);
      l.bit_rate_gbps = x.bit_rate == 0xFFFFFFFFu ? 0 : x.bit_rate;
      l.max_bandwidth_gbps = x.max_bandwidth == 0xFFFFFFFFu ? 0 : x.max_bandwidth;
      l.read_kb = x.read == ~0ULL ? 0 : x.read;
      l.write_kb = x.write == ~0ULL ? 0 : x.write;
      out.push_back(std::move(l));
    }
    return out;
  }

  Telemetry sample(int index, SampleLevel level) override {
    const bool full = level >= SampleLevel::Slow;
    Telemetry t;
    t.index = index;
    int64_t t0 = metrics::now_ns();
    t.ts_ns = t0;
    if (index < 0 || static_cast<size_t>(index) >= handles_.size()) {
      t.error = "no such device";
      return t;
    }
    auto h = handles_[static_cast<size_t>(index)];
    // One call at a time per handle: the poller samples different handles concurrently
    // (safe: libamd_smi/rocm_smi lock per device), while the diagnostics thread's
    // busy_processes() may hit the same handle — serialized here instead of letting the
    // library's device mutex answer AMDSMI_STATUS_BUSY.
    std::unique_lock<std::mutex> hl(*handle_mu_[static_cast<size_t>(index)], std::defer_lock);
    {
      roctx::Range r("bgc.amdsmi.handle_lock");  // waiting for the diagnostics thread's call, if any
      hl.lock();
    }
    if (!api_.get_metrics) {
      t.error = "amdsmi_get_gpu_metrics_info unavailable";
      return t;
    }
    amdsmi_gpu_metrics_t m;
    std::memset(&m, 0, sizeof(m));
    amdsmi_status_t st;
    {
      roctx::Range r("bgc.amdsmi.gpu_metrics_info");
      st = api_.get_metrics(h, &m);
    }
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
    // Both throttle words use all-ones as "not reported" (MI355X firmware leaves the
    // 32-bit legacy word at 0xFFFFFFFF; round 1 exported that as if it were a state).
    if (m.indep_throttle_status != ~0ULL) {
      t.throttle_valid = true;
      t.throttle_status = m.indep_throttle_status;
    } else if (m.throttle_status != 0xFFFFFFFFu) {
      t.throttle_valid = true;
      t.throttle_status = m.throttle_status;
    }
    // Violation residency accumulators (the cheap path amdsmi_get_violation_status's own
    // documentation points bare-metal callers to; that call blocks >= 100 ms per device).
    if (m.accumulation_counter != ~0ULL && m.accumulation_counter != 0) {
      t.acc_counter = m.accumulation_counter;
      if (m.ppt_residency_acc != ~0ULL) t.acc_ppt = m.ppt_residency_acc;
      uint64_t thermal = Telemetry::kNoAcc;
      for (uint64_t a : {m.socket_thm_residency_acc, m.hbm_thm_residency_acc, m.vr_thm_residency_acc,
                         m.prochot_residency_acc}) {
        if (a == ~0ULL) continue;
        thermal = thermal == Telemetry::kNoAcc ? a : std::max(thermal, a);
      }
      t.acc_thermal = thermal;
    }
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
      roctx::Range r("bgc.amdsmi.vram_usage");
      if (api_.get_vram_usage(h, &u) == AMDSMI_STATUS_SUCCESS) {
        t.vram_used_mb = u.vram_used;
        t.vram_total_mb = u.vram_total;
      }
    }
    if (full && api_.get_ecc) {
      amdsmi_error_count_t e{};
      roctx::Range r("bgc.amdsmi.total_ecc_count");
      if (api_.get_ecc(h, &e) == AMDSMI_STATUS_SUCCESS) {
        t.ecc_correctable = e.correctable_count;
        t.ecc_uncorrectable = e.uncorrectable_count;
        t.ecc_deferred = e.deferred_count;
      }
    }
    if (full && api_.pcie_info) {
      amdsmi_pcie_info_t pi;
      std::memset(&pi, 0, sizeof(pi));
      roctx::Range r("bgc.amdsmi.pcie_info");
      if (api_.pcie_info(h, &pi) == AMDSMI_STATUS_SUCCESS) {
        const auto& pm = pi.pcie_metric;
        auto cnt = [](uint64_t v) { return v == ~0ULL ? int64_t{-1} : static_cast<int64_t>(v); };
        if (pm.pcie_width != 0xFFFF) t.pcie_width = pm.pcie_width;
        if (pm.pcie_speed != 0xFFFFFFFFu) t.pcie_speed_mts = static_cast<int>(pm.pcie_speed);
        t.pcie_replays = cnt(pm.pcie_replay_count);
        t.pcie_recoveries = cnt(pm.pcie_l0_to_recovery_count);
        t.pcie_nak_sent = cnt(pm.pcie_nak_sent_count);
        t.pcie_nak_received = cnt(pm.pcie_nak_received_count);
      }
    }
    if (level == SampleLevel::Ras) sample_ras(h, t);
    t.poll_us = static_cast<double>(metrics::now_ns() - t0) / 1e3;
    return t;
  }

 private:
  void sample_ras(amdsmi_processor_handle h, Telemetry& t) {
    t.ras_ok = true;
    if (api_.bad_pages) {
      roctx::Range r("bgc.amdsmi.bad_page_info");
      uint32_t n = 0;
      if (api_.bad_pages(h, &n, nullptr) == AMDSMI_STATUS_SUCCESS && n > 0) {
        std::vector<amdsmi_retired_page_record_t> recs(n);
        if (api_.bad_pages(h, &n, recs.data()) == AMDSMI_STATUS_SUCCESS) {
          for (uint32_t k = 0; k < n && k < recs.size(); ++k) {
            if (recs[k].status == AMDSMI_MEM_PAGE_STATUS_UNRESERVABLE) ++t.unreservable_pages;
            else ++t.retired_pages;
          }
        }
      }
    }
    if (api_.ecc_count) {
      roctx::Range r("bgc.amdsmi.ecc_count_per_block");
      uint64_t enabled = ~0ULL;
      if (api_.ecc_enabled && api_.ecc_enabled(h, &enabled) != AMDSMI_STATUS_SUCCESS) enabled = ~0ULL;
      for (const auto& b : kEccBlocks) {
        if (!(enabled & static_cast<uint64_t>(b.block))) continue;
        amdsmi_error_count_t e{};
        if (api_.ecc_count(h, b.block, &e) != AMDSMI_STATUS_SUCCESS) continue;
        t.ecc_blocks.push_back({b.name, e.correctable_count, e.uncorrectable_count, e.deferred_count});
      }
    }
    roctx::Range r("bgc.amdsmi.link_metrics");
    t.links = read_links(h);
  }

  AmdSmiApi api_;
  bool initialized_ = false;
  std::vector<amdsmi_processor_handle> handles_;
  std::vector<std::unique_ptr<std::mutex>> handle_mu_;  // per-handle call serialization
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

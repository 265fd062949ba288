#include "gpu/node_agent.h"

#include <cctype>
#include <cmath>
#include <cstdio>
#include <set>

#include <unistd.h>

#include "core/log.h"
#include "core/metrics.h"
#include "gpu/diag.h"
#include "kube/leader.h"
#include "kube/runtime.h"

namespace bgc::gpu {

using json::Value;
namespace types = kube::types;

NodeAgentConfig NodeAgentConfig::from_env(const EnvConfig& env) {
  NodeAgentConfig c;
  c.listen_addr = env.str("listen_addr");
  c.listen_port = env.u16("listen_port");
  c.node_name = env.str("node_name");
  c.backend = env.str_or("gpu_backend", "auto");
  c.mock_fixture_path = env.str_or("mock_fixture_path", "");
  c.poll_interval_ms = env.u64_or("poll_interval_ms", 1000);
  c.heartbeat_secs = env.u64_or("heartbeat_secs", 30);
  c.telemetry_stall_ms = env.u64_or("telemetry_stall_ms", c.telemetry_stall_ms);
  c.shutdown_timeout_secs = env.u64_or("shutdown_timeout_secs", c.shutdown_timeout_secs);
  c.resource_name = env.str_or("resource_name", "amd.com/gpu");
  c.partition_resource_name = env.str_or("partition_resource_name", c.partition_resource_name);
  c.label_prefix = env.str_or("label_prefix", "amd.com/gpu");
  c.max_gpus = static_cast<int>(env.u64_or("max_gpus", 0));
  c.run_diag = env.boolean_or("run_diag", false);
  c.diag_hbm_bytes = env.u64_or("diag_hbm_bytes", 1ULL << 30);
  c.diag_interval_secs = env.u64_or("diag_interval_secs", 0);
  c.diag_hbm_walk_fraction = env.f64_or("diag_hbm_walk_fraction", c.diag_hbm_walk_fraction);
  c.diag_hbm_walk_chunk_mb = env.u64_or("diag_hbm_walk_chunk_mb", c.diag_hbm_walk_chunk_mb);
  c.diag_hbm_walk_budget_ms = env.u64_or("diag_hbm_walk_budget_ms", c.diag_hbm_walk_budget_ms);
  c.diag_fence_settle_ms = env.u64_or("diag_fence_settle_ms", c.diag_fence_settle_ms);
  c.diag_start_busy = env.str_or("diag_start_busy", c.diag_start_busy);
  if (c.diag_start_busy != "skip" && c.diag_start_busy != "diagnose") {
    throw std::runtime_error("CONF_DIAG_START_BUSY must be skip or diagnose, not " + c.diag_start_busy);
  }
  c.diag_floors.min_hbm_walk_coverage = env.f64_or("diag_min_hbm_walk_coverage", c.diag_floors.min_hbm_walk_coverage);
  c.diag_floors.min_node_burn_balance = env.f64_or("diag_min_node_burn_balance", c.diag_floors.min_node_burn_balance);
  c.diag_floors.max_node_power_w = env.f64_or("diag_max_node_power_w", c.diag_floors.max_node_power_w);
  c.diag_burn_ms = env.u64_or("diag_burn_ms", 0);
  c.diag_burn_dtype = env.str_or("diag_burn_dtype", c.diag_burn_dtype);
  (void)burn_dtype_code(c.diag_burn_dtype);  // bf16 | fp8 | fp4, else the agent does not start
  c.diag_pcie_bytes = env.u64_or("diag_pcie_bytes", c.diag_pcie_bytes);
  c.diag_soak_size = static_cast<int>(env.u64_or("diag_soak_size", static_cast<uint64_t>(c.diag_soak_size)));
  c.diag_soak_launches = static_cast<int>(env.u64_or("diag_soak_launches", static_cast<uint64_t>(c.diag_soak_launches)));
  c.diag_floors.min_soak_tflops = env.f64_or("diag_min_soak_tflops", c.diag_floors.min_soak_tflops);
  c.diag_lowp = env.boolean_or("diag_lowp", c.diag_lowp);
  c.diag_floors.min_fp8_tflops = env.f64_or("diag_min_fp8_tflops", c.diag_floors.min_fp8_tflops);
  c.diag_floors.min_fp4_tflops = env.f64_or("diag_min_fp4_tflops", c.diag_floors.min_fp4_tflops);
  c.diag_floors.min_pcie_h2d_gbps = env.f64_or("diag_min_pcie_h2d_gbps", c.diag_floors.min_pcie_h2d_gbps);
  c.diag_floors.min_pcie_d2h_gbps = env.f64_or("diag_min_pcie_d2h_gbps", c.diag_floors.min_pcie_d2h_gbps);
  c.diag_floors.require_full_pcie_width = env.boolean_or("diag_require_full_pcie_width", c.diag_floors.require_full_pcie_width);
  c.diag_floors.min_pcie_speed_fraction = env.f64_or("diag_min_pcie_speed_fraction", c.diag_floors.min_pcie_speed_fraction);
  c.diag_floors.min_burn_tflops = env.f64_or("diag_min_burn_tflops", c.diag_floors.min_burn_tflops);
  c.diag_floors.min_burn_sustain = env.f64_or("diag_min_burn_sustain", c.diag_floors.min_burn_sustain);
  c.diag_floors.max_burn_hotspot_c = env.f64_or("diag_max_burn_hotspot_c", c.diag_floors.max_burn_hotspot_c);
  c.diag_floors.max_burn_thermal_violation_pct =
      env.f64_or("diag_max_burn_thermal_violation_pct", c.diag_floors.max_burn_thermal_violation_pct);
  c.diag_floors.min_read_gbps = env.f64_or("diag_min_read_gbps", c.diag_floors.min_read_gbps);
  c.diag_floors.min_copy_gbps = env.f64_or("diag_min_copy_gbps", c.diag_floors.min_copy_gbps);
  c.diag_floors.min_write_gbps = env.f64_or("diag_min_write_gbps", c.diag_floors.min_write_gbps);
  c.diag_floors.min_mfma_tflops = env.f64_or("diag_min_mfma_tflops", c.diag_floors.min_mfma_tflops);
  c.diag_floors.min_xcc_balance = env.f64_or("diag_min_xcc_balance", c.diag_floors.min_xcc_balance);
  c.diag_floors.min_xccs = static_cast<int>(env.u64_or("diag_min_xccs", static_cast<uint64_t>(c.diag_floors.min_xccs)));
  c.pod_resources_socket = env.str_or("pod_resources_socket", c.pod_resources_socket);
  HealthPolicy& h = c.health;
  h.max_hotspot_c = env.f64_or("max_hotspot_c", h.max_hotspot_c);
  h.max_mem_c = env.f64_or("max_mem_c", h.max_mem_c);
  h.max_new_uncorrectable = env.u64_or("max_new_uncorrectable", h.max_new_uncorrectable);
  h.max_uncorrectable_at_start = env.u64_or("max_uncorrectable_at_start", h.max_uncorrectable_at_start);
  h.require_all_xgmi_links = env.boolean_or("require_all_xgmi_links", h.require_all_xgmi_links);
  h.max_retired_pages = env.u64_or("max_retired_pages", h.max_retired_pages);
  h.max_thermal_violation_pct = env.f64_or("max_thermal_violation_pct", h.max_thermal_violation_pct);
  h.max_ppt_violation_pct = env.f64_or("max_ppt_violation_pct", h.max_ppt_violation_pct);
  h.violation_sustain_polls = static_cast<int>(env.u64_or("violation_sustain_polls", static_cast<uint64_t>(h.violation_sustain_polls)));
  h.require_full_pcie_width = env.boolean_or("require_full_pcie_width", h.require_full_pcie_width);
  h.max_pcie_replays_per_poll = static_cast<int64_t>(env.u64_or("max_pcie_replays_per_poll", static_cast<uint64_t>(h.max_pcie_replays_per_poll)));
  h.fail_threshold = static_cast<int>(env.u64_or("fail_threshold", static_cast<uint64_t>(h.fail_threshold)));
  h.recover_threshold = static_cast<int>(env.u64_or("recover_threshold", static_cast<uint64_t>(h.recover_threshold)));
  c.slow_every = static_cast<int>(env.u64_or("slow_every", static_cast<uint64_t>(c.slow_every)));
  c.ras_every = static_cast<int>(env.u64_or("ras_every", static_cast<uint64_t>(c.ras_every)));
  c.create_node = env.boolean_or("create_node", false);
  c.events = env.boolean_or("events", true);
  c.device_plugin = env.boolean_or("device_plugin", false);
  c.device_plugin_dir = env.str_or("device_plugin_dir", c.device_plugin_dir);
  c.device_plugin_socket = env.str_or("device_plugin_socket", c.device_plugin_socket);
  c.device_plugin_cdi = env.boolean_or("device_plugin_cdi", false);
  c.cdi_dir = env.str_or("cdi_dir", c.cdi_dir);
  c.dev_root = env.str_or("dev_root", c.dev_root);
  c.sysfs_root = env.str_or("sysfs_root", c.sysfs_root);
  c.advertiser_check = env.boolean_or("advertiser_check", c.advertiser_check);
  c.take_over = env.boolean_or("take_over", c.take_over);
  if (env.raw("known_labellers")) c.known_labellers = env.comma_list("known_labellers");
  return c;
}

std::string sanitize_label_value(const std::string& v) {
  std::string out;
  for (char c : v) {
    if (std::isalnum(static_cast<unsigned char>(c)) || c == '-' || c == '_' || c == '.') out.push_back(c);
    else if (c == ' ' || c == '/' || c == ':') out.push_back('_');
  }
  while (!out.empty() && !std::isalnum(static_cast<unsigned char>(out.front()))) out.erase(0, 1);
  while (!out.empty() && !std::isalnum(static_cast<unsigned char>(out.back()))) out.pop_back();
  if (out.size() > 63) out.resize(63);
  while (!out.empty() && !std::isalnum(static_cast<unsigned char>(out.back()))) out.pop_back();
  return out;
}

std::string advertised_resource(const NodeAgentConfig& cfg, const std::vector<GpuInfo>& gpus) {
  if (cfg.partition_resource_name.empty() || gpus.empty()) return cfg.resource_name;
  for (const auto& g : gpus) {
    const std::string& p = g.compute_partition;
    if (p.empty() || p == "SPX" || p == "unknown") return cfg.resource_name;
  }
  return cfg.partition_resource_name;
}

std::string product_label(const GpuInfo& g) {
  const std::string& m = g.market_name;
  if (m.find("MI355") != std::string::npos) return "MI355X";
  if (m.find("MI350") != std::string::npos) return "MI350X";
  if (g.gfx_target.rfind("gfx950", 0) == 0) return "MI355X";
  std::string s = m;
  const std::string prefix = "AMD Instinct ";
  if (s.rfind(prefix, 0) == 0) s = s.substr(prefix.size());
  return sanitize_label_value(s);
}

static std::string hex16(uint64_t v) {
  char buf[32];
  std::snprintf(buf, sizeof(buf), "%016llx", static_cast<unsigned long long>(v));
  return buf;
}

Value node_labels_patch(const NodeAgentConfig& cfg, const std::vector<GpuInfo>& gpus, int healthy,
                        const DiagOutcome& diag) {
  const std::string& p = cfg.label_prefix;
  Value labels = Value::object();
  labels[p + ".present"] = gpus.empty() ? "false" : "true";
  labels[p + ".count"] = std::to_string(gpus.size());
  labels[p + ".healthy-count"] = std::to_string(healthy);
  if (!gpus.empty()) {
    const GpuInfo& g = gpus.front();
    std::string family = g.gfx_target;
    size_t colon = family.find(':');
    if (colon != std::string::npos) family = family.substr(0, colon);
    labels[p + ".family"] = sanitize_label_value(family);
    labels[p + ".product"] = product_label(g);
    labels[p + ".market-name"] = sanitize_label_value(g.market_name);
    uint64_t min_vram = UINT64_MAX;
    std::set<uint64_t> hives;
    for (const auto& x : gpus) {
      min_vram = std::min(min_vram, x.vram_total_mb);
      hives.insert(x.xgmi_hive_id);
    }
    labels[p + ".vram-gb"] = std::to_string(static_cast<uint64_t>(std::llround(static_cast<double>(min_vram) / 1024.0)));
    // One hive id when every GPU sits on the same xGMI island; otherwise "mixed" plus
    // the number of islands (TP groups must then be pinned per island).
    labels[p + ".xgmi-hive-id"] = hives.size() == 1 ? hex16(*hives.begin()) : "mixed";
    labels[p + ".xgmi-hives"] = std::to_string(hives.size());
    labels[p + ".compute-partition"] = sanitize_label_value(g.compute_partition.empty() ? "unknown" : g.compute_partition);
    labels[p + ".memory-partition"] = sanitize_label_value(g.memory_partition.empty() ? "unknown" : g.memory_partition);
    if (g.num_cus) labels[p + ".cu-count"] = std::to_string(g.num_cus);
    // Driver / VBIOS identity; "mixed" flags a node caught mid-way through a firmware
    // rollout (one value per node, as every GPU of a UBB should match).
    auto common = [&](auto field) {
      std::set<std::string> vals;
      for (const auto& x : gpus) vals.insert(x.*field);
      if (vals.size() > 1) return std::string("mixed");
      std::string v = sanitize_label_value(*vals.begin());
      return v.empty() ? std::string("unknown") : v;
    };
    labels[p + ".driver-version"] = common(&GpuInfo::driver_version);
    labels[p + ".vbios-version"] = common(&GpuInfo::vbios_version);
  }
  labels[p + ".diag"] = !diag.ran ? "skipped" : diag.passed ? "passed" : "failed";
  Value topo = Value::array();
  for (const auto& g : gpus) {
    Value links = Value::array();
    for (const auto& l : g.links) {
      links.push_back(Value::object({{"peer", l.peer}, {"type", l.type}, {"hops", static_cast<unsigned long long>(l.hops)},
                                     {"weight", static_cast<unsigned long long>(l.weight)},
                                     {"bw_mbps", static_cast<unsigned long long>(l.max_bw_mbps)}}));
    }
    int xgmi_up = 0;
    for (const auto& l : g.phys_links) xgmi_up += (l.type == "xgmi" && l.bit_rate_gbps > 0) ? 1 : 0;
    topo.push_back(Value::object({{"index", g.index}, {"uuid", g.uuid}, {"bdf", g.bdf}, {"hive", hex16(g.xgmi_hive_id)},
                                  {"node", static_cast<unsigned long long>(g.xgmi_node_id)}, {"numa", g.numa_node},
                                  {"render", g.drm_render}, {"xgmi_links_up", xgmi_up}, {"links", links}}));
  }
  Value meta = Value::object({{"name", cfg.node_name}, {"labels", labels},
                              {"annotations", Value::object({{p + ".topology", topo.dump()}})}});
  return Value::object({{"apiVersion", "v1"}, {"kind", "Node"}, {"metadata", meta}});
}

Value node_status_patch(const NodeAgentConfig& cfg, const std::vector<GpuInfo>& gpus, int healthy,
                        const std::string& unhealthy_reason) {
  Value status = Value::object();
  if (!cfg.device_plugin) {  // with the device plugin the kubelet owns these counts
    status["capacity"] = Value::object({{cfg.resource_name, std::to_string(gpus.size())}});
    status["allocatable"] = Value::object({{cfg.resource_name, std::to_string(healthy)}});
  }
  bool all_ok = healthy == static_cast<int>(gpus.size()) && !gpus.empty();
  Value cond = Value::object({{"type", "AMDGPUHealthy"},
                              {"status", all_ok ? "True" : "False"},
                              {"reason", all_ok ? "AllGPUsHealthy" : "GPUUnhealthy"},
                              {"message", all_ok ? std::to_string(healthy) + " MI355X GPUs healthy" : unhealthy_reason},
                              {"lastHeartbeatTime", kube::rfc3339_micro_now().substr(0, 19) + "Z"}});
  status["conditions"] = Value::array({cond});
  return Value::object({{"apiVersion", "v1"}, {"kind", "Node"}, {"metadata", Value::object({{"name", cfg.node_name}})},
                        {"status", status}});
}

bool label_owner_conflicts(const NodeAgentConfig& cfg, const std::string& manager, const std::string& operation) {
  for (const auto& k : cfg.known_labellers) {
    if (!k.empty() && manager == k) return true;
  }
  (void)operation;  // labelling controllers write with Update as often as with Apply
  return manager.rfind("kubectl", 0) != 0;
}

Value foreign_field_owners(const NodeAgentConfig& cfg, const Value& node) {
  Value out = Value::array();
  const std::string label_key = "f:" + cfg.label_prefix + ".";
  const std::string res_key = "f:" + cfg.resource_name;
  for (const auto& mf : node.get("metadata").get("managedFields").items()) {
    const std::string manager = mf.get_string("manager");
    if (manager == kNodeAgentManager) continue;
    const Value& f = mf.get("fieldsV1");
    Value labels = Value::array();
    const Value& lf = f.get("f:metadata").get("f:labels");
    if (lf.is_object()) {
      for (const auto& k : lf.keys()) {
        if (k.rfind(label_key, 0) == 0) labels.push_back(k.substr(2));
      }
    }
    if (!labels.empty()) {
      const std::string op = mf.get_string("operation");
      out.push_back(Value::object({{"kind", "labels"}, {"manager", manager}, {"operation", op}, {"fields", labels},
                                   {"conflict", label_owner_conflicts(cfg, manager, op)}}));
    }
    // the kubelet writes a device plugin's counts: that is this agent's own plugin unless
    // the agent advertises through the Node status itself
    if (manager == "kubelet" && cfg.device_plugin) continue;
    Value res = Value::array();
    for (const char* sect : {"f:capacity", "f:allocatable"}) {
      const Value& sf = f.get("f:status").get(sect);
      if (sf.is_object() && sf.contains(res_key)) res.push_back(std::string("status.") + (sect + 2) + "." + cfg.resource_name);
    }
    if (!res.empty()) {
      out.push_back(Value::object({{"kind", "capacity"}, {"manager", manager}, {"operation", mf.get_string("operation")},
                                   {"fields", res}, {"conflict", true}}));
    }
  }
  return out;
}

NodeAgent::NodeAgent(kube::KubeClient& client, std::unique_ptr<Backend> backend, NodeAgentConfig cfg)
    : client_(client), backend_(std::move(backend)), cfg_(std::move(cfg)) {
  if (cfg_.events) {
    kube::EventOptions eo;
    eo.component = "bgc-node-agent";
    eo.host = cfg_.node_name;
    events_ = std::make_unique<kube::EventRecorder>(client_, eo);
  }
}

static bool diag_failed(const DiagOutcome& d, size_t i);

void NodeAgent::node_event(const std::string& type, const std::string& reason, const std::string& message) {
  if (!events_) return;
  events_->record(types::Node, Value::object({{"metadata", Value::object({{"name", cfg_.node_name}})}}), type, reason,
                  message);
}

std::string NodeAgent::gpu_reason(size_t i) const {
  auto snap = poller_ ? poller_->snapshot() : nullptr;
  std::string why;
  if (snap && i < snap->health.size() && !snap->health[i].healthy) why = snap->health[i].reason;
  std::lock_guard<std::mutex> lk(diag_mu_);
  if (diag_failed(diag_, i)) {
    if (!why.empty()) why += "; ";
    why += "diagnostics failed " + diag_.per_gpu.items()[i].get("failures").dump();
  }
  return why;
}

void NodeAgent::emit_health_events() {
  if (!events_) return;
  const std::vector<bool> flags = healthy_flags();
  std::lock_guard<std::mutex> lk(event_mu_);
  event_state_.resize(gpus_.size(), -1);
  for (size_t i = 0; i < gpus_.size() && i < flags.size(); ++i) {
    const int now = flags[i] ? 1 : 0;
    const int was = event_state_[i];
    event_state_[i] = now;
    if (now == was || (was == -1 && now == 1)) continue;  // healthy at start is not news
    const std::string id = "gpu " + std::to_string(gpus_[i].index) + " (" + gpus_[i].bdf + ")";
    if (now == 0) node_event("Warning", "GPUUnhealthy", id + " unhealthy: " + gpu_reason(i));
    else node_event("Normal", "GPUHealthy", id + " healthy again");
  }
}

NodeAgent::~NodeAgent() { stop(); }

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

void NodeAgent::mark_advertised() {
  double zero = 0;
  first_advertise_ms_.compare_exchange_strong(zero, ms_since(t_created_));
}

void NodeAgent::init() {
  gpus_ = backend_->discover();
  discover_ms_ = ms_since(t_created_);
  if (cfg_.max_gpus > 0 && static_cast<int>(gpus_.size()) > cfg_.max_gpus) gpus_.resize(static_cast<size_t>(cfg_.max_gpus));
  if (gpus_.empty()) throw std::runtime_error("no GPUs discovered via " + backend_->name());
  const std::string res = advertised_resource(cfg_, gpus_);
  if (res != cfg_.resource_name) {
    LOG_INFO("node_agent") << "GPUs run " << gpus_.front().compute_partition << " compute partitions: advertising "
                           << gpus_.size() << " x " << res << " instead of " << cfg_.resource_name;
    cfg_.resource_name = res;
  }
  LOG_INFO("node_agent") << "discovered " << gpus_.size() << " GPU(s) via " << backend_->name() << ": "
                         << gpus_.front().market_name << " " << gpus_.front().gfx_target << " "
                         << gpus_.front().vram_total_mb << " MB";
  if (cfg_.run_diag) {
    const auto t0 = std::chrono::steady_clock::now();
    run_diagnostics(true);
    startup_diag_ms_ = ms_since(t0);
  }
  std::vector<int> idx;
  std::vector<uint64_t> page_limits;
  for (const auto& g : gpus_) {
    idx.push_back(g.index);
    page_limits.push_back(g.bad_page_threshold);
  }
  poller_ = std::make_unique<TelemetryPoller>(*backend_, idx, std::chrono::milliseconds(cfg_.poll_interval_ms),
                                              cfg_.health, cfg_.slow_every, cfg_.ras_every, page_limits);
  for (size_t k = 0; k < gpus_.size(); ++k) poller_->set_pcie_max_width(k, gpus_[k].pcie_max_width);
  poller_->set_stall_timeout(std::chrono::milliseconds(cfg_.telemetry_stall_ms));
  poller_->poll_once();
  bool exists = client_.get_opt(types::Node, "", cfg_.node_name).has_value();
  if (cfg_.create_node && !exists) {
    client_.create(types::Node, "", Value::object({{"apiVersion", "v1"}, {"kind", "Node"},
                                                   {"metadata", Value::object({{"name", cfg_.node_name}})}}));
    exists = true;
  }
  node_present_ = exists;
  if (!exists) LOG_WARN("node_agent") << "node " << cfg_.node_name << " is not registered yet; waiting for the kubelet";
  check_advertisers();
}

Value NodeAgent::advertiser_conflicts() const {
  std::lock_guard<std::mutex> lk(conflict_mu_);
  return conflicts_;
}

bool NodeAgent::check_advertisers() {
  if (!cfg_.advertiser_check) return false;
  Value found = Value::array();
  for (const auto& fp : foreign_plugins_for(cfg_.device_plugin_dir, "kubelet.sock", cfg_.device_plugin_socket,
                                            cfg_.resource_name, device_ids_for(gpus_))) {
    Value ids = Value::array();
    for (size_t k = 0; k < fp.ids.size() && k < 8; ++k) ids.push_back(fp.ids[k]);
    found.push_back(Value::object({{"kind", "device-plugin"},
                                   {"socket", cfg_.device_plugin_dir + "/" + fp.socket},
                                   {"resource", cfg_.resource_name},
                                   {"devices", static_cast<unsigned long long>(fp.ids.size())},
                                   {"device_ids", ids},
                                   {"evidence", fp.via_checkpoint ? "kubelet checkpoint" : "device ids"}}));
  }
  try {
    if (auto node = client_.get_opt(types::Node, "", cfg_.node_name)) {
      const Value owners = foreign_field_owners(cfg_, *node);
      for (const auto& o : owners.items()) found.push_back(o);
    }
  } catch (const std::exception& e) {
    LOG_WARN("node_agent") << "advertiser check: reading node " << cfg_.node_name << " failed: " << e.what();
  }
  // Foreign label owners that are no labelling controller (an admin's `kubectl label`) are
  // reported in /gpus but do not make the agent stand down.
  const bool conflict = std::any_of(found.items().begin(), found.items().end(), [](const Value& f) {
    return !f.get("conflict").is_bool() || f.get("conflict").as_bool();
  });
  const bool down = conflict && !cfg_.take_over;
  const std::string sig = found.dump();
  bool report;
  {
    std::lock_guard<std::mutex> lk(conflict_mu_);
    report = sig != conflict_sig_;
    conflict_sig_ = sig;
    conflicts_ = found;
  }
  const bool was_down = standing_down_.exchange(down);
  auto& reg = metrics::Registry::global();
  reg.gauge("bgc_node_agent_advertiser_conflicts", "Other advertisers of this node's GPUs found by the last check")
      .set(static_cast<double>(found.size()));
  reg.gauge("bgc_node_agent_standing_down", "1 while the agent leaves the GPUs to another advertiser").set(down ? 1 : 0);
  if (report && conflict) {
    const std::string what = "another advertiser of " + cfg_.resource_name + " on node " + cfg_.node_name + ": " + sig;
    if (down) {
      LOG_ERROR("node_agent") << what << "; standing down: no device-plugin registration and no label or status "
                              << "writes. Disable the other advertiser (e.g. the GPU Operator's device plugin and "
                              << "labeller), give this agent another resource_name/label_prefix, or set "
                              << "CONF_TAKE_OVER=true";
      node_event("Warning", "GPUAdvertiserConflict", what + "; bgc node agent standing down");
    } else {
      LOG_WARN("node_agent") << what << "; CONF_TAKE_OVER=true: advertising anyway";
      node_event("Warning", "GPUAdvertiserTakeOver", what + "; bgc node agent advertising anyway (take_over)");
    }
  } else if (!conflict && was_down) {
    LOG_INFO("node_agent") << "no other advertiser of " << cfg_.resource_name << " any more; advertising";
    node_event("Normal", "GPUAdvertiserConflictResolved", "no other advertiser of " + cfg_.resource_name);
  }
  return down;
}

bool NodeAgent::node_up_to_date(const Value& node) const {
  const Value& labels = node.get("metadata").get("labels");
  if (labels.get_string(cfg_.label_prefix + ".count") != std::to_string(gpus_.size())) return false;
  int healthy = healthy_count(nullptr);
  if (labels.get_string(cfg_.label_prefix + ".healthy-count") != std::to_string(healthy)) return false;
  if (cfg_.device_plugin) return true;
  const Value& st = node.get("status");
  return st.get("capacity").get_string(cfg_.resource_name) == std::to_string(gpus_.size()) &&
         st.get("allocatable").get_string(cfg_.resource_name) == std::to_string(healthy);
}

static bool diag_failed(const DiagOutcome& d, size_t i) {
  if (!d.ran || i >= d.per_gpu.items().size()) return false;
  const Value& r = d.per_gpu.items()[i];
  return r.is_object() && r.get("passed").is_bool() && !r.get("passed").as_bool();
}

std::vector<bool> NodeAgent::healthy_flags() const {
  auto snap = poller_ ? poller_->snapshot() : nullptr;
  std::lock_guard<std::mutex> lk(diag_mu_);
  std::vector<bool> out(gpus_.size(), true);
  for (size_t i = 0; i < gpus_.size(); ++i) {
    if (snap && i < snap->health.size() && !snap->health[i].healthy) out[i] = false;
    if (diag_failed(diag_, i)) out[i] = false;
  }
  return out;
}

DiagOutcome NodeAgent::diag_outcome() const {
  std::lock_guard<std::mutex> lk(diag_mu_);
  return diag_;
}

DiagPlan NodeAgent::diag_plan() const {
  DiagPlan p;
  p.hbm_bytes = cfg_.diag_hbm_bytes;
  p.hbm_walk_fraction = cfg_.diag_hbm_walk_fraction;
  p.hbm_walk_chunk_bytes = cfg_.diag_hbm_walk_chunk_mb << 20;
  p.hbm_walk_budget_ms = static_cast<int>(cfg_.diag_hbm_walk_budget_ms);
  p.pcie_bytes = cfg_.diag_pcie_bytes;
  p.soak_size = cfg_.diag_soak_size;
  p.soak_launches = cfg_.diag_soak_launches;
  p.lowp = cfg_.diag_lowp;
  p.burn_ms = static_cast<int>(cfg_.diag_burn_ms);
  return p;
}

void NodeAgent::setup_diag() {
  if (engine_) return;
  const Value script = backend_->diag_script();
  // HIP work runs in worker processes (make_process_diag_engine); BGC_DIAG_IN_PROCESS=1
  // keeps it in the agent, which then holds a GPU context on every GPU from the first pass
  const char* inproc = std::getenv("BGC_DIAG_IN_PROCESS");
  diag_in_process_ = inproc && std::string(inproc) == "1";
  // BGC_DIAG_WORKERS=1 with a scripted mock: the script runs inside worker processes, so
  // CPU tests cover the worker plumbing (spawn, results, common burn start, cancellation)
  const char* workers = std::getenv("BGC_DIAG_WORKERS");
  const bool scripted_workers = script.is_object() && workers && std::string(workers) == "1";
  if (script.is_object() && !scripted_workers) {
    engine_ = make_scripted_diag_engine(*backend_);
  } else if (diag_in_process_) {
    engine_ = make_hip_diag_engine();
  } else {
    pcie_lock_path_ = "/tmp/bgc-node-agent-" + std::to_string(::getpid()) + ".pcie.lock";
    engine_ = make_process_diag_engine("", cfg_.backend, cfg_.mock_fixture_path, pcie_lock_path_, &stop_);
  }
  std::vector<std::string> bdfs;
  if (engine_->name() == "hip" && !scripted_workers) {
    try {
      if (diag_in_process_) {
        Diag& d = Diag::instance();
        for (int i = 0, n = d.device_count(); i < n; ++i) bdfs.push_back(d.device_bdf(i));
      } else {
        bdfs = worker_device_bdfs("");
      }
    } catch (const std::exception& e) {
      LOG_WARN("node_agent") << "HIP device BDFs unavailable (" << e.what() << "); using amdsmi hip ids";
    }
  }
  hip_devs_ = hip_devices_for(gpus_, bdfs);
  {
    // workers verify that the one GPU they see is the one meant (BDF); partitions share a
    // BDF and are told apart by amdsmi's numbering only
    std::map<std::string, int> count;
    for (const auto& g : gpus_) count[g.bdf]++;
    std::map<int, std::string> by_dev;
    for (size_t i = 0; i < gpus_.size(); ++i) {
      if (!gpus_[i].bdf.empty() && count[gpus_[i].bdf] == 1) by_dev[hip_devs_[i]] = gpus_[i].bdf;
    }
    engine_->set_device_bdfs(std::move(by_dev));
  }
  LOG_INFO("node_agent") << "diagnostics engine " << engine_->name() << (diag_in_process_ ? " (in process)" : " (worker processes)")
                         << ", " << bdfs.size() << " HIP devices named by BDF";
}

std::vector<bool> NodeAgent::in_use() const {
  std::vector<bool> out(gpus_.size(), false);
  std::set<std::string> held;
  bool pod_api = false;
  if (!cfg_.pod_resources_socket.empty() && ::access(cfg_.pod_resources_socket.c_str(), F_OK) == 0) {
    try {
      held = allocated_device_ids(cfg_.pod_resources_socket, cfg_.resource_name);
      pod_api = true;
    } catch (const std::exception& e) {
      LOG_WARN("node_agent") << "pod-resources List failed: " << e.what() << "; falling back to amdsmi process lists";
    }
  }
  const std::vector<std::string> ids = plugin_ ? plugin_->ids() : std::vector<std::string>{};
  for (size_t i = 0; i < gpus_.size(); ++i) {
    if (pod_api && i < ids.size() && held.count(ids[i])) out[i] = true;
    if (backend_->busy_processes(gpus_[i].index) > 0) out[i] = true;
  }
  return out;
}

void NodeAgent::record_diag_gauges(size_t i, const Value& r) {
  auto get = [&](const char* sect, const char* k) {
    const Value& v = r.get(sect).get(k);
    return v.is_number() ? v.as_double() : 0.0;
  };
  // per-GPU results as gauges (Prometheus), so fleet dashboards see a slow GPU before it fails a floor
  auto& reg = metrics::Registry::global();
  const metrics::Labels gl{{"gpu", std::to_string(gpus_[i].index)}};
  struct G {
    const char *name, *help, *sect, *key;
  };
  static const G kGauges[] = {
      {"amd_gpu_diag_hbm_read_gbps", "Diagnostics: HBM read GB/s", "hbm", "read_gbps"},
      {"amd_gpu_diag_hbm_write_gbps", "Diagnostics: HBM write GB/s", "hbm", "write_gbps"},
      {"amd_gpu_diag_hbm_copy_gbps", "Diagnostics: HBM copy GB/s", "hbm", "copy_gbps"},
      {"amd_gpu_diag_hbm_walk_covered_bytes", "Diagnostics: HBM bytes pattern-walked", "hbm_walk", "bytes_covered"},
      {"amd_gpu_diag_hbm_walk_mismatches", "Diagnostics: HBM walk words read back wrong", "hbm_walk", "mismatches"},
      {"amd_gpu_diag_mfma_tflops", "Diagnostics: bf16 MFMA TFLOP/s (register operands)", "mfma", "tflops"},
      {"amd_gpu_diag_xcc_balance", "Diagnostics: fastest/slowest XCC wave time", "mfma", "xcc_balance"},
      {"amd_gpu_diag_fp8_tflops", "Diagnostics: MX fp8 MFMA TFLOP/s (register operands)", "lowp", "fp8_tflops"},
      {"amd_gpu_diag_fp4_tflops", "Diagnostics: MX fp4 MFMA TFLOP/s (register operands)", "lowp", "fp4_tflops"},
      {"amd_gpu_diag_soak_tflops", "Diagnostics: LDS-tiled MFMA GEMM soak TFLOP/s", "soak", "tflops_mean"},
      {"amd_gpu_diag_pcie_h2d_gbps", "Diagnostics: PCIe host-to-device GB/s", "pcie", "h2d_gbps"},
      {"amd_gpu_diag_pcie_d2h_gbps", "Diagnostics: PCIe device-to-host GB/s", "pcie", "d2h_gbps"},
      {"amd_gpu_diag_burn_tflops", "Diagnostics: burn-in mean MFMA TFLOP/s", "burn", "tflops_mean"},
      {"amd_gpu_diag_burn_max_hotspot_celsius", "Diagnostics: burn-in peak hotspot temperature", "burn", "max_hotspot_c"},
  };
  for (const auto& g : kGauges) {
    if (r.get(g.sect).get(g.key).is_number()) reg.gauge(g.name, g.help, gl).set(get(g.sect, g.key));
  }
  reg.gauge("amd_gpu_diag_passed", "1 when the last diagnostics pass of the GPU succeeded", gl)
      .set(r.get("passed").as_bool() ? 1 : 0);
  if (r.get("passed").as_bool()) {
    LOG_INFO("node_agent") << "diag gpu " << gpus_[i].index << ": passed in " << r.get("checks_ms").dump()
                           << " ms, read " << get("hbm", "read_gbps") << " GB/s, walk "
                           << get("hbm_walk", "bytes_covered") / 1e9 << " GB, mfma " << get("mfma", "tflops")
                           << " TFLOP/s, xcc balance " << get("mfma", "xcc_balance") << ", mx fp8/fp4 "
                           << get("lowp", "fp8_tflops") << "/" << get("lowp", "fp4_tflops") << " TFLOP/s, soak "
                           << get("soak", "tflops_mean") << " TFLOP/s, pcie " << get("pcie", "h2d_gbps") << "/"
                           << get("pcie", "d2h_gbps") << " GB/s, burn " << get("burn", "tflops_mean") << " TFLOP/s";
  } else {
    LOG_WARN("node_agent") << "diag gpu " << gpus_[i].index << ": FAILED " << r.get("failures").dump();
    node_event("Warning", "GPUDiagnosticsFailed",
               "gpu " + std::to_string(gpus_[i].index) + " (" + gpus_[i].bdf + "): " + r.get("failures").dump());
  }
}

bool NodeAgent::run_diagnostics(bool at_start) {
  setup_diag();
  using clock = std::chrono::steady_clock;
  const auto t_pass = clock::now();
  auto since = [&](clock::time_point t) { return std::chrono::duration<double, std::milli>(t - t_pass).count(); };
  DiagOutcome prev = diag_outcome();
  std::vector<Value> results(gpus_.size());
  uint64_t skipped = 0;
  auto keep_previous = [&](size_t i, const char* why) {
    ++skipped;
    if (i < prev.per_gpu.items().size()) results[i] = prev.per_gpu.items()[i];
    LOG_INFO("node_agent") << "diag gpu " << gpus_[i].index << ": skipped (" << why << ")";
  };
  // Allocation counters first: an Allocate that lands between the in_use() snapshot and
  // the fence shows up as a changed counter.
  const std::vector<uint64_t> allocs0 = plugin_ ? plugin_->allocation_counts() : std::vector<uint64_t>{};
  // Busy GPUs are left alone at start as well: an agent restarted (an upgrade, a crash) on
  // a node whose GPUs run tenants' jobs must not burn or walk them.  They keep no verdict
  // (not failed) until a periodic pass finds them free.
  const std::vector<bool> busy =
      at_start && cfg_.diag_start_busy == "diagnose" ? std::vector<bool>(gpus_.size(), false) : in_use();
  std::vector<size_t> todo;
  for (size_t i = 0; i < gpus_.size(); ++i) {
    if (busy[i]) keep_previous(i, "in use");
    else todo.push_back(i);
  }
  // Fence: withdraw the candidates from the kubelet (Unhealthy in ListAndWatch, refused
  // by Allocate), give an in-flight admission time to land, then re-check. Only GPUs
  // still free are diagnosed; the rest are released untouched.
  const bool fence = !at_start && plugin_ && !todo.empty();  // at start nothing is advertised yet
  // whatever happens below (an engine or judge exception), fenced GPUs are released
  struct Unfence {
    DevicePlugin* plugin;
    std::vector<size_t>* gpus;
    bool armed;
    ~Unfence() {
      if (!armed) return;
      try {
        plugin->set_fenced(*gpus, false);
      } catch (...) {
      }
    }
  } unfence{plugin_.get(), &todo, fence};
  if (fence) {
    plugin_->set_fenced(todo, true);
    if (stop_.wait_for(std::chrono::milliseconds(cfg_.diag_fence_settle_ms))) return false;  // unfenced on return
    const std::vector<bool> busy2 = in_use();
    const std::vector<uint64_t> allocs1 = plugin_->allocation_counts();
    std::vector<size_t> still, released;
    for (size_t i : todo) {
      const bool raced = busy2[i] || (i < allocs0.size() && i < allocs1.size() && allocs1[i] != allocs0[i]);
      (raced ? released : still).push_back(i);
    }
    for (size_t i : released) keep_previous(i, "allocated while being fenced");
    if (!released.empty()) plugin_->set_fenced(released, false);
    fence_races_ += released.size();
    todo = still;
  }
  const DiagPlan plan = diag_plan();
  // Phase 1: every GPU's checks at once, one thread per GPU.
  {
    std::vector<std::thread> threads;
    for (size_t i : todo) {
      threads.emplace_back([&, i] {
        const int dev = hip_devs_[i];
        const auto t0 = clock::now();
        Value r;
        try {
          r = engine_->checks(*backend_, gpus_[i], dev, plan, 0x5eed + static_cast<uint32_t>(dev));
        } catch (const std::exception& e) {
          r = Value::object({{"error", std::string(e.what())}});
        }
        r["index"] = gpus_[i].index;
        r["hip_device"] = dev;
        r["checks_started_ms"] = since(t0);
        r["checks_ms"] = std::chrono::duration<double, std::milli>(clock::now() - t0).count();
        results[i] = std::move(r);
      });
    }
    for (auto& t : threads) t.join();
  }
  // The agent is stopping (a DaemonSet rolling update): its workers were killed, so these
  // results say nothing about the GPUs.  Drop the pass — no verdicts, gauges, Events or
  // health change; the Unfence guard releases fenced GPUs.
  auto abandoned = [&](const char* phase) {
    if (!stop_.cancelled()) return false;
    LOG_WARN("node_agent") << "diagnostics pass abandoned " << phase << ": the agent is shutting down";
    return true;
  };
  if (abandoned("after the checks")) return false;
  // Phase 2: the node-level burn — every GPU under diagnosis at full MFMA load together.
  Value node = Value();
  std::vector<std::vector<std::string>> node_failures(todo.size());
  if (cfg_.diag_burn_ms > 0 && !todo.empty()) {
    NodeBurnResult nb = node_burn(*backend_, *engine_, gpus_, hip_devs_, todo, static_cast<int>(cfg_.diag_burn_ms), 0xb0c4,
                                  burn_dtype_code(cfg_.diag_burn_dtype));
    node_failures = judge_node_burn(nb, cfg_.diag_floors);
    for (size_t k = 0; k < todo.size(); ++k) results[todo[k]]["burn"] = nb.per_gpu[k];
    node = nb.node;
    if (abandoned("after the burn")) return false;
    auto& reg = metrics::Registry::global();
    reg.gauge("amd_gpu_diag_node_burn_power_watts", "Diagnostics: peak summed GPU power during the node-level burn")
        .set(node.get("power_sum_max_w").as_double());
    reg.gauge("amd_gpu_diag_node_burn_balance", "Diagnostics: slowest/fastest GPU burn rate under shared load")
        .set(node.get("balance").as_double());
    LOG_INFO("node_agent") << "node burn: " << todo.size() << " GPUs, peak " << node.get("power_sum_max_w").as_double()
                           << " W summed, peak hotspot " << node.get("peak_hotspot_c").as_double() << " C, balance "
                           << node.get("balance").as_double();
  }
  for (size_t k = 0; k < todo.size(); ++k) {
    const size_t i = todo[k];
    Value r = judge_diag(results[i], cfg_.diag_floors);
    if (!node_failures[k].empty()) {
      Value f = r.get("failures");
      for (const auto& s : node_failures[k]) f.push_back(s);
      r["failures"] = f;
      r["passed"] = false;
    }
    results[i] = std::move(r);
    record_diag_gauges(i, results[i]);
  }
  const double pass_ms = since(clock::now());
  bool changed = false;
  {
    std::lock_guard<std::mutex> lk(diag_mu_);
    Value per = Value::array();
    bool passed = true;
    for (size_t i = 0; i < gpus_.size(); ++i) {
      const bool was_bad = diag_failed(diag_, i);
      per.push_back(results[i]);
      const bool bad = results[i].is_object() && !results[i].get("passed").as_bool();
      changed = changed || (was_bad != bad);
      passed = passed && !bad;
    }
    diag_.ran = true;
    diag_.passed = passed;
    diag_.per_gpu = per;
    diag_.runs++;
    diag_.skipped_in_use += skipped;
    diag_.last_pass_ms = pass_ms;
    diag_.last_diagnosed = todo.size();
    if (!node.is_null()) diag_.node_burn = node;
  }
  if (fence) {  // verdicts first, so a failed GPU never flashes Healthy on release
    plugin_->set_health(healthy_flags());
    plugin_->set_fenced(todo, false);
    unfence.armed = false;
  }
  auto& reg = metrics::Registry::global();
  reg.counter("bgc_gpu_diag_runs_total", "Diagnostics passes").inc();
  reg.gauge("bgc_gpu_diag_pass_seconds", "Wall time of the last diagnostics pass").set(pass_ms / 1e3);
  if (skipped) reg.counter("bgc_gpu_diag_skipped_in_use_total", "GPUs skipped by a diagnostics pass because a container held them").inc(static_cast<double>(skipped));
  LOG_INFO("node_agent") << "diagnostics pass: " << todo.size() << " GPU(s) in " << pass_ms << " ms, " << skipped
                         << " skipped";
  return changed;
}

void NodeAgent::on_health_changed() {
  if (plugin_) plugin_->set_health(healthy_flags());
  emit_health_events();
  try {
    publish();
  } catch (const std::exception& e) {
    LOG_ERROR("node_agent") << "publish after health change failed: " << e.what();
  }
}

int NodeAgent::healthy_count(std::string* reason) const {
  auto snap = poller_ ? poller_->snapshot() : nullptr;
  std::lock_guard<std::mutex> lk(diag_mu_);
  int healthy = 0;
  std::string why;
  for (size_t i = 0; i < gpus_.size(); ++i) {
    bool ok = true;
    if (snap && i < snap->health.size()) {
      ok = snap->health[i].healthy;
      if (!ok) why += "gpu" + std::to_string(gpus_[i].index) + ": " + snap->health[i].reason + "; ";
    }
    if (diag_failed(diag_, i)) {
      ok = false;
      why += "gpu" + std::to_string(gpus_[i].index) + ": diagnostics failed " + diag_.per_gpu.items()[i].get("failures").dump() + "; ";
    }
    if (ok) ++healthy;
  }
  if (reason) *reason = why;
  return healthy;
}

void NodeAgent::publish() {
  std::lock_guard<std::mutex> lk(publish_mu_);
  if (!cfg_.create_node && !node_present_) return;  // the kubelet registers the Node, not us
  if (standing_down_) return;                        // another advertiser owns these fields
  std::string reason;
  int healthy = healthy_count(&reason);
  client_.apply(types::Node, "", cfg_.node_name, node_labels_patch(cfg_, gpus_, healthy, diag_outcome()), kNodeAgentManager,
                true);
  client_.apply_status(types::Node, "", cfg_.node_name, node_status_patch(cfg_, gpus_, healthy, reason),
                       kNodeAgentManager, true);
  publishes_.fetch_add(1);
  if (!cfg_.device_plugin) mark_advertised();  // capacity/allocatable is the advertisement
  LOG_INFO("node_agent") << "published node " << cfg_.node_name << ": " << cfg_.resource_name << " capacity "
                         << gpus_.size() << ", allocatable " << healthy;
}

// The plugin object exists from start() on (diagnostics fence it, health flips reach it);
// its server and kubelet registration start only while no other advertiser is found.
void NodeAgent::start_plugin() {
  std::lock_guard<std::mutex> lk(plugin_mu_);
  if (stop_.cancelled() || !plugin_ || plugin_started_.exchange(true)) return;
  plugin_->set_health(healthy_flags());
  plugin_->start();
  mark_advertised();  // ListAndWatch serves from here on
}

void NodeAgent::start() {
  if (cfg_.device_plugin) {
    DevicePluginConfig pc;
    pc.plugin_dir = cfg_.device_plugin_dir;
    pc.socket_name = cfg_.device_plugin_socket;
    pc.resource_name = cfg_.resource_name;
    pc.dev_root = cfg_.dev_root;
    pc.sysfs_root = cfg_.sysfs_root;
    pc.cdi = cfg_.device_plugin_cdi;
    pc.cdi_dir = cfg_.cdi_dir;
    plugin_ = std::make_unique<DevicePlugin>(gpus_, pc);
    plugin_->set_health(healthy_flags());
    if (!standing_down_) start_plugin();
  }
  poller_->on_health_change([this](const Snapshot&) { on_health_changed(); });
  poller_->start();
  emit_health_events();  // GPUs already unhealthy at start (pre-existing UEs, failed diagnostics)
  if (cfg_.run_diag && cfg_.diag_interval_secs > 0) {
    diag_thread_ = std::thread([this] {
      while (!stop_.wait_for(std::chrono::seconds(cfg_.diag_interval_secs))) {
        try {
          if (run_diagnostics(false)) on_health_changed();
        } catch (const std::exception& e) {
          LOG_ERROR("node_agent") << "periodic diagnostics failed: " << e.what();
        }
      }
    });
  }
  heartbeat_ = std::thread([this] {
    while (!stop_.wait_for(std::chrono::seconds(cfg_.heartbeat_secs))) {
      try {
        const bool was_down = standing_down_.load();
        const bool down = check_advertisers();
        if (down && !was_down && plugin_started_) {
          std::lock_guard<std::mutex> lk(plugin_mu_);
          if (!stop_.cancelled() && !plugin_stopped_.exchange(true)) {
            // found while advertising: unregister from the kubelet until the conflict clears
            plugin_->stop();
            LOG_ERROR("node_agent") << "device plugin stopped: another advertiser appeared; it starts again once "
                                    << "that advertiser is gone";
          }
        }
        if (!down && was_down) {
          bool restart = false;
          {
            std::lock_guard<std::mutex> lk(plugin_mu_);
            // re-checked under the lock: NodeAgent::stop() cancels stop_ while holding it
            if (!stop_.cancelled() && plugin_stopped_.exchange(false)) {
              plugin_->set_health(healthy_flags());
              plugin_->start();  // registers with the kubelet again
              restart = true;
            }
          }
          if (restart) {
            LOG_INFO("node_agent") << "device plugin restarted: the other advertiser is gone";
          } else {
            start_plugin();
          }
        }
        publish();
      } catch (const std::exception& e) {
        LOG_ERROR("node_agent") << "heartbeat publish failed: " << e.what();
      }
    }
  });
  node_watch_ = std::thread([this] {
    kube::Watcher w(client_, types::Node, "", "", "metadata.name=" + cfg_.node_name);
    auto consider = [this](const kube::ObjPtr& obj) {
      if (!obj) {
        node_present_ = false;
        if (!cfg_.create_node) {
          LOG_WARN("node_agent") << "node " << cfg_.node_name << " deleted; waiting for re-registration";
          return;
        }
        LOG_WARN("node_agent") << "node " << cfg_.node_name << " deleted; re-creating";
      } else {
        node_present_ = true;
        if (standing_down_) return;  // the heartbeat re-checks the other advertiser
        if (node_up_to_date(*obj)) return;
        LOG_INFO("node_agent") << "node " << cfg_.node_name << " (re)registered or drifted; re-publishing";
        // drift may be another manager writing the same labels: look before forcing ours back
        check_advertisers();
      }
      // A failed publish (e.g. the first request on a path that was just found dead) is
      // retried a few times rather than left to the next heartbeat.
      for (int attempt = 0;; ++attempt) {
        try {
          publish();
          break;
        } catch (const std::exception& e) {
          LOG_ERROR("node_agent") << "publish after node change failed: " << e.what();
          if (attempt == 3 || stop_.wait_for(std::chrono::milliseconds(200 << attempt))) break;
        }
      }
    };
    w.run(stop_, [&](const kube::WatchEvent& ev) {
      switch (ev.type) {
        case kube::WatchEvent::Type::Restarted:
          consider(ev.objects.empty() ? nullptr : ev.objects.front());
          break;
        case kube::WatchEvent::Type::Deleted:
          consider(nullptr);
          break;
        default:
          consider(ev.object);
      }
    });
  });
}

void NodeAgent::stop() {
  {
    // under plugin_mu_: a heartbeat between its stop_ check and plugin_->start() would
    // otherwise re-register the plugin with the kubelet during shutdown
    std::lock_guard<std::mutex> lk(plugin_mu_);
    stop_.cancel();
  }
  if (!pcie_lock_path_.empty()) ::unlink(pcie_lock_path_.c_str());
  // the device plugin first (unregistered, socket removed), the telemetry poller last: a
  // poll stuck in amdsmi must not keep the kubelet allocating from a stopping agent
  if (plugin_) {
    std::lock_guard<std::mutex> lk(plugin_mu_);
    plugin_->stop();
  }
  if (heartbeat_.joinable()) heartbeat_.join();
  if (diag_thread_.joinable()) diag_thread_.join();
  if (node_watch_.joinable()) node_watch_.join();
  if (poller_) poller_->stop();
}

Value NodeAgent::describe() const {
  Value gpus = Value::array();
  for (const auto& g : gpus_) gpus.push_back(to_json(g));
  Value out = Value::object({{"node", cfg_.node_name}, {"backend", backend_->name()}, {"gpus", gpus}});
  if (poller_) {
    auto snap = poller_->snapshot();
    Value tel = Value::array();
    for (const auto& t : snap->devices) tel.push_back(to_json(t));
    out["telemetry"] = tel;
    out["poll_us"] = snap->poll_us;
    out["polls"] = static_cast<unsigned long long>(poller_->polls());
    out["telemetry_stalled"] = snap->stalled;
  }
  std::string reason;
  out["healthy"] = healthy_count(&reason);
  out["unhealthy_reason"] = reason;
  DiagOutcome d = diag_outcome();
  out["diag"] = d.per_gpu;
  out["diag_runs"] = static_cast<unsigned long long>(d.runs);
  out["diag_skipped_in_use"] = static_cast<unsigned long long>(d.skipped_in_use);
  out["diag_last_pass_ms"] = d.last_pass_ms;
  out["diag_last_diagnosed"] = static_cast<unsigned long long>(d.last_diagnosed);
  out["diag_node_burn"] = d.node_burn;
  out["diag_fence_races"] = static_cast<unsigned long long>(fence_races_.load());
  Value procs = Value::array();  // what the driver lists on each GPU (why a pass skipped it)
  for (const auto& g : gpus_) procs.push_back(backend_->processes(g.index));
  out["processes"] = procs;
  out["diag_engine"] = engine_ ? Value(engine_->name()) : Value();
  out["diag_isolation"] = !engine_ ? Value() : Value(engine_->name() != "hip" ? "none" : diag_in_process_ ? "in-process" : "worker-process");
  Value hd = Value::array();
  for (int h : hip_devs_) hd.push_back(h);
  out["hip_devices"] = hd;
  out["startup_ms"] = Value::object({{"discover", discover_ms_},
                                     {"diagnostics", startup_diag_ms_},
                                     {"first_advertise", first_advertise_ms_.load()}});
  if (plugin_) out["device_plugin"] = plugin_->describe();
  out["advertiser"] = Value::object({{"standing_down", standing_down_.load()},
                                     {"take_over", cfg_.take_over},
                                     {"check", cfg_.advertiser_check},
                                     {"plugin_started", plugin_started_.load()},
                                     {"plugin_stopped", plugin_stopped_.load()},
                                     {"conflicts", advertiser_conflicts()}});
  return out;
}

}  // namespace bgc::gpu

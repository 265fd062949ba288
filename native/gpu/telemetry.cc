#include "gpu/telemetry.h"

#include <future>

#include "core/log.h"
#include "core/metrics.h"
#include "core/roctx.h"

namespace bgc::gpu {

TelemetryPoller::TelemetryPoller(Backend& backend, std::vector<int> indices, std::chrono::milliseconds interval,
                                 HealthPolicy policy, int slow_every)
    : backend_(backend), indices_(std::move(indices)), interval_(interval), policy_(policy),
      slow_every_(std::max(1, slow_every)) {
  for (int i : indices_) {
    DeviceHealth h;
    h.index = i;
    health_.push_back(h);
  }
  slow_cache_.resize(indices_.size());
  if (indices_.size() > 1) pool_ = std::make_unique<ThreadPool>(indices_.size());
  auto& reg = metrics::Registry::global();
  for (int i : indices_) {
    metrics::Labels l{{"gpu", std::to_string(i)}};
    gauges_.push_back({&reg.gauge("amd_gpu_gfx_activity_percent", "GFX engine activity", l),
                       &reg.gauge("amd_gpu_umc_activity_percent", "Memory controller activity", l),
                       &reg.gauge("amd_gpu_power_watts", "Socket power", l),
                       &reg.gauge("amd_gpu_temperature_hotspot_celsius", "Hotspot temperature", l),
                       &reg.gauge("amd_gpu_temperature_mem_celsius", "HBM temperature", l),
                       &reg.gauge("amd_gpu_vram_used_bytes", "VRAM in use", l),
                       &reg.gauge("amd_gpu_vram_total_bytes", "VRAM capacity", l),
                       &reg.gauge("amd_gpu_gfxclk_mhz", "GFX clock", l),
                       &reg.gauge("amd_gpu_ecc_uncorrectable_total", "Uncorrectable ECC errors", l),
                       &reg.gauge("amd_gpu_xgmi_links_up", "xGMI links up", l),
                       &reg.gauge("amd_gpu_healthy", "1 when the device passes the health policy", l)});
  }
  snap_ = std::make_shared<Snapshot>();
}

TelemetryPoller::~TelemetryPoller() { stop(); }

void TelemetryPoller::on_health_change(std::function<void(const Snapshot&)> cb) { cb_ = std::move(cb); }

std::shared_ptr<const Snapshot> TelemetryPoller::snapshot() const {
  std::lock_guard<std::mutex> lk(snap_mu_);
  return snap_;
}

void TelemetryPoller::evaluate(const Telemetry& t, const HealthPolicy& p, DeviceHealth& h) {
  std::string problem;
  if (!t.ok) {
    problem = "telemetry unavailable: " + t.error;
  } else {
    if (!h.baseline_set) {
      h.baseline_uncorrectable = t.ecc_uncorrectable;
      h.baseline_set = true;
    }
    if (t.temp_hotspot_c > p.max_hotspot_c) problem = "hotspot temperature " + std::to_string(t.temp_hotspot_c) + "C";
    else if (t.temp_mem_c > p.max_mem_c) problem = "HBM temperature " + std::to_string(t.temp_mem_c) + "C";
    else if (t.ecc_uncorrectable > h.baseline_uncorrectable + p.max_new_uncorrectable) {
      problem = "uncorrectable ECC errors: " + std::to_string(t.ecc_uncorrectable - h.baseline_uncorrectable);
    } else if (p.require_all_xgmi_links && t.xgmi_links_total > 0 && t.xgmi_links_up < t.xgmi_links_total) {
      problem = "xGMI links down: " + std::to_string(t.xgmi_links_total - t.xgmi_links_up) + "/" +
                std::to_string(t.xgmi_links_total);
    }
  }
  if (problem.empty()) {
    h.consecutive_bad = 0;
    ++h.consecutive_good;
    if (!h.healthy && h.consecutive_good >= p.recover_threshold) {
      h.healthy = true;
      h.reason.clear();
    }
  } else {
    h.consecutive_good = 0;
    ++h.consecutive_bad;
    if (h.healthy && h.consecutive_bad >= p.fail_threshold) h.healthy = false;
    if (!h.healthy) h.reason = problem;
  }
}

void TelemetryPoller::poll_once() {
  roctx::Range range("bgc.telemetry.poll");
  auto& reg = metrics::Registry::global();
  static auto& poll_hist = reg.histogram("bgc_telemetry_poll_seconds", "Wall time of one telemetry poll over all devices");
  static auto& poll_ring = reg.samples("telemetry_poll");
  int64_t t0 = metrics::now_ns();
  auto snap = std::make_shared<Snapshot>();
  snap->devices.reserve(indices_.size());
  bool changed = false;
  const bool full = polls_.load() % static_cast<uint64_t>(slow_every_) == 0;
  std::vector<Telemetry> samples(indices_.size());
  if (pool_) {
    std::vector<std::future<void>> futs;
    for (size_t k = 0; k < indices_.size(); ++k) {
      futs.push_back(pool_->submit([&, k] { samples[k] = backend_.sample(indices_[k], full); }));
    }
    for (auto& f : futs) f.get();
  } else {
    for (size_t k = 0; k < indices_.size(); ++k) samples[k] = backend_.sample(indices_[k], full);
  }
  for (size_t k = 0; k < indices_.size(); ++k) {
    Telemetry t = std::move(samples[k]);
    if (full) {
      slow_cache_[k] = t;
    } else if (t.ok) {
      t.ecc_correctable = slow_cache_[k].ecc_correctable;
      t.ecc_uncorrectable = slow_cache_[k].ecc_uncorrectable;
      t.vram_used_mb = slow_cache_[k].vram_used_mb;
      t.vram_total_mb = slow_cache_[k].vram_total_mb;
    }
    bool was = health_[k].healthy;
    evaluate(t, policy_, health_[k]);
    if (was != health_[k].healthy) {
      changed = true;
      if (health_[k].healthy) {
        LOG_INFO("gpu") << "gpu " << indices_[k] << " recovered";
      } else {
        LOG_WARN("gpu") << "gpu " << indices_[k] << " unhealthy: " << health_[k].reason;
      }
    }
    const Gauges& g = gauges_[k];
    g.gfx->set(t.gfx_activity_pct);
    g.umc->set(t.umc_activity_pct);
    g.power->set(t.power_w);
    g.hotspot->set(t.temp_hotspot_c);
    g.mem_temp->set(t.temp_mem_c);
    g.vram_used->set(static_cast<double>(t.vram_used_mb) * 1048576.0);
    g.vram_total->set(static_cast<double>(t.vram_total_mb) * 1048576.0);
    g.gfxclk->set(t.gfxclk_mhz);
    g.ecc_ue->set(static_cast<double>(t.ecc_uncorrectable));
    g.xgmi_up->set(t.xgmi_links_up);
    g.healthy->set(health_[k].healthy ? 1 : 0);
    snap->devices.push_back(std::move(t));
  }
  snap->health = health_;
  snap->ts_ns = metrics::now_ns();
  snap->poll_us = static_cast<double>(snap->ts_ns - t0) / 1e3;
  snap->poll_seq = polls_.fetch_add(1) + 1;
  poll_hist.observe(snap->poll_us * 1e-6);
  poll_ring.add(snap->poll_us * 1e-6);
  {
    std::lock_guard<std::mutex> lk(snap_mu_);
    snap_ = snap;
  }
  if (changed && cb_) cb_(*snap);
}

void TelemetryPoller::start() {
  if (thread_.joinable()) return;
  thread_ = std::thread([this] {
    while (!stop_.cancelled()) {
      try {
        poll_once();
      } catch (const std::exception& e) {
        LOG_ERROR("gpu") << "telemetry poll failed: " << e.what();
      }
      if (stop_.wait_for(interval_)) break;
    }
  });
}

void TelemetryPoller::stop() {
  stop_.cancel();
  if (thread_.joinable()) thread_.join();
}

}  // namespace bgc::gpu

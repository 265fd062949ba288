#include "gpu/telemetry.h"

#include <algorithm>
#include <future>

#include "core/log.h"
#include "core/metrics.h"
#include "core/roctx.h"
#include "core/process.h"
#include "core/schedstat.h"

namespace bgc::gpu {

TelemetryPoller::TelemetryPoller(Backend& backend, std::vector<int> indices, std::chrono::milliseconds interval,
                                 HealthPolicy policy, int slow_every, int ras_every, std::vector<uint64_t> page_limits)
    : backend_(backend), indices_(std::move(indices)), interval_(interval), policy_(policy),
      slow_every_(std::max(1, slow_every)), ras_every_(std::max(1, ras_every)) {
  for (size_t k = 0; k < indices_.size(); ++k) {
    DeviceHealth h;
    h.index = indices_[k];
    h.page_limit = policy_.max_retired_pages;
    if (k < page_limits.size() && page_limits[k] > 0) h.page_limit = std::min(h.page_limit, page_limits[k]);
    health_.push_back(h);
  }
  slow_cache_.resize(indices_.size());
  ras_cache_.resize(indices_.size());
  prev_.resize(indices_.size());
  if (indices_.size() > 1) pool_ = std::make_unique<ThreadPool>(indices_.size(), "telemetry-dev");
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
                       &reg.gauge("amd_gpu_healthy", "1 when the device passes the health policy", l),
                       &reg.gauge("amd_gpu_violation_ppt_percent", "Power-cap (PPT) throttle residency, last interval", l),
                       &reg.gauge("amd_gpu_violation_thermal_percent", "Thermal throttle residency, last interval", l),
                       &reg.gauge("amd_gpu_retired_pages", "Retired + pending HBM pages", l),
                       &reg.gauge("amd_gpu_throttle_status", "Independent throttle status bits (-1 = not reported)", l),
                       &reg.gauge("amd_gpu_pcie_link_width", "PCIe link width (lanes)", l),
                       &reg.gauge("amd_gpu_pcie_link_speed_mts", "PCIe link rate per lane (MT/s)", l),
                       &reg.gauge("amd_gpu_pcie_replays_total", "PCIe replays since boot", l)});
  }
  snap_ = std::make_shared<Snapshot>();
  // exported from the start (0), so a dashboard or alert sees the series before any stall
  reg.gauge("bgc_telemetry_stalled", "1 while a telemetry poll has been stuck past the stall timeout");
}

TelemetryPoller::~TelemetryPoller() { stop(); }

void TelemetryPoller::on_health_change(std::function<void(const Snapshot&)> cb) { cb_ = std::move(cb); }

std::shared_ptr<const Snapshot> TelemetryPoller::snapshot() const {
  std::lock_guard<std::mutex> lk(snap_mu_);
  return snap_;
}

void TelemetryPoller::violation_deltas(const Telemetry& prev, Telemetry& cur) {
  cur.violation_ppt_pct = cur.violation_thermal_pct = -1;
  if (cur.acc_counter == Telemetry::kNoAcc || prev.acc_counter == Telemetry::kNoAcc) return;
  if (cur.acc_counter <= prev.acc_counter) return;  // no new accumulation cycle (or a reset)
  const double span = static_cast<double>(cur.acc_counter - prev.acc_counter);
  auto pct = [&](uint64_t a, uint64_t b) -> double {
    if (a == Telemetry::kNoAcc || b == Telemetry::kNoAcc || a < b) return -1;
    return std::min(100.0, 100.0 * static_cast<double>(a - b) / span);
  };
  cur.violation_ppt_pct = pct(cur.acc_ppt, prev.acc_ppt);
  cur.violation_thermal_pct = pct(cur.acc_thermal, prev.acc_thermal);
}

void TelemetryPoller::evaluate(const Telemetry& t, const HealthPolicy& p, DeviceHealth& h) {
  std::string problem;
  if (t.ras_ok) {
    h.retired_pages = t.retired_pages;
    h.unreservable_pages = t.unreservable_pages;
  }
  if (h.page_limit == 0) h.page_limit = p.max_retired_pages;
  if (!t.ok) {
    problem = "telemetry unavailable: " + t.error;
  } else {
    if (!h.baseline_set) {
      h.baseline_uncorrectable = t.ecc_uncorrectable;
      h.baseline_set = true;
    }
    if (t.pcie_replays >= 0) {  // fresh only on slow polls: the verdict holds until the next one
      h.pcie_replay_delta = h.pcie_last_replays >= 0 && t.pcie_replays >= h.pcie_last_replays
                                ? t.pcie_replays - h.pcie_last_replays
                                : 0;
      h.pcie_last_replays = t.pcie_replays;
    }
    h.consecutive_thermal = t.violation_thermal_pct > p.max_thermal_violation_pct ? h.consecutive_thermal + 1 : 0;
    h.consecutive_ppt = t.violation_ppt_pct > p.max_ppt_violation_pct ? h.consecutive_ppt + 1 : 0;
    if (t.temp_hotspot_c > p.max_hotspot_c) problem = "hotspot temperature " + std::to_string(t.temp_hotspot_c) + "C";
    else if (t.temp_mem_c > p.max_mem_c) problem = "HBM temperature " + std::to_string(t.temp_mem_c) + "C";
    else if (h.baseline_uncorrectable > p.max_uncorrectable_at_start && t.ecc_uncorrectable >= h.baseline_uncorrectable) {
      problem = std::to_string(h.baseline_uncorrectable) + " uncorrectable ECC errors already present at agent start";
    } else if (t.ecc_uncorrectable > h.baseline_uncorrectable + p.max_new_uncorrectable) {
      problem = "uncorrectable ECC errors: " + std::to_string(t.ecc_uncorrectable - h.baseline_uncorrectable);
    } else if (h.unreservable_pages > 0) {
      problem = std::to_string(h.unreservable_pages) + " bad HBM pages could not be retired";
    } else if (h.retired_pages > h.page_limit) {
      problem = "retired HBM pages " + std::to_string(h.retired_pages) + " > " + std::to_string(h.page_limit);
    } else if (p.require_all_xgmi_links && t.xgmi_links_total > 0 && t.xgmi_links_up < t.xgmi_links_total) {
      problem = "xGMI links down: " + std::to_string(t.xgmi_links_total - t.xgmi_links_up) + "/" +
                std::to_string(t.xgmi_links_total);
    } else if (h.consecutive_thermal >= p.violation_sustain_polls) {
      problem = "sustained thermal throttling: " + std::to_string(static_cast<int>(t.violation_thermal_pct)) + "% for " +
                std::to_string(h.consecutive_thermal) + " polls";
    } else if (h.consecutive_ppt >= p.violation_sustain_polls) {
      problem = "sustained power-cap throttling: " + std::to_string(static_cast<int>(t.violation_ppt_pct)) + "% for " +
                std::to_string(h.consecutive_ppt) + " polls";
    } else if (p.require_full_pcie_width && h.pcie_max_width > 0 && t.pcie_width > 0 && t.pcie_width < h.pcie_max_width) {
      problem = "PCIe link x" + std::to_string(t.pcie_width) + " of x" + std::to_string(h.pcie_max_width);
    } else if (p.max_pcie_replays_per_poll >= 0 && h.pcie_replay_delta > p.max_pcie_replays_per_poll) {
      problem = "PCIe link replays: " + std::to_string(h.pcie_replay_delta) + " since the previous slow poll";
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
  auto& reg = metrics::Registry::global();
  static auto& poll_hist = reg.histogram("bgc_telemetry_poll_seconds", "Wall time of one telemetry poll over all devices");
  static auto& poll_ring = reg.samples("telemetry_poll");
  int64_t t0 = metrics::now_ns();
  poll_started_ns_.store(t0);
  // a poll that throws has not stalled: the watchdog only watches polls in progress
  struct Finished {
    std::atomic<int64_t>& started;
    ~Finished() { started.store(0); }
  } finished{poll_started_ns_};
  auto snap = std::make_shared<Snapshot>();
  snap->devices.reserve(indices_.size());
  bool changed = false;
  const uint64_t seq = polls_.load();
  const SampleLevel level = seq % static_cast<uint64_t>(ras_every_) == 0    ? SampleLevel::Ras
                            : seq % static_cast<uint64_t>(slow_every_) == 0 ? SampleLevel::Slow
                                                                            : SampleLevel::Fast;
  const bool full = level >= SampleLevel::Slow;
  // one roctx range per poll, named by cadence, so rocprofv3 --marker-trace separates the
  // every-poll cost from the slow-counter polls
  roctx::Range range(level == SampleLevel::Ras    ? "bgc.telemetry.poll.ras"
                     : level == SampleLevel::Slow ? "bgc.telemetry.poll.slow"
                                                  : "bgc.telemetry.poll.fast");
  std::vector<Telemetry> samples(indices_.size());
  // The poll's wall time split into on-CPU, run-queue wait and blocked (amdsmi's ioctls
  // waiting on the SMU): on a saturated CPU share the first two grow, on a busy SMU the
  // third.  With a pool, each device's task is measured on its own thread and the slowest
  // device's split is added to the polling thread's.
  const sched::ThreadSched s0 = sched::thread_sched();
  int64_t dev_cpu = 0, dev_runq = 0;
  if (pool_) {
    std::vector<std::future<std::pair<int64_t, int64_t>>> futs;
    for (size_t k = 0; k < indices_.size(); ++k) {
      futs.push_back(pool_->submit([&, k] {
        const sched::ThreadSched a = sched::thread_sched();
        samples[k] = backend_.sample(indices_[k], level);
        const sched::ThreadSched b = sched::thread_sched();
        return a.ok() && b.ok() ? std::make_pair(b.cpu_ns - a.cpu_ns, b.runq_ns - a.runq_ns) : std::make_pair(int64_t{0}, int64_t{0});
      }));
    }
    for (auto& f : futs) {
      const auto [c, q] = f.get();
      dev_cpu = std::max(dev_cpu, c);
      dev_runq = std::max(dev_runq, q);
    }
  } else {
    for (size_t k = 0; k < indices_.size(); ++k) samples[k] = backend_.sample(indices_[k], level);
  }
  const sched::ThreadSched s1 = sched::thread_sched();
  if (s0.ok() && s1.ok()) {
    static auto& cpu_ring = reg.samples("telemetry_poll_cpu");
    static auto& runq_ring = reg.samples("telemetry_poll_runq");
    static auto& runq_hist = reg.histogram("bgc_telemetry_poll_runq_seconds",
                                           "Run-queue wait (runnable, no CPU) inside one telemetry poll");
    const double runq = static_cast<double>(s1.runq_ns - s0.runq_ns + dev_runq) * 1e-9;
    cpu_ring.add(static_cast<double>(s1.cpu_ns - s0.cpu_ns + dev_cpu) * 1e-9);
    runq_ring.add(runq);
    runq_hist.observe(runq);
  }
  for (size_t k = 0; k < indices_.size(); ++k) {
    Telemetry t = std::move(samples[k]);
    if (full) {
      slow_cache_[k] = t;
    } else if (t.ok) {
      t.ecc_correctable = slow_cache_[k].ecc_correctable;
      t.ecc_uncorrectable = slow_cache_[k].ecc_uncorrectable;
      t.ecc_deferred = slow_cache_[k].ecc_deferred;
      t.vram_used_mb = slow_cache_[k].vram_used_mb;
      t.vram_total_mb = slow_cache_[k].vram_total_mb;
      t.pcie_width = slow_cache_[k].pcie_width;
      t.pcie_speed_mts = slow_cache_[k].pcie_speed_mts;
      // the error counters stay -1 on fast polls: evaluate() diffs fresh readings only
    }
    if (level == SampleLevel::Ras) {
      ras_cache_[k] = t;
    } else if (t.ok && ras_cache_[k].ras_ok) {
      t.ras_ok = true;
      t.retired_pages = ras_cache_[k].retired_pages;
      t.unreservable_pages = ras_cache_[k].unreservable_pages;
      t.ecc_blocks = ras_cache_[k].ecc_blocks;
      t.links = ras_cache_[k].links;
    }
    if (t.ok) {
      violation_deltas(prev_[k], t);
      prev_[k].acc_counter = t.acc_counter;
      prev_[k].acc_ppt = t.acc_ppt;
      prev_[k].acc_thermal = t.acc_thermal;
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
    g.viol_ppt->set(t.violation_ppt_pct);
    g.viol_thermal->set(t.violation_thermal_pct);
    g.retired->set(static_cast<double>(health_[k].retired_pages));
    g.throttle->set(t.throttle_valid ? static_cast<double>(t.throttle_status) : -1.0);
    g.pcie_width->set(t.pcie_width);
    g.pcie_speed->set(t.pcie_speed_mts);
    if (t.pcie_replays >= 0) g.pcie_replays->set(static_cast<double>(t.pcie_replays));
    snap->devices.push_back(std::move(t));
  }
  snap->health = health_;
  snap->ts_ns = metrics::now_ns();
  snap->poll_us = static_cast<double>(snap->ts_ns - t0) / 1e3;
  snap->poll_seq = polls_.fetch_add(1) + 1;
  poll_hist.observe(snap->poll_us * 1e-6);
  poll_ring.add(snap->poll_us * 1e-6);
  bool resumed = false;
  {
    std::lock_guard<std::mutex> sl(stall_mu_);
    poll_started_ns_.store(0);
    // A stall ends with a poll that completes inside the stall timeout: one that itself took
    // longer (an amdsmi that answers, but only after the timeout) keeps the GPUs withdrawn,
    // so a slow backend does not flap them every poll.
    const double took_s = static_cast<double>(snap->ts_ns - t0) / 1e9;
    if (stalled_.load() && stall_timeout_.count() > 0 && took_s * 1e3 >= static_cast<double>(stall_timeout_.count())) {
      mark_stalled(*snap, took_s);
      changed = false;
    } else {
      resumed = stalled_.exchange(false);
    }
    std::lock_guard<std::mutex> lk(snap_mu_);
    snap_ = snap;
  }
  if (resumed) {
    reg.gauge("bgc_telemetry_stalled", "1 while a telemetry poll has been stuck past the stall timeout").set(0);
    LOG_WARN("gpu") << "telemetry polls resumed; device health is read from telemetry again";
  }
  if (changed || resumed) notify(*snap);
}

void TelemetryPoller::notify(const Snapshot& s) {
  std::lock_guard<std::mutex> lk(cb_mu_);
  if (cb_) cb_(s);
}

void TelemetryPoller::mark_stalled(Snapshot& snap, double stuck_s) const {
  snap.stalled = true;
  for (size_t k = snap.health.size(); k < indices_.size(); ++k) {
    DeviceHealth h;
    h.index = indices_[k];
    snap.health.push_back(h);
  }
  const std::string why = "telemetry stalled: no reading from the " + backend_.name() + " backend for " +
                          std::to_string(static_cast<long long>(stuck_s)) + " s";
  for (auto& h : snap.health) {
    h.healthy = false;
    h.reason = why;
  }
  for (const auto& g : gauges_) g.healthy->set(0);
}

void TelemetryPoller::check_stall() {
  std::shared_ptr<Snapshot> snap;
  double stuck_s = 0;
  {
    std::lock_guard<std::mutex> sl(stall_mu_);
    const int64_t started = poll_started_ns_.load();
    if (started == 0 || stalled_.load()) return;
    stuck_s = static_cast<double>(metrics::now_ns() - started) / 1e9;
    if (stuck_s * 1e3 < static_cast<double>(stall_timeout_.count())) return;
    snap = std::make_shared<Snapshot>(*snapshot());
    mark_stalled(*snap, stuck_s);
    stalled_.store(true);
    std::lock_guard<std::mutex> lk(snap_mu_);
    snap_ = snap;
  }
  auto& reg = metrics::Registry::global();
  reg.gauge("bgc_telemetry_stalled", "1 while a telemetry poll has been stuck past the stall timeout").set(1);
  reg.counter("bgc_telemetry_stalls_total", "Telemetry polls that got stuck past the stall timeout").inc();
  LOG_ERROR("gpu") << "telemetry poll stuck for " << stuck_s << " s in the " << backend_.name()
                   << " backend: advertising every GPU unhealthy until a poll completes";
  notify(*snap);
}

void TelemetryPoller::start() {
  if (thread_.joinable()) return;
  thread_ = std::thread([this] {
    set_thread_name("telemetry");
    while (!stop_.cancelled()) {
      try {
        poll_once();
      } catch (const std::exception& e) {
        LOG_ERROR("gpu") << "telemetry poll failed: " << e.what();
      }
      if (stop_.wait_for(interval_)) break;
    }
  });
  if (stall_timeout_.count() > 0) {
    const auto tick = std::clamp(stall_timeout_ / 4, std::chrono::milliseconds(10), std::chrono::milliseconds(1000));
    watchdog_ = std::thread([this, tick] {
      set_thread_name("telemetry-dog");
      while (!stop_.wait_for(tick)) check_stall();
    });
  }
}

void TelemetryPoller::stop() {
  stop_.cancel();
  if (watchdog_.joinable()) watchdog_.join();
  if (thread_.joinable()) thread_.join();
}

}  // namespace bgc::gpu

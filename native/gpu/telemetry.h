// Side-thread telemetry poller + health evaluation (north-star N2).
//
// One background thread samples every managed device each `interval` (amdsmi
// gpu_metrics: activity, power, temperatures, clocks, throttle, violation residency, xGMI
// link status; every Nth poll VRAM usage and ECC totals; every Mth poll retired pages,
// per-block ECC and xGMI link traffic), publishes an immutable snapshot (readers never block the poll),
// exports `amd_gpu_*` Prometheus gauges, and drives a per-device health state machine
// with hysteresis.  Each poll is bracketed by a roctx range so rocprofv3 --marker-trace
// shows its cost; the reconcile/admission paths never touch it.
#pragma once

#include <atomic>
#include <chrono>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "core/cancel.h"
#include "core/metrics.h"
#include "core/threadpool.h"
#include "gpu/device.h"

namespace bgc::gpu {

struct HealthPolicy {
  double max_hotspot_c = 105.0;      // above -> unhealthy
  double max_mem_c = 95.0;
  uint64_t max_new_uncorrectable = 0;  // new uncorrectable ECC errors tolerated since start
  // Uncorrectable errors already counted when the agent starts (the counters reset on
  // driver load, so these happened during this boot): more than this -> unhealthy.
  uint64_t max_uncorrectable_at_start = 0;
  bool require_all_xgmi_links = true;  // a down xGMI link breaks TP=8 all-reduce placement
  // Retired (reserved + pending) HBM pages above this -> unhealthy; the driver's own
  // bad-page threshold, when readable, caps it.  Any page the driver could not retire
  // (unreservable) is always unhealthy.
  uint64_t max_retired_pages = 64;
  // Sustained throttling: thermal (socket/HBM/VR/PROCHOT) residency above this
  // percentage for `violation_sustain_polls` consecutive polls -> unhealthy.  Power
  // (PPT) capping is normal for an MI355X at full load, so it is off by default (>100).
  double max_thermal_violation_pct = 20.0;
  double max_ppt_violation_pct = 101.0;
  int violation_sustain_polls = 30;
  // PCIe: the link must run at its full width (a link that trained x8 on an x16 slot
  // halves host bandwidth), and more than this many replays between two slow polls
  // (a marginal link retrying packets) is a fault until a later slow poll is clean.
  bool require_full_pcie_width = true;
  int64_t max_pcie_replays_per_poll = 100;
  int fail_threshold = 3;              // consecutive bad polls before flipping to unhealthy
  int recover_threshold = 3;           // consecutive good polls before flipping back
};

struct DeviceHealth {
  int index = 0;
  bool healthy = true;
  std::string reason;
  int consecutive_bad = 0;
  int consecutive_good = 0;
  uint64_t baseline_uncorrectable = 0;
  bool baseline_set = false;
  int consecutive_thermal = 0;  // polls in a row over the thermal violation limit
  int consecutive_ppt = 0;
  uint64_t retired_pages = 0;   // last RAS reading (cached between RAS polls)
  uint64_t unreservable_pages = 0;
  uint64_t page_limit = 0;      // effective retired-page limit (policy, capped by driver)
  int pcie_max_width = -1;      // from discovery (-1 = unknown: width rule off)
  int64_t pcie_last_replays = -1;
  int64_t pcie_replay_delta = 0;  // over the last slow-poll interval
};

struct Snapshot {
  int64_t ts_ns = 0;
  uint64_t poll_seq = 0;
  double poll_us = 0;  // wall time of the whole poll
  std::vector<Telemetry> devices;
  std::vector<DeviceHealth> health;
  // Published by the stall watchdog: a poll has been stuck in the backend for longer than
  // the stall timeout, so every device reads unhealthy until a poll completes again.
  bool stalled = false;
};

class TelemetryPoller {
 public:
  // slow_every: the expensive counters (ECC totals, VRAM usage) are read every Nth poll
  // and cached in between; devices are sampled concurrently (one task per GPU), so a
  // poll over 8 MI355X costs about one device's latency, not eight.
  // ras_every: bad pages, per-block ECC and xGMI link metrics are read every Nth poll.
  // page_limits[k] (optional): the driver's bad-page threshold of device k.
  TelemetryPoller(Backend& backend, std::vector<int> indices, std::chrono::milliseconds interval,
                  HealthPolicy policy = {}, int slow_every = 10, int ras_every = 60,
                  std::vector<uint64_t> page_limits = {});
  ~TelemetryPoller();
  // Link capability of device k (GpuInfo::pcie_max_width), for the PCIe width rule;
  // call before start().
  void set_pcie_max_width(size_t k, int width) {
    if (k < health_.size()) health_[k].pcie_max_width = width;
  }
  // A poll stuck in the backend (amdsmi blocks while the driver resets a wedged GPU)
  // longer than this publishes every device unhealthy until a poll completes (0 = off).
  // Call before start().
  void set_stall_timeout(std::chrono::milliseconds t) { stall_timeout_ = t; }
  void start();
  void stop();
  // Runs one poll synchronously (tests, and the first poll before start()).
  void poll_once();
  std::shared_ptr<const Snapshot> snapshot() const;
  // Invoked (on the poller thread) whenever any device's health flips.
  void on_health_change(std::function<void(const Snapshot&)> cb);
  uint64_t polls() const { return polls_.load(); }
  bool stalled() const { return stalled_.load(); }

  // Pure health step (exposed for tests).
  static void evaluate(const Telemetry& t, const HealthPolicy& p, DeviceHealth& h);
  // Violation percentages of `cur` over the interval since `prev` (pure, exposed for tests).
  static void violation_deltas(const Telemetry& prev, Telemetry& cur);
  const HealthPolicy& policy() const { return policy_; }

 private:
  Backend& backend_;
  std::vector<int> indices_;
  std::chrono::milliseconds interval_;
  HealthPolicy policy_;
  std::vector<DeviceHealth> health_;
  int slow_every_;
  int ras_every_;
  std::vector<Telemetry> slow_cache_;
  std::vector<Telemetry> ras_cache_;
  std::vector<Telemetry> prev_;  // last sample per device (violation deltas)
  std::unique_ptr<ThreadPool> pool_;
  struct Gauges {
    metrics::Gauge *gfx, *umc, *power, *hotspot, *mem_temp, *vram_used, *vram_total, *gfxclk, *ecc_ue, *xgmi_up, *healthy,
        *viol_ppt, *viol_thermal, *retired, *throttle, *pcie_width, *pcie_speed, *pcie_replays;
  };
  std::vector<Gauges> gauges_;  // resolved once: the poll path does no registry lookups
  mutable std::mutex snap_mu_;
  std::shared_ptr<const Snapshot> snap_;
  std::function<void(const Snapshot&)> cb_;
  std::mutex cb_mu_;  // the poll thread and the watchdog both report changes
  std::atomic<uint64_t> polls_{0};
  // Stall watchdog: poll_started_ns_ is the start of the poll in progress (0 = none);
  // stall_mu_ orders "the poll finished" against "the watchdog declared it stalled".
  std::chrono::milliseconds stall_timeout_{0};
  std::mutex stall_mu_;
  std::atomic<int64_t> poll_started_ns_{0};
  std::atomic<bool> stalled_{false};
  void check_stall();
  void mark_stalled(Snapshot& snap, double stuck_s) const;
  void notify(const Snapshot& s);
  CancelToken stop_;
  std::thread thread_;
  std::thread watchdog_;
};

}  // namespace bgc::gpu

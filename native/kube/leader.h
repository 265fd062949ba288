// Lease-based leader election (coordination.k8s.io/v1).  The reference's chart already
// grants the controller `leases` get/create/update/patch (reference
// charts/.../templates/serviceaccount.yaml:26-28) but never uses it, so two controller
// replicas double-write; CONF_LEADER_ELECTION=true enables this.
//
// Timing follows client-go's leaderelection: a lease lasts `lease_seconds` (15), the
// holder renews every `retry_seconds` (2) and steps down once no renew has succeeded
// within `renew_deadline_seconds` (10) of the last successful renew's *send* time, so it
// stops acting before a standby (which waits the full lease duration by its own clock)
// can take over.  It also steps down at once when the lease names another holder.
// The deadline holds even while a renew request hangs: Lease calls go through their own
// client (request timeout renew_deadline - retry_period, no 429 retries), and a watchdog
// thread cancels the guarded work at last_ok_sent + renew_deadline regardless of any
// request in flight.
#pragma once

#include <atomic>
#include <chrono>
#include <memory>
#include <string>
#include <thread>

#include "core/cancel.h"
#include "core/env_config.h"
#include "kube/client.h"

namespace bgc::kube {

struct LeaseSettings {
  bool enabled = false;
  std::string ns = "default";
  std::string name;
  int lease_seconds = 15;
  int renew_deadline_seconds = 10;
  int retry_seconds = 2;
  // CONF_LEADER_ELECTION, CONF_LEASE_NAMESPACE, CONF_LEASE_NAME, CONF_LEASE_DURATION_SECS,
  // CONF_LEASE_RENEW_DEADLINE_SECS, CONF_LEASE_RETRY_PERIOD_SECS.
  static LeaseSettings from_env(const EnvConfig& env, const std::string& default_name);
};

class LeaderElector {
 public:
  enum class Attempt { Held, HeldByOther, Failed };

  LeaderElector(KubeClient& client, LeaseSettings s, std::string identity = "");
  ~LeaderElector();
  LeaderElector(const LeaderElector&) = delete;
  LeaderElector& operator=(const LeaderElector&) = delete;
  // Blocks until leadership is acquired (true) or `stop` is cancelled (false).
  bool acquire(CancelToken& stop);
  // One attempt.  Held: this identity holds the lease afterwards.  HeldByOther: another
  // identity holds an unexpired lease (or won a write race).  Failed: API error.
  Attempt try_acquire_or_renew();
  // Renews in the background until destroyed; on loss of the lease cancels `stop_on_loss`.
  // The elector must outlive the work it guards (keep it in main's scope).
  void keep_renewing(std::shared_ptr<CancelToken> stop_on_loss);
  // True once keep_renewing() stepped down (renew deadline passed or another holder):
  // the process should exit non-zero, as client-go's OnStoppedLeading does.
  bool lost() const { return lost_.load(); }
  const std::string& identity() const { return identity_; }

 private:
  KubeClient& client_;  // the caller's client (kept for identity of the API server)
  std::unique_ptr<KubeClient> lease_client_;  // bounded timeout, no throttle retries
  LeaseSettings s_;
  std::string identity_;
  std::thread renew_thread_;
  std::thread watchdog_;
  CancelToken stop_renew_;
  std::atomic<int64_t> last_ok_sent_ns_{0};  // steady clock
  std::atomic<bool> lost_{false};
};

// Acquires leadership when `s.enabled` (blocking until acquired or stopped) and keeps it
// renewed.  Returns nullptr with *standby_stopped=false when election is disabled; returns
// nullptr with *standby_stopped=true when `stop` fired before this replica became leader.
std::unique_ptr<LeaderElector> lead_or_wait(KubeClient& client, const LeaseSettings& s,
                                            const std::shared_ptr<CancelToken>& stop, bool* standby_stopped);

std::string rfc3339_micro_now();
int64_t parse_rfc3339_micros(const std::string& s);  // micros since epoch, -1 on error

}  // namespace bgc::kube

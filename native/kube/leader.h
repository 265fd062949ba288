// Lease-based leader election (coordination.k8s.io/v1).  The reference's chart already
// grants the controller `leases` get/create/update/patch (reference
// charts/.../templates/serviceaccount.yaml:26-28) but never uses it, so two controller
// replicas double-write; CONF_LEADER_ELECTION=true enables this.
#pragma once

#include <memory>
#include <string>
#include <thread>

#include "core/cancel.h"
#include "kube/client.h"

namespace bgc::kube {

class LeaderElector {
 public:
  LeaderElector(KubeClient& client, std::string ns, std::string name, std::string identity = "",
                int lease_seconds = 15, int renew_seconds = 5);
  ~LeaderElector();
  // Blocks until leadership is acquired (true) or `stop` is cancelled (false).
  bool acquire(CancelToken& stop);
  // One attempt; true when this identity holds the lease afterwards.
  bool try_acquire_or_renew();
  // Renews in the background; on loss of the lease cancels `stop_on_loss`.
  void keep_renewing(std::shared_ptr<CancelToken> stop_on_loss);
  const std::string& identity() const { return identity_; }

 private:
  KubeClient& client_;
  std::string ns_, name_, identity_;
  int lease_seconds_, renew_seconds_;
  std::thread renew_thread_;
  CancelToken stop_renew_;
};

std::string rfc3339_micro_now();
int64_t parse_rfc3339_micros(const std::string& s);  // micros since epoch, -1 on error

}  // namespace bgc::kube

// Retry pacing for failed work items: client-go's default controller rate limiter
// (workqueue.DefaultControllerRateLimiter: ItemExponentialFailureRateLimiter max'd with a
// BucketRateLimiter), rebuilt here because kube-runtime's callers in the reference never
// retry at all — the synchronizer exits on the first error (reference
// src/synchronizer.rs:302-330,426-430).  Used when that exit is turned off
// (CONF_EXIT_ON_ERROR=false): a failing UserBootstrap is retried after
// base * 2^(failures-1), capped, and all retries together stay under `qps` with `burst`.
#pragma once

#include <chrono>
#include <map>
#include <mutex>
#include <string>

namespace bgc::kube {

class RetryLimiter {
 public:
  using ms = std::chrono::milliseconds;
  RetryLimiter(ms base = ms(5), ms cap = ms(60000), double qps = 10.0, int burst = 100);
  // Records one more failure of `key`; returns how long to wait before retrying it.
  ms when(const std::string& key);
  // The key succeeded: its backoff starts over.
  void forget(const std::string& key);
  int failures(const std::string& key) const;
  size_t tracked() const;

 private:
  ms base_, cap_;
  double qps_;
  double burst_;
  mutable std::mutex mu_;
  std::map<std::string, int> failures_;
  double tokens_;
  std::chrono::steady_clock::time_point last_;
};

}  // namespace bgc::kube

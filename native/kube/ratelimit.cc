#include "kube/ratelimit.h"

#include <algorithm>
#include <cmath>

namespace bgc::kube {

RetryLimiter::RetryLimiter(ms base, ms cap, double qps, int burst)
    : base_(std::max(ms(1), base)),
      cap_(std::max(base_, cap)),
      qps_(qps > 0 ? qps : 1e9),
      burst_(std::max(1, burst)),
      tokens_(burst_),
      last_(std::chrono::steady_clock::now()) {}

RetryLimiter::ms RetryLimiter::when(const std::string& key) {
  std::lock_guard<std::mutex> lk(mu_);
  const int n = failures_[key]++;
  // per key: base * 2^n, capped (the exponent is clamped before it can overflow)
  const double item = std::min(static_cast<double>(cap_.count()), static_cast<double>(base_.count()) * std::ldexp(1.0, std::min(n, 40)));
  // overall: a token bucket with reservation semantics (golang.org/x/time/rate Reserve):
  // take a token now, wait until the bucket would have produced it
  const auto now = std::chrono::steady_clock::now();
  tokens_ = std::min(burst_, tokens_ + std::chrono::duration<double>(now - last_).count() * qps_);
  last_ = now;
  tokens_ -= 1.0;
  const double bucket = tokens_ >= 0 ? 0.0 : -tokens_ / qps_ * 1000.0;
  return ms(static_cast<int64_t>(std::ceil(std::max(item, bucket))));
}

void RetryLimiter::forget(const std::string& key) {
  std::lock_guard<std::mutex> lk(mu_);
  failures_.erase(key);
}

int RetryLimiter::failures(const std::string& key) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = failures_.find(key);
  return it == failures_.end() ? 0 : it->second;
}

size_t RetryLimiter::tracked() const {
  std::lock_guard<std::mutex> lk(mu_);
  return failures_.size();
}

}  // namespace bgc::kube

#include "kube/leader.h"

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <ctime>

#include "core/crypto.h"
#include "core/log.h"

namespace bgc::kube {

using json::Value;

std::string rfc3339_micro_now() {
  auto now = std::chrono::system_clock::now();
  auto secs = std::chrono::time_point_cast<std::chrono::seconds>(now);
  auto micros = std::chrono::duration_cast<std::chrono::microseconds>(now - secs).count();
  std::time_t t = std::chrono::system_clock::to_time_t(now);
  std::tm tm{};
  gmtime_r(&t, &tm);
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%04d-%02d-%02dT%02d:%02d:%02d.%06ldZ", tm.tm_year + 1900, tm.tm_mon + 1, tm.tm_mday,
                tm.tm_hour, tm.tm_min, tm.tm_sec, static_cast<long>(micros));
  return buf;
}

int64_t parse_rfc3339_micros(const std::string& s) {
  std::tm tm{};
  int frac_len = 0;
  long frac = 0;
  if (s.size() < 20) return -1;
  if (std::sscanf(s.c_str(), "%4d-%2d-%2dT%2d:%2d:%2d", &tm.tm_year, &tm.tm_mon, &tm.tm_mday, &tm.tm_hour, &tm.tm_min,
                  &tm.tm_sec) != 6) {
    return -1;
  }
  tm.tm_year -= 1900;
  tm.tm_mon -= 1;
  size_t i = 19;
  if (i < s.size() && s[i] == '.') {
    ++i;
    while (i < s.size() && std::isdigit(static_cast<unsigned char>(s[i]))) {
      if (frac_len < 6) {
        frac = frac * 10 + (s[i] - '0');
        ++frac_len;
      }
      ++i;
    }
    while (frac_len < 6) {
      frac *= 10;
      ++frac_len;
    }
  }
  return static_cast<int64_t>(timegm(&tm)) * 1000000 + frac;
}

static int64_t now_micros() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

LeaderElector::LeaderElector(KubeClient& client, std::string ns, std::string name, std::string identity,
                             int lease_seconds, int renew_seconds)
    : client_(client), ns_(std::move(ns)), name_(std::move(name)), identity_(std::move(identity)),
      lease_seconds_(lease_seconds), renew_seconds_(renew_seconds) {
  if (identity_.empty()) {
    char host[256] = {0};
    gethostname(host, sizeof(host) - 1);
    identity_ = std::string(host) + "_" + crypto::uuid_v4().substr(0, 8);
  }
}

LeaderElector::~LeaderElector() {
  stop_renew_.cancel();
  if (renew_thread_.joinable()) renew_thread_.join();
}

bool LeaderElector::try_acquire_or_renew() {
  std::string now = rfc3339_micro_now();
  auto cur = client_.get_opt(types::Lease, ns_, name_);
  if (!cur) {
    Value lease = Value::object({{"apiVersion", "coordination.k8s.io/v1"}, {"kind", "Lease"}});
    lease["metadata"] = Value::object({{"name", name_}, {"namespace", ns_}});
    lease["spec"] = Value::object({{"holderIdentity", identity_},
                                   {"leaseDurationSeconds", lease_seconds_},
                                   {"acquireTime", now},
                                   {"renewTime", now},
                                   {"leaseTransitions", 0}});
    try {
      client_.create(types::Lease, ns_, lease);
      return true;
    } catch (const ApiError& e) {
      if (e.code() == 409) return false;  // somebody else created it first
      throw;
    }
  }
  Value lease = *cur;
  Value& spec = lease["spec"];
  std::string holder = spec.get_string("holderIdentity");
  int64_t renew = parse_rfc3339_micros(spec.get_string("renewTime"));
  int64_t dur = spec.get("leaseDurationSeconds").is_int() ? spec.get("leaseDurationSeconds").as_int() : lease_seconds_;
  bool expired = renew < 0 || now_micros() > renew + dur * 1000000;
  if (holder != identity_ && !expired && !holder.empty()) return false;
  if (holder != identity_) {
    spec["acquireTime"] = now;
    int64_t transitions = spec.get("leaseTransitions").is_int() ? spec.get("leaseTransitions").as_int() : 0;
    spec["leaseTransitions"] = transitions + 1;
  }
  spec["holderIdentity"] = identity_;
  spec["leaseDurationSeconds"] = lease_seconds_;
  spec["renewTime"] = now;
  try {
    client_.replace(types::Lease, ns_, name_, lease);  // resourceVersion precondition
    return true;
  } catch (const ApiError& e) {
    if (e.code() == 409) return false;
    throw;
  }
}

bool LeaderElector::acquire(CancelToken& stop) {
  LOG_INFO("leader") << "attempting to acquire lease " << ns_ << "/" << name_ << " as " << identity_;
  while (!stop.cancelled()) {
    try {
      if (try_acquire_or_renew()) {
        LOG_INFO("leader") << "acquired lease " << ns_ << "/" << name_;
        return true;
      }
    } catch (const std::exception& e) {
      LOG_WARN("leader") << "lease attempt failed: " << e.what();
    }
    if (stop.wait_for(std::chrono::seconds(2))) break;
  }
  return false;
}

void LeaderElector::keep_renewing(std::shared_ptr<CancelToken> stop_on_loss) {
  renew_thread_ = std::thread([this, stop_on_loss] {
    auto last_ok = std::chrono::steady_clock::now();
    while (!stop_renew_.wait_for(std::chrono::seconds(renew_seconds_))) {
      if (stop_on_loss->cancelled()) return;
      bool ok = false;
      try {
        ok = try_acquire_or_renew();
      } catch (const std::exception& e) {
        LOG_WARN("leader") << "lease renew failed: " << e.what();
      }
      if (ok) {
        last_ok = std::chrono::steady_clock::now();
      } else if (std::chrono::steady_clock::now() - last_ok > std::chrono::seconds(lease_seconds_)) {
        LOG_ERROR("leader") << "lost lease " << ns_ << "/" << name_ << "; shutting down";
        stop_on_loss->cancel();
        return;
      }
    }
  });
}

}  // namespace bgc::kube

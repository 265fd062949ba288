#include "kube/leader.h"

#include <unistd.h>

#include <algorithm>
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

LeaseSettings LeaseSettings::from_env(const EnvConfig& env, const std::string& default_name) {
  LeaseSettings s;
  s.enabled = env.boolean_or("leader_election", false);
  s.ns = env.str_or("lease_namespace", s.ns);
  s.name = env.str_or("lease_name", default_name);
  s.lease_seconds = static_cast<int>(env.u64_or("lease_duration_secs", 15));
  s.renew_deadline_seconds = static_cast<int>(env.u64_or("lease_renew_deadline_secs", 10));
  s.retry_seconds = static_cast<int>(env.u64_or("lease_retry_period_secs", 2));
  if (s.retry_seconds < 1 || s.renew_deadline_seconds <= s.retry_seconds ||
      s.lease_seconds <= s.renew_deadline_seconds) {
    throw ConfigError("lease timing must satisfy 1 <= retry_period < renew_deadline < lease_duration");
  }
  return s;
}

LeaderElector::LeaderElector(KubeClient& client, LeaseSettings s, std::string identity)
    : client_(client), s_(std::move(s)), identity_(std::move(identity)) {
  KubeConfig lc = client_.config();
  lc.timeout_ms = std::max(1, s_.renew_deadline_seconds - s_.retry_seconds) * 1000;
  lc.max_throttle_retries = 0;  // a throttled renew is a failed renew: retried on the next period
  lease_client_ = std::make_unique<KubeClient>(lc);
  if (identity_.empty()) {
    char host[256] = {0};
    gethostname(host, sizeof(host) - 1);
    identity_ = std::string(host) + "_" + crypto::uuid_v4().substr(0, 8);
  }
}

LeaderElector::~LeaderElector() {
  stop_renew_.cancel();
  if (watchdog_.joinable()) watchdog_.join();
  if (renew_thread_.joinable()) renew_thread_.join();
}

LeaderElector::Attempt LeaderElector::try_acquire_or_renew() {
  std::string now = rfc3339_micro_now();
  auto cur = lease_client_->get_opt(types::Lease, s_.ns, s_.name);
  if (!cur) {
    Value lease = Value::object({{"apiVersion", "coordination.k8s.io/v1"}, {"kind", "Lease"}});
    lease["metadata"] = Value::object({{"name", s_.name}, {"namespace", s_.ns}});
    lease["spec"] = Value::object({{"holderIdentity", identity_},
                                   {"leaseDurationSeconds", s_.lease_seconds},
                                   {"acquireTime", now},
                                   {"renewTime", now},
                                   {"leaseTransitions", 0}});
    try {
      lease_client_->create(types::Lease, s_.ns, lease);
      return Attempt::Held;
    } catch (const ApiError& e) {
      if (e.code() == 409) return Attempt::HeldByOther;  // somebody else created it first
      throw;
    }
  }
  Value lease = *cur;
  Value& spec = lease["spec"];
  std::string holder = spec.get_string("holderIdentity");
  int64_t renew = parse_rfc3339_micros(spec.get_string("renewTime"));
  int64_t dur = spec.get("leaseDurationSeconds").is_int() ? spec.get("leaseDurationSeconds").as_int() : s_.lease_seconds;
  bool expired = renew < 0 || now_micros() > renew + dur * 1000000;
  if (holder != identity_ && !expired && !holder.empty()) return Attempt::HeldByOther;
  if (holder != identity_) {
    spec["acquireTime"] = now;
    int64_t transitions = spec.get("leaseTransitions").is_int() ? spec.get("leaseTransitions").as_int() : 0;
    spec["leaseTransitions"] = transitions + 1;
  }
  spec["holderIdentity"] = identity_;
  spec["leaseDurationSeconds"] = s_.lease_seconds;
  spec["renewTime"] = now;
  try {
    lease_client_->replace(types::Lease, s_.ns, s_.name, lease);  // resourceVersion precondition
    return Attempt::Held;
  } catch (const ApiError& e) {
    if (e.code() == 409) return Attempt::HeldByOther;  // lost a write race: re-read next time
    throw;
  }
}

bool LeaderElector::acquire(CancelToken& stop) {
  LOG_INFO("leader") << "attempting to acquire lease " << s_.ns << "/" << s_.name << " as " << identity_;
  while (!stop.cancelled()) {
    try {
      if (try_acquire_or_renew() == Attempt::Held) {
        LOG_INFO("leader") << "acquired lease " << s_.ns << "/" << s_.name;
        return true;
      }
    } catch (const std::exception& e) {
      LOG_WARN("leader") << "lease attempt failed: " << e.what();
    }
    if (stop.wait_for(std::chrono::seconds(s_.retry_seconds))) break;
  }
  return false;
}

void LeaderElector::keep_renewing(std::shared_ptr<CancelToken> stop_on_loss) {
  using clock = std::chrono::steady_clock;
  auto ns_now = [] { return clock::now().time_since_epoch().count(); };
  // the deadline runs from when the last successful renew was *sent*: the lease's
  // renewTime is at or after that instant, so a standby (waiting lease_seconds from
  // renewTime by its own clock) cannot take over before we stop.
  last_ok_sent_ns_ = ns_now();
  const int64_t deadline_ns = std::chrono::nanoseconds(std::chrono::seconds(s_.renew_deadline_seconds)).count();
  renew_thread_ = std::thread([this, stop_on_loss, ns_now] {
    while (!stop_renew_.wait_for(std::chrono::seconds(s_.retry_seconds))) {
      if (stop_on_loss->cancelled()) return;
      const int64_t sent = ns_now();
      Attempt a = Attempt::Failed;
      try {
        a = try_acquire_or_renew();
      } catch (const std::exception& e) {
        LOG_WARN("leader") << "lease renew failed: " << e.what();
      }
      if (stop_on_loss->cancelled()) return;  // the watchdog already stepped down
      if (a == Attempt::Held) {
        last_ok_sent_ns_ = sent;
        continue;
      }
      if (a == Attempt::HeldByOther) {
        LOG_ERROR("leader") << "lease " << s_.ns << "/" << s_.name << " is held by another replica; stepping down";
        lost_ = true;
        stop_on_loss->cancel();
        return;
      }
      // transient failure: retried every period; the watchdog enforces the deadline
    }
  });
  // Watchdog: steps down at last_ok_sent + renew_deadline even when a renew request is
  // still hanging on a stalled API server.
  watchdog_ = std::thread([this, stop_on_loss, ns_now, deadline_ns] {
    while (!stop_renew_.wait_for(std::chrono::milliseconds(100))) {
      if (stop_on_loss->cancelled()) return;
      if (ns_now() - last_ok_sent_ns_.load() >= deadline_ns) {
        LOG_ERROR("leader") << "lost lease " << s_.ns << "/" << s_.name << " (renew deadline " << s_.renew_deadline_seconds
                            << " s passed); shutting down";
        lost_ = true;
        stop_on_loss->cancel();
        return;
      }
    }
  });
}

std::unique_ptr<LeaderElector> lead_or_wait(KubeClient& client, const LeaseSettings& s,
                                            const std::shared_ptr<CancelToken>& stop, bool* standby_stopped) {
  *standby_stopped = false;
  if (!s.enabled) return nullptr;
  auto le = std::make_unique<LeaderElector>(client, s);
  if (!le->acquire(*stop)) {
    *standby_stopped = true;
    return nullptr;
  }
  le->keep_renewing(stop);
  return le;
}

}  // namespace bgc::kube

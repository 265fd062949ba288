#include "kube/events.h"

#include <cinttypes>
#include <cstdio>
#include <ctime>

#include "core/log.h"
#include "core/metrics.h"

namespace bgc::kube {

using json::Value;

namespace {

std::string rfc3339_now() {  // Event timestamps are whole seconds (metav1.Time)
  std::time_t t = std::time(nullptr);
  std::tm tm{};
  gmtime_r(&t, &tm);
  char buf[32];
  std::strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%SZ", &tm);
  return buf;
}

}  // namespace

EventRecorder::EventRecorder(KubeClient& client, EventOptions opts)
    : client_(client), opts_(std::move(opts)), limiter_(opts_.burst, opts_.refill_per_minute) {
  worker_ = std::thread([this] { run(); });
}

EventRecorder::~EventRecorder() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (worker_.joinable()) worker_.join();
}

bool EventRateLimiter::allow(const std::string& key, std::chrono::steady_clock::time_point now) {
  auto [it, fresh] = buckets_.try_emplace(key);
  Bucket& b = it->second;
  if (fresh) {
    b.tokens = burst_;
    b.refilled = now;
  } else {
    const double mins = std::chrono::duration<double>(now - b.refilled).count() / 60.0;
    b.tokens = std::min(burst_, b.tokens + mins * refill_per_minute_);
    b.refilled = now;
  }
  if (b.tokens < 1.0) return false;
  b.tokens -= 1.0;
  if (buckets_.size() > max_keys_) evict(now, key);  // bound memory on huge clusters
  return true;
}

// Drops buckets that have refilled to the burst (a fresh bucket is identical, so this
// loses nothing); if every bucket is still draining, drops the one refilled longest ago.
// `keep` (the key just charged) is never dropped.
void EventRateLimiter::evict(std::chrono::steady_clock::time_point now, const std::string& keep) {
  auto oldest = buckets_.end();
  for (auto it = buckets_.begin(); it != buckets_.end();) {
    if (it->first == keep) {
      ++it;
      continue;
    }
    const double mins = std::chrono::duration<double>(now - it->second.refilled).count() / 60.0;
    if (it->second.tokens + mins * refill_per_minute_ >= burst_) {
      it = buckets_.erase(it);
      continue;
    }
    if (oldest == buckets_.end() || it->second.refilled < oldest->second.refilled) oldest = it;
    ++it;
  }
  if (buckets_.size() > max_keys_ && oldest != buckets_.end()) buckets_.erase(oldest);
}

void EventRecorder::record(const ResourceType& rt, const Value& obj, const std::string& type, const std::string& reason,
                           const std::string& message) {
  static auto& dropped = metrics::Registry::global().counter("bgc_events_dropped_total",
                                                             "Events not written (queue full or per-object rate limit)");
  const Value& meta = obj.get("metadata");
  Item it;
  it.ref = Value::object({{"apiVersion", rt.api_version()}, {"kind", rt.kind}, {"name", meta.get_string("name")}});
  if (rt.namespaced) it.ref["namespace"] = meta.get_string("namespace");
  if (meta.contains("uid")) it.ref["uid"] = meta.get_string("uid");
  if (meta.contains("resourceVersion")) it.ref["resourceVersion"] = meta.get_string("resourceVersion");
  it.ns = rt.namespaced ? meta.get_string("namespace") : opts_.cluster_namespace;
  it.type = type;
  it.reason = reason;
  it.message = message.size() > 1024 ? message.substr(0, 1021) + "..." : message;  // Event message limit
  it.at = std::chrono::steady_clock::now();
  const std::string object_key = rt.plural + "/" + it.ns + "/" + meta.get_string("name");
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_ || q_.size() >= opts_.max_queue || !limiter_.allow(object_key, it.at)) {
      dropped_.fetch_add(1);
      dropped.inc();
      return;
    }
    q_.push_back(std::move(it));
  }
  cv_.notify_one();
}

void EventRecorder::flush(std::chrono::milliseconds timeout) {
  std::unique_lock<std::mutex> lk(mu_);
  idle_cv_.wait_for(lk, timeout, [&] { return q_.empty() && !busy_; });
}

void EventRecorder::run() {
  while (true) {
    Item it;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) break;  // stopping and drained
      it = std::move(q_.front());
      q_.pop_front();
      busy_ = true;
    }
    try {
      write(it);
    } catch (const std::exception& e) {
      LOG_WARN("events") << "event " << it.reason << " for " << it.ref.get_string("kind") << "/"
                         << it.ref.get_string("name") << " not written: " << e.what();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      busy_ = false;
    }
    idle_cv_.notify_all();
  }
  idle_cv_.notify_all();
}

void EventRecorder::write(const Item& it) {
  static auto& events = metrics::Registry::global().counter("bgc_events_total", "Events written (created or aggregated)");
  const std::string now = rfc3339_now();
  const std::string key = it.ns + "|" + it.ref.get_string("kind") + "|" + it.ref.get_string("name") + "|" +
                          it.ref.get_string("uid") + "|" + it.type + "|" + it.reason + "|" + it.message;
  auto found = seen_.find(key);
  if (found != seen_.end() && it.at - found->second.last < opts_.aggregate_window) {
    Seen& s = found->second;
    try {
      client_.patch_merge(types::Event, s.ns, s.name,
                          Value::object({{"count", s.count + 1}, {"lastTimestamp", now}}));
      ++s.count;
      s.last = it.at;
      aggregated_.fetch_add(1);
      events.inc();
      return;
    } catch (const ApiError& e) {
      if (e.code() != 404) throw;  // the Event expired meanwhile: create a new one
      seen_.erase(found);
    }
  }
  // name: <object>.<nanoseconds, hex> as client-go does
  char suffix[32];
  std::snprintf(suffix, sizeof(suffix), ".%" PRIx64,
                static_cast<uint64_t>(std::chrono::system_clock::now().time_since_epoch().count()));
  const std::string name = it.ref.get_string("name") + suffix;
  Value ev = Value::object({{"apiVersion", "v1"}, {"kind", "Event"},
                            {"metadata", Value::object({{"name", name}, {"namespace", it.ns}})},
                            {"involvedObject", it.ref}, {"reason", it.reason}, {"message", it.message},
                            {"type", it.type}, {"count", 1}, {"firstTimestamp", now}, {"lastTimestamp", now},
                            {"source", Value::object({{"component", opts_.component}, {"host", opts_.host}})},
                            {"reportingComponent", opts_.component}, {"reportingInstance", opts_.host}});
  client_.create(types::Event, it.ns, ev);
  created_.fetch_add(1);
  events.inc();
  Seen s;
  s.name = name;
  s.ns = it.ns;
  s.count = 1;
  s.first = now;
  s.last = it.at;
  seen_[key] = std::move(s);
  if (seen_.size() > 4096) {  // forget the oldest correlation entries
    auto oldest = seen_.begin();
    for (auto i = seen_.begin(); i != seen_.end(); ++i) {
      if (i->second.last < oldest->second.last) oldest = i;
    }
    seen_.erase(oldest);
  }
}

}  // namespace bgc::kube

// Kubernetes Event recorder (core/v1 Event), the client-go record.EventRecorder /
// kube-runtime Recorder equivalent: `kubectl describe node` / `kubectl describe
// userbootstrap` then shows why a GPU went Unhealthy or a reconcile failed.
//
// Recording never blocks the caller: events go through a bounded queue to one worker
// thread.  The worker correlates repeats like client-go's EventCorrelator: the same
// (object, type, reason, message) within `aggregate_window` bumps `count` and
// `lastTimestamp` of the existing Event (one merge patch) instead of creating another,
// and a per-object token bucket drops event storms (counted in
// bgc_events_dropped_total).  Cluster-scoped objects (Node, UserBootstrap) get their
// Events in `cluster_namespace` ("default", as the apiserver does).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>

#include "core/json.h"
#include "kube/client.h"
#include "kube/resource.h"

namespace bgc::kube {

struct EventOptions {
  std::string component;                  // source.component / reportingComponent
  std::string host;                       // source.host / reportingInstance
  std::string cluster_namespace = "default";
  std::chrono::seconds aggregate_window{600};
  double burst = 10;                      // per involved object
  double refill_per_minute = 6;
  size_t max_queue = 1024;
};

// Per-object token bucket of the recorder (client-go's EventSourceObjectSpamFilter): `burst`
// events, refilled at `refill_per_minute`.  Past `max_keys` objects it evicts buckets that
// have refilled to the burst (a fresh bucket is identical), else the one refilled longest
// ago, so an object that floods events keeps its drained bucket.  Not thread-safe.
class EventRateLimiter {
 public:
  EventRateLimiter(double burst, double refill_per_minute, size_t max_keys = 4096)
      : burst_(burst), refill_per_minute_(refill_per_minute), max_keys_(max_keys) {}
  bool allow(const std::string& object_key, std::chrono::steady_clock::time_point now);
  size_t size() const { return buckets_.size(); }

 private:
  struct Bucket {
    double tokens = 0;
    std::chrono::steady_clock::time_point refilled;
  };
  void evict(std::chrono::steady_clock::time_point now, const std::string& keep);
  double burst_, refill_per_minute_;
  size_t max_keys_;
  std::map<std::string, Bucket> buckets_;
};

class EventRecorder {
 public:
  EventRecorder(KubeClient& client, EventOptions opts);
  ~EventRecorder();
  EventRecorder(const EventRecorder&) = delete;
  EventRecorder& operator=(const EventRecorder&) = delete;

  // type: "Normal" | "Warning".  `obj` is the involved object (its metadata names it).
  void record(const ResourceType& rt, const json::Value& obj, const std::string& type, const std::string& reason,
              const std::string& message);
  // Blocks until everything queued so far was written (tests, shutdown).
  void flush(std::chrono::milliseconds timeout = std::chrono::milliseconds(5000));
  uint64_t created() const { return created_.load(); }
  uint64_t aggregated() const { return aggregated_.load(); }
  uint64_t dropped() const { return dropped_.load(); }

 private:
  struct Item {
    json::Value ref;  // involvedObject
    std::string ns;   // where the Event lives
    std::string type, reason, message;
    std::chrono::steady_clock::time_point at;
  };
  struct Seen {
    std::string name;
    std::string ns;
    int64_t count = 0;
    std::string first;  // firstTimestamp
    std::chrono::steady_clock::time_point last;
  };
  void run();
  void write(const Item& it);

  KubeClient& client_;
  EventOptions opts_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::condition_variable idle_cv_;
  std::deque<Item> q_;
  bool busy_ = false;
  bool stop_ = false;
  std::map<std::string, Seen> seen_;      // correlation key -> existing Event (worker only)
  EventRateLimiter limiter_;              // object key -> tokens (under mu_)
  std::atomic<uint64_t> created_{0}, aggregated_{0}, dropped_{0};
  std::thread worker_;
};

}  // namespace bgc::kube

// Controller runtime: watcher (LIST+WATCH with resourceVersion bookkeeping, 410 relist,
// reconnect backoff), reflector store, de-duplicating work queue with delayed requeue
// and per-key exclusivity, and a Controller that wires them to a reconcile function.
//
// Equivalent of kube-runtime 0.84's watcher/reflector/scheduler/applier used by the
// reference (`Controller::new(..).owns(..)...run(reconcile, error_policy, ctx)`,
// src/controller.rs:233-246).  Differences, by design:
//  * owned objects map to their owner by *name* (the owner is cluster-scoped), fixing
//    the namespaced-child -> cluster-scoped-owner mapping gap;
//  * N worker threads reconcile different keys concurrently, one key at a time.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "core/metrics.h"
#include <vector>

#include "core/cancel.h"
#include "core/env_config.h"
#include "core/json.h"
#include "kube/client.h"
#include "kube/resource.h"

namespace bgc::kube {

using ObjPtr = std::shared_ptr<const json::Value>;

struct WatchEvent {
  enum class Type { Added, Modified, Deleted, Restarted };
  Type type;
  ObjPtr object;                 // Added/Modified/Deleted
  std::vector<ObjPtr> objects;   // Restarted (full relist)
  int64_t read_ns = 0;           // when its line came off the watch stream (monotonic)
};

std::string meta_name(const json::Value& obj);
std::string meta_namespace(const json::Value& obj);
std::string meta_rv(const json::Value& obj);

// Runs LIST then WATCH forever (until cancelled), emitting events. 410 Gone (an ERROR
// event, or the HTTP status at watch start) triggers a relist; connection failures back
// off exponentially (0.8s..30s).
//
// The initial state comes from a paginated LIST (limit=page_size, following continue
// tokens; an expired token restarts the list — kube-runtime's watcher::Config default
// of 500), or, with streaming lists on, from one WATCH with sendInitialEvents=true whose
// initial ADDED events end at a BOOKMARK annotated k8s.io/initial-events-end (the
// apiserver never materialises the whole list).  A server that rejects streaming lists
// (4xx) makes the watcher fall back to LIST for good.
//
// Liveness: a watch stream that delivers no byte (no event, no BOOKMARK) for
// idle_timeout_ms is closed and resumed from the last resourceVersion on a new connection,
// and the client's pooled connections are dropped with it (kube-client puts a 295 s read
// timeout on its watch connections, hyper-timeout in the reference's Cargo.lock:982-997;
// kube-runtime's watcher then restarts the stream).  The server-side timeoutSeconds is kept
// below that deadline, so a healthy quiet watch ends cleanly first.  Every running watcher
// also feeds the "watches" readiness check (/readyz): it fails while any watcher has not
// completed its initial list, or has seen no event, bookmark or (re)started stream for
// three of the server's bookmark intervals (once two bookmarks have shown the cadence;
// at least 2 s) or, before that, for its idle deadline.  So a silent stall reads as
// not-ready on /readyz before the deadline reconnects the watch.
class Watcher {
 public:
  struct Defaults {
    int64_t page_size = 500;   // 0 = unpaginated LIST
    bool streaming_lists = false;
    int64_t idle_timeout_ms = 295000;  // 0 = no client-side deadline (and no readiness check)
  };
  // Process-wide defaults (each binary sets them from CONF_LIST_PAGE_SIZE /
  // CONF_STREAMING_LISTS / CONF_WATCH_IDLE_TIMEOUT_SECS before starting its watchers;
  // configure_from_env below).
  static void set_defaults(Defaults d);
  static Defaults defaults();
  // CONF_LIST_PAGE_SIZE, CONF_STREAMING_LISTS, CONF_WATCH_IDLE_TIMEOUT_SECS (default 295)
  // and the TCP keepalive of API connections, CONF_TCP_KEEPALIVE_SECS (30, 0 = off) and
  // CONF_TCP_USER_TIMEOUT_SECS (60, 0 = kernel default).  Throws ConfigError.
  static void configure_from_env(const EnvConfig& env);
  void set_idle_timeout_ms(int64_t ms) { idle_timeout_ms_ = ms; }
  uint64_t idle_timeouts() const { return idle_timeouts_.load(); }

  Watcher(KubeClient& client, ResourceType rt, std::string ns = "", std::string label_selector = "",
          std::string field_selector = "");
  void set_page_size(int64_t n) { page_size_ = n; }
  void set_streaming_lists(bool on) { streaming_ = on; }
  // Only object metadata (PartialObjectMetadata lists and events); cached objects keep
  // the watched type's kind/apiVersion and carry just "metadata".
  void set_metadata_only(bool on) { metadata_only_ = on; }
  void run(CancelToken& stop, const std::function<void(const WatchEvent&)>& on_event);
  // Optional pre-parse filter on raw watch lines (e.g. a name prefix): ADDED/MODIFIED/
  // DELETED lines it rejects are skipped without JSON parsing.  A consumer whose filter
  // drops events must not rely on them (the resume resourceVersion may lag; a resumed
  // watch replays them, and they are filtered again).
  void set_line_filter(std::function<bool(std::string_view)> f) { line_filter_ = std::move(f); }
  // Optional selective parse of ADDED/MODIFIED/DELETED events (json::parse_projected over
  // the whole event line, so the root projection names "type" and "object"): members the
  // consumer never reads (annotations such as kubectl's last-applied copy of the spec,
  // managedFields) are scanned, not built.  ERROR and BOOKMARK lines and the initial
  // events of a streaming list are always parsed in full.  `p` must outlive the watcher.
  void set_projection(const json::Projection* p) { projection_ = p; }
  uint64_t relists() const { return relists_.load(); }
  uint64_t reconnects() const { return reconnects_.load(); }
  uint64_t list_pages() const { return list_pages_.load(); }

 private:
  // Paginated LIST; returns the list resourceVersion.
  std::string list_all(std::vector<ObjPtr>& out, CancelToken& stop);
  ObjPtr typed(json::Value obj) const;
  int64_t page_size_;
  bool streaming_;
  int64_t idle_timeout_ms_;
  std::atomic<uint64_t> idle_timeouts_{0};
  bool metadata_only_ = false;
  std::atomic<uint64_t> list_pages_{0};
  KubeClient& client_;
  ResourceType rt_;
  std::string ns_;
  std::string selector_;
  std::string field_selector_;
  std::function<bool(std::string_view)> line_filter_;
  const json::Projection* projection_ = nullptr;
  std::atomic<uint64_t> relists_{0};
  std::atomic<uint64_t> reconnects_{0};
};

// Thread-safe object cache keyed by "ns/name" (namespaced) or "name".
class Store {
 public:
  explicit Store(ResourceType rt) : rt_(std::move(rt)) {}
  void apply(const WatchEvent& ev);
  ObjPtr get(const std::string& key) const;
  ObjPtr get(const std::string& ns, const std::string& name) const { return get(rt_.key(ns, name)); }
  std::vector<ObjPtr> list() const;
  size_t size() const { return size_.load(std::memory_order_relaxed); }  // lock-free (gauges)
  bool synced() const { return synced_.load(); }
  // Blocks until the first full list has been applied (or timeout).
  bool wait_synced(std::chrono::milliseconds timeout) const;
  const ResourceType& type() const { return rt_; }

 private:
  ResourceType rt_;
  mutable std::mutex mu_;
  mutable std::condition_variable cv_;
  std::unordered_map<std::string, ObjPtr> items_;
  std::atomic<size_t> size_{0};
  std::atomic<bool> synced_{false};
};

// De-duplicating delayed work queue (client-go workqueue + kube-runtime scheduler
// semantics): at most one pending entry per key, earliest due time wins; a key being
// processed is never handed to a second worker — re-adds while in flight are deferred
// until done().
//
// Optionally sharded by key: each shard has its own lock and its own workers (worker i
// serves shard i % shards).  Every key lives in one shard, which keeps the per-key
// guarantees above.  Round 6 traced open-loop tails to this lock: the watcher's add and the
// workers' finish waited up to 10-15 ms behind a holder preempted by the worker it had just
// signalled (profiles/r6_locks/).  Signals now go out after the unlock; shards cut the
// remaining waits further but split the worker pool (see shards_for).
class WorkQueue {
 public:
  using Clock = std::chrono::steady_clock;
  // `shards` >= 1; run at least as many workers as shards (each shard needs one).
  explicit WorkQueue(size_t shards = 1);
  ~WorkQueue();
  // The controller's and synchronizer's shard count: BGC_QUEUE_SHARDS (default 1), at most
  // one per worker and 8.
  static size_t shards_for(int workers);
  size_t shards() const { return shards_.size(); }
  void add(const std::string& key) { add_after(key, std::chrono::milliseconds(0)); }
  void add_after(const std::string& key, std::chrono::milliseconds delay);
  // Blocks until a key of worker `worker`'s shard is due or the queue shuts down (false).
  bool get(std::string& key, size_t worker = 0);
  void done(const std::string& key);
  // Drops a pending entry, e.g. the periodic requeue of an object that was deleted: keeps
  // the queue proportional to live objects under churn.  A key forgotten while in flight
  // also ignores the worker's own requeue() of it (the reconcile that raced the deletion);
  // an add()/add_after() (a new event, e.g. the object re-created) clears that.
  void forget(const std::string& key);
  // The worker's periodic/error requeue of the key it is processing.
  void requeue(const std::string& key, std::chrono::milliseconds delay);
  // A worker is done with `key`: requeue (when `requeue`) and done() under one lock.
  void finish(const std::string& key, bool requeue, std::chrono::milliseconds delay);
  void shutdown();
  size_t pending() const;  // lock-free (gauges)
  size_t in_flight() const;

 private:
  struct Shard;
  Shard& shard_of(const std::string& key) const;
  std::vector<std::unique_ptr<Shard>> shards_;
};

struct Action {
  bool requeue = false;
  std::chrono::milliseconds after{0};
  static Action requeue_after(std::chrono::milliseconds d) { return {true, d}; }
  static Action await_change() { return {false, std::chrono::milliseconds(0)}; }
};

class Controller {
 public:
  using Reconciler = std::function<Action(const ObjPtr& obj)>;
  using ErrorPolicy = std::function<Action(const ObjPtr& obj, const std::exception& err)>;
  // Maps a child object to owner keys to enqueue.
  using Mapper = std::function<std::vector<std::string>(const json::Value& child)>;

  struct Options {
    int workers = 8;
    // Owners of a DELETED child are enqueued after this delay: during cascading deletion the
    // children's DELETED events can overtake the owner's own DELETED event, and reconciling
    // the stale owner would re-create children the garbage collector is removing.
    std::chrono::milliseconds child_delete_delay{50};
    // kube-runtime's controller::Config::debounce: a watch event schedules its object's
    // reconcile this much later, and further events for the object meanwhile merge into
    // that one reconcile (the earliest due time wins, so a burst is delayed by at most this).
    std::chrono::milliseconds debounce{0};
    // Selective parse of the primary watch's and the owned-kind watches' events
    // (Watcher::set_projection).
    const json::Projection* primary_projection = nullptr;
    const json::Projection* child_projection = nullptr;
  };

  Controller(KubeClient& client, ResourceType primary, Options opts);
  ~Controller();
  // Watches `child` and enqueues its owners (by default: ownerReferences whose kind
  // and apiVersion match the primary type, mapped by name).
  // `label_selector` limits the child watch server-side (e.g. to children this controller
  // labelled); empty = every object of the kind, like kube-runtime's default.
  // `metadata_only`: watch PartialObjectMetadata (enough for the default mapper and for
  // resourceVersion checks; the child store then holds metadata only).
  void owns(const ResourceType& child, Mapper mapper = nullptr, std::string label_selector = "",
            bool metadata_only = false);
  // Child ADDED/MODIFIED events for which `filter` returns false do not enqueue the owner
  // (e.g. the echo of the reconciler's own apply). DELETED events and relists always do.
  using ChildFilter = std::function<bool(const ResourceType& child_type, const json::Value& child)>;
  void set_child_filter(ChildFilter f) { child_filter_ = std::move(f); }
  // Called for every child DELETED event (e.g. to drop per-child caches).
  void set_child_deleted_hook(ChildFilter f) { child_deleted_ = std::move(f); }
  // Called for every primary DELETED event (drop per-owner caches).
  using PrimaryHook = std::function<void(const json::Value& primary)>;
  void set_primary_deleted_hook(PrimaryHook f) { primary_deleted_ = std::move(f); }
  uint64_t filtered_events() const { return filtered_.load(); }
  // Extra trigger source (e.g. a periodic external refresh).
  void enqueue(const std::string& key) { queue_.add(key); }
  void enqueue_all();
  Store& store() { return *primary_store_; }
  Store* child_store(const std::string& plural);
  // Blocks until `stop` is cancelled; in-flight reconciles finish before returning.
  void run(CancelToken& stop, Reconciler reconcile, ErrorPolicy error_policy);
  bool wait_synced(std::chrono::milliseconds timeout);

 private:
  struct Child {
    ResourceType rt;
    Mapper mapper;
    std::string selector;
    bool metadata_only = false;
    std::unique_ptr<Store> store;
    metrics::Gauge* gauge = nullptr;  // bgc_controller_store_objects{resource=...}
  };
  KubeClient& client_;
  ResourceType primary_;
  Options opts_;
  std::unique_ptr<Store> primary_store_;
  std::vector<std::unique_ptr<Child>> children_;
  WorkQueue queue_;
  ChildFilter child_filter_;
  ChildFilter child_deleted_;
  PrimaryHook primary_deleted_;
  std::atomic<uint64_t> filtered_{0};
};

Controller::Mapper owner_mapper(const ResourceType& owner);

}  // namespace bgc::kube

// UserBootstrap reconciler (reference src/controller.rs:50-175).
//
// Semantics preserved from the reference:
//  * namespace name = metadata.name lower-cased; every child carries a controller
//    ownerReference to the UserBootstrap (GC handles deletion, no finalizer);
//  * server-side apply with field manager "bacchus-gpu-controller.bacchus.io" + force,
//    Namespace first, then ResourceQuota (if spec.quota), Role (if spec.role) and
//    RoleBinding (if spec.rolebinding AND status.synchronized_with_sheet);
//  * success requeues after 30 s, errors after 3 s (error_policy);
//  * removing a spec field never deletes an existing child.
//
// MI355X-era improvements (observable end state unchanged):
//  * ResourceQuota and Role are applied concurrently once the Namespace exists, and
//    the RoleBinding last (at most 3 round trips instead of 4 sequential ones);
//  * an apply is skipped when the watch cache shows the child exactly as this
//    controller last wrote it (same body hash AND same resourceVersion), so the 30 s
//    drift-repair pass costs zero API writes unless something actually drifted;
//  * the watch cache is not the only source of truth: every resync_secs (300 s) a
//    UserBootstrap's reconcile re-reads each child from the apiserver (one GET) and
//    re-applies the ones that no longer carry what this controller applies.  A missed
//    watch event, a stalled watch or a cache bug is healed within one resync period; the
//    reference heals within its 30 s requeue by re-applying everything unconditionally
//    (controller.rs:67-154), at 1-4 writes per UserBootstrap per 30 s.
#pragma once

#include <array>
#include <chrono>
#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "core/env_config.h"
#include "core/json.h"
#include "core/threadpool.h"
#include "kube/client.h"
#include "kube/leader.h"
#include "kube/events.h"
#include "kube/runtime.h"

namespace bgc::controller {

constexpr const char* kFieldManager = "bacchus-gpu-controller.bacchus.io";
// Label put on every child this controller applies (CONF_LABEL_CHILDREN): the owned-kind
// watches then select only these, so the apiserver filters events server-side instead of
// streaming every Namespace/ResourceQuota/Role/RoleBinding in the cluster to the
// controller (the reference's .owns() watches all of them, controller.rs:235-238).
constexpr const char* kManagedByLabel = "app.kubernetes.io/managed-by";
constexpr const char* kManagedByValue = "bacchus-gpu-controller";

struct Config {
  std::string listen_addr = "0.0.0.0";
  uint16_t listen_port = 12322;
  int workers = 8;  // 8 against 16: -17 % controller CPU, -21 % reconcile p99 (profiles/r6_workers_ab/)
  bool skip_unchanged = true;
  bool parallel_children = true;
  int64_t requeue_secs = 30;
  // Server-side verification period of each UserBootstrap's children (CONF_RESYNC_SECS;
  // 0 = trust the watch cache for good).  The first one after a UserBootstrap's first
  // reconcile is spread over [0.75, 1] of the period.
  int64_t resync_secs = 300;
  int64_t error_requeue_ms = 3000;
  // Optional per-UB exponential backoff on errors: the n-th consecutive
  // failure requeues after min(error_requeue_ms, base * 2^(n-1)), so a transient apiserver
  // error is retried in milliseconds while a persistent one settles at the reference's
  // 3 s.  0 = the reference's fixed error_requeue_ms (controller.rs:174).
  int64_t error_backoff_base_ms = 0;
  int64_t child_delete_delay_ms = 50;
  // kube::Controller::Options::debounce (CONF_DEBOUNCE_MS).  0 (kube-runtime's default):
  // every event reconciles at once.  1 ms merges the synchronizer's back-to-back quota and
  // status writes into one reconcile (3.0 -> 2.1 reconciles, controller CPU -15-23 % per CR)
  // at the price of a higher reconcile p99, since the merged reconcile applies the
  // ResourceQuota and then the RoleBinding (profiles/controller_cpu_r4/ab_applyrv/).
  int64_t debounce_ms = 0;
  bool label_children = true;  // see kManagedByLabel
  // Child watches ask for PartialObjectMetadata only: the controller reads a child's
  // resourceVersion and ownerReferences, never its spec (kube-rs metadata_watcher).
  bool metadata_watches = true;
  // Warning Events (kubectl describe userbootstrap) for failed reconciles.
  bool events = true;
  // UserBootstrap watch events parsed through user_bootstrap_event_projection().
  bool projected_watch = true;
  kube::LeaseSettings lease;  // optional leader election (CONF_LEADER_ELECTION, ...)
  // reference fields are required (controller.rs:24-28); the rest default
  static Config from_env(const EnvConfig& env);
};

struct DesiredChild {
  const kube::ResourceType* rt;
  std::string ns;
  std::string name;
  std::string body;  // the apply body, JSON text
};

// Pure planning step: the children the reference would apply for `ub`, in its order.
// Throws std::runtime_error("missing object key: .metadata.name") like
// ControllerError::MissingObjectKey.
// With `label`, every child also carries kManagedByLabel=kManagedByValue.
std::vector<DesiredChild> desired_children(const json::Value& ub, bool label = false);
// The owned-kind watch selector matching those labels.
std::string child_label_selector();
// What a reconcile reads from a UserBootstrap watch event: type, apiVersion, kind,
// metadata.{name,namespace,uid,resourceVersion,generation,deletionTimestamp}, spec and
// status (reference controller.rs:50-155).  Everything else (managedFields, annotations,
// labels) is stepped over and left out of the cached object.
const json::Projection& user_bootstrap_event_projection();
// What the controller reads from a child's watch event: type and the child's
// metadata.{name,namespace,resourceVersion,ownerReferences,deletionTimestamp}.
const json::Projection& child_event_projection();
json::Value controller_owner_ref(const json::Value& ub);

class Reconciler {
 public:
  Reconciler(kube::KubeClient& client, kube::Controller& ctrl, Config cfg);
  kube::Action reconcile(const kube::ObjPtr& ub);
  kube::Action error_policy(const kube::ObjPtr& ub, const std::exception& err);
  // True when `child` is exactly the object our last apply returned (same resourceVersion):
  // the watch echo of our own write, which needs no reconcile.
  bool is_own_write(const kube::ResourceType& rt, const json::Value& child) const;
  // Test hook: runs after an apply returns and before its result is recorded (the window in
  // which a watch event of the same child can overtake the record).
  void set_after_apply_hook(std::function<void(const DesiredChild&)> h) { after_apply_ = std::move(h); }
  // Drops the last-applied record of a deleted child (keeps the cache bounded under churn).
  void forget(const kube::ResourceType& rt, const json::Value& child);
  // The UserBootstrap itself is gone: drop its fast-path state and its children's apply
  // records (their DELETED events may be missed across a watch relist).
  void forget_owner(const std::string& owner);
  size_t cached_children() const;
  // Optional (null = no Events): failed reconciles are recorded on the UserBootstrap.
  void set_event_recorder(kube::EventRecorder* r) { events_ = r; }

  struct Stats {
    uint64_t applied = 0;
    uint64_t skipped = 0;
    uint64_t verified = 0;  // children read back from the apiserver by a resync
    uint64_t repaired = 0;  // of those, re-applied because they had drifted or were gone
  };
  Stats stats() const;

 private:
  struct Applied {
    std::string body_hash;
    std::string rv;       // what our apply returned
    std::string prev_rv;  // what the watch cache showed just before it (prev_present)
    bool prev_present = false;
    std::chrono::steady_clock::time_point at{};  // when the apply returned
  };
  // Fast path for periodic resyncs: after a fully successful reconcile, the UB's
  // resourceVersion and each child's resourceVersion. A later reconcile of the same UB
  // version whose children are still at those versions in the watch cache does nothing.
  struct ChildRef {
    const kube::ResourceType* rt;
    std::string ns, name, rv;
  };
  struct UbState {
    std::string owner_rv;
    std::vector<ChildRef> children;
    std::chrono::steady_clock::time_point next_resync{};  // next server-side verification
  };
  // The per-tenant records, split into lock shards by namespace name: a child watch event
  // (is_own_write), a reconcile's checks and applies and a deletion (forget) touch one
  // tenant's shard only, so 16 workers and 5 watch threads rarely meet on a lock.
  struct Shard {
    std::mutex mu;
    std::unordered_map<std::string, Applied> last_applied;  // "plural/ns/name"
    std::unordered_map<std::string, UbState> ub_state;      // owner name
    std::unordered_map<std::string, int> failures;          // consecutive errors per UB (backoff)
    // Applies in flight, by child key: true once a forget() of that child ran meanwhile (its
    // DELETED event overtook the apply's response), so the apply's result is not recorded.
    std::unordered_map<std::string, bool> applying;
  };
  static constexpr size_t kShards = 64;
  Shard& shard(const std::string& ns_name) const;
  void erase_applied_locked(Shard& sh, const std::string& key);
  void erase_owner_state_locked(Shard& sh, const std::string& owner);
  void forget_owner_locked(Shard& sh, const std::string& owner);  // sh.mu held
  void publish_cache_sizes();
  bool up_to_date(const DesiredChild& c, const std::string& body_hash);
  // Stage order: Namespace, then ResourceQuota ‖ Role, then RoleBinding.
  void apply_all(const std::vector<DesiredChild>& children, const std::function<void(size_t)>& run_one);
  bool owner_live(const std::string& name, const std::string& uid);
  bool fresh(const std::string& owner_name, const std::string& owner_rv);
  // The owner has fast-path state and its server-side verification is due.
  bool resync_due(const std::string& owner_name);
  std::chrono::steady_clock::time_point next_resync_time();
  // Resync: reads the child from the apiserver; true (and records it as applied) when it
  // still carries everything `c.body` applies, false when it must be re-applied.
  bool verified_in_sync(const DesiredChild& c, const std::string& body_hash);
  std::function<void(const DesiredChild&)> after_apply_;
  kube::EventRecorder* events_ = nullptr;
  void apply_child(const DesiredChild& c, const std::string& body_hash, const std::string& body_json);

  kube::KubeClient& client_;
  kube::Controller& ctrl_;
  Config cfg_;
  ThreadPool pool_;
  mutable std::array<Shard, kShards> shards_;
  std::atomic<size_t> applied_entries_{0}, owner_entries_{0};
  std::atomic<uint64_t> stats_applied_{0}, stats_skipped_{0}, stats_verified_{0}, stats_repaired_{0};
};

}  // namespace bgc::controller

// Sheet -> UserBootstrap quota/status synchronizer (reference src/synchronizer.rs:171-337).
//
// Reference semantics kept: every `sync_interval_secs` (first tick immediate) export the
// sheet as CSV, keep rows whose gpu_server contains `gpu_server_name`, and for each
// UserBootstrap with an authorized row (last match wins) write spec.quota (JSON Patch:
// add {} if absent, then replace) and status.synchronized_with_sheet=true.  Any error — a
// sheet export, the LIST, a status PUT or a quota PATCH, in the periodic tick or in a watch
// worker — ends the process (kubelet restarts it; SURVEY Q7, reference
// src/synchronizer.rs:302-330,426-430) unless CONF_EXIT_ON_ERROR=false, which retries a
// failed UserBootstrap with per-key exponential backoff under a global retry budget.
//
// Changes (end state identical):
//  * Q5: quota is written BEFORE status, closing the window in which the controller could
//    bind a user into a namespace without a ResourceQuota;
//  * Q6: a UserBootstrap already carrying the desired quota and synced status is not
//    rewritten every tick (no resourceVersion churn, no reconcile storm);
//  * watch mode (CONF_WATCH, default on): new/changed UserBootstraps are synced as soon as
//    they appear, against the last fetched sheet (re-fetched at most every
//    CONF_MIN_REFRESH_MS for unknown users), instead of waiting up to a full interval —
//    apply->Ready drops from ~U(0, 60 s) to milliseconds;
//  * O(1) row lookup per UserBootstrap (hash index) instead of a reverse scan.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>
#include <string>

#include "core/cancel.h"
#include "core/env_config.h"
#include "kube/client.h"
#include "kube/leader.h"
#include "kube/runtime.h"
#include "sync/google.h"
#include "sync/sheet.h"

namespace bgc::sync {

constexpr const char* kPatchManager = "bacchus-gpu-controller.bacchus.io";

struct Config {
  std::string listen_addr;
  uint16_t listen_port = 12323;
  std::string google_service_account_json_path;
  std::string google_file_id;
  uint64_t sync_interval_secs = 60;
  std::string gpu_server_name;
  // additions
  QuotaKeys quota_keys;
  bool watch = true;
  uint64_t min_refresh_ms = 5000;
  // Watch mode: poll the sheet's Drive `version` (a metadata call) this often and export
  // only when it changed, so an operator's approval reaches the cluster within about one
  // poll instead of one sync tick (reference: export every 60 s tick only).  0 = off.
  uint64_t sheet_poll_ms = 5000;
  bool exit_on_error = true;
  // exit_on_error=false: retry a failed UserBootstrap after base * 2^(n-1) ms (capped),
  // all retries together at most retry_qps with retry_burst (client-go's defaults)
  uint64_t retry_base_ms = 5;
  uint64_t retry_max_ms = 60000;
  double retry_qps = 10;
  int retry_burst = 100;
  bool skip_unchanged = true;
  int workers = 8;
  // Lease-based leader election (reference: none; two synchronizer replicas would both
  // write every tenant).  Off by default like the controller's.
  kube::LeaseSettings lease;
  static Config from_env(const EnvConfig& env);
};

struct TickStats {
  size_t rows = 0;
  size_t target_rows = 0;
  size_t userbootstraps = 0;
  size_t matched = 0;
  size_t written = 0;
};

// Source of the sheet CSV (Drive in production; a lambda in tests).
using SheetSource = std::function<std::string()>;

class Synchronizer {
 public:
  Synchronizer(kube::KubeClient& client, SheetSource source, Config cfg);
  // Fetch + parse + index. Throws on fetch/parse errors.
  void refresh();
  // refresh() when the index is older than min_refresh_ms; concurrent callers share one
  // export.  Returns true when this call downloaded the sheet.
  bool refresh_if_stale();
  // One reference-style pass over every UserBootstrap. Throws on the first error.
  TickStats tick();
  // Syncs one UserBootstrap object against the current index; returns true if it wrote.
  // Writes quota then status for one UserBootstrap. Returns true when it wrote; `produced`
  // receives the resourceVersions of the versions its own writes created.
  bool sync_one(const json::Value& ub, std::vector<std::string>* produced = nullptr);
  // Main loop; returns non-zero exit status on fatal error.
  int run(CancelToken& stop);
  // Cheap change detector for the sheet (Drive file version); enables sheet_poll_ms.
  void set_version_source(std::function<std::string()> v) { version_source_ = std::move(v); }

 private:
  std::shared_ptr<const RowIndex> index() const;
  void refresh_locked();  // refresh_mu_ held
  std::string known_version() const;  // Drive version read with the last export
  kube::KubeClient& client_;
  SheetSource source_;
  std::function<std::string()> version_source_;
  Config cfg_;
  mutable std::mutex mu_;
  std::shared_ptr<const RowIndex> index_;
  std::string known_version_;  // guarded by mu_
  std::atomic<int64_t> last_refresh_ns_{0};
  std::atomic<uint64_t> index_gen_{0};  // bumped by every refresh() that read a changed sheet
  std::atomic<size_t> csv_digest_{0};   // hash of the last sheet export read
  std::mutex refresh_mu_;
};

}  // namespace bgc::sync

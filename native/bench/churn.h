// Native churn driver for the headline benchmark (BASELINE.json: "reconcile p99 (ms) +
// admission p50 (ms); CR apply->Ready/sec").
//
// One driver per benchmark rank.  It creates UserBootstraps as OIDC users (through the
// apiserver -> TLS webhook path, exactly like `kubectl apply` by a tenant), and watches
// Namespaces, ResourceQuotas and RoleBindings to timestamp "Ready" — the harness
// definition from BASELINE.md: Namespace, ResourceQuota (with the GPU key) and
// RoleBinding all exist.  Everything runs on native threads so the load generator is
// never the bottleneck being measured.
#pragma once

#include <array>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "core/cancel.h"
#include "core/http.h"
#include "core/json.h"
#include "core/threadpool.h"
#include "kube/client.h"

namespace bgc::bench {

struct ChurnOptions {
  std::string server;
  std::string admin_token;
  std::string ca_pem;  // trust root for an HTTPS apiserver
  std::string user_prefix = "oidc:";
  std::string group = "gpu";
  std::string gpu_quota_key = "requests.amd.com/gpu";
  int concurrency = 32;
  std::string name_prefix;  // only names with this prefix are tracked (one driver per rank)
  // Ask kube-lite to filter the child watches by name_prefix on the server (its
  // kube-lite.test/name-prefix field selector), so N per-rank drivers do not receive, and
  // the server does not encrypt and write, every other rank's child events.
  bool server_filter = false;
  // Approve-after-create (the reference's real onboarding order):
  // when set, a step first waits for every tenant's Namespace, then approves the whole
  // batch with one sheet edit (POST {"rows":[{"id_username":...}],"append":true} to this
  // URL, the fake Google's operator endpoint), then waits for Ready.
  std::string approve_url;
  // Tenant creates and admin deletes over HTTP/2 (one multiplexed connection each), as
  // kubectl/client-go talk to a TLS apiserver; false = HTTP/1.1 keep-alive pools.
  bool http2 = false;
};

class ChurnDriver {
 public:
  explicit ChurnDriver(ChurnOptions o);
  ~ChurnDriver();
  void start();
  // Creates every name concurrently and waits for all to be Ready (or timeout).
  // Returns {"ready": n, "failed": n, "timeouts": n, "elapsed_s": x,
  //          "ready_latency_s": [...], "create_latency_s": [...], "ns_latency_s": [...],
  //          "rq_latency_s": [...], "rb_latency_s": [...], "errors": [...]}; with approve_url
  //          also "approve_to_ready_latency_s" and "approve_latency_s" (create -> approval).
  json::Value step(const std::vector<std::string>& names, double timeout_s);
  // Same, while deleting `previous` concurrently (churn: the previous step's tenants
  // leave while the next ones arrive); the step ends when both are done.
  json::Value step_with_delete(const std::vector<std::string>& names, const std::vector<std::string>& previous,
                               double timeout_s);
  // Open loop: the creates arrive as a Poisson process of rate names.size() / duration_s,
  // whatever the system's progress (arrival times: sorted uniforms over the window, i.e.
  // a Poisson process conditioned on that many arrivals), each tenant is deleted once
  // Ready, and latencies count from the scheduled arrival, so a lagging system shows up as
  // latency instead of as a lower offered rate (no coordinated omission).  Waits for every
  // tenant (or timeout).  Returns step()'s fields plus "offered_rate", "achieved_rate"
  // (Ready tenants / first arrival to last Ready) and "issue_lag_p99_s" (how late the
  // dispatcher issued creates).
  json::Value open_loop(const std::vector<std::string>& names, double duration_s, double timeout_s, uint64_t seed);
  // Deletes (as cluster admin) concurrently; returns number of failures.
  int remove(const std::vector<std::string>& names);
  void stop();

 private:
  struct Track {
    int64_t t_start = 0;
    int64_t t_created = 0;
    int64_t t_approved = 0;
    int64_t t_ns = 0, t_rq = 0, t_rb = 0;
    bool failed = false;
    bool delete_when_ready = false;  // open loop: the tenant leaves once Ready
    std::string error;
  };
  void mark(const std::string& name, int which, int64_t t);
  void issue_delete(const std::string& name);  // asynchronous, on delete_pool_
  // Approve-after-create: waits for the batch's Namespaces, then edits the sheet once.
  void approve_batch(const std::vector<std::string>& names, std::chrono::steady_clock::time_point deadline);
  bool ready_locked(const Track& t) const { return t.t_ns && t.t_rq && t.t_rb; }

  ChurnOptions opts_;
  std::unique_ptr<kube::KubeClient> admin_;
  std::unique_ptr<http::Client> http_;
  std::unique_ptr<ThreadPool> pool_;
  std::unique_ptr<ThreadPool> delete_pool_;
  CancelToken stop_;
  std::vector<std::thread> watchers_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::unordered_map<std::string, Track> tracks_;
  // events that arrived before the step registered the name
  std::unordered_map<std::string, std::array<int64_t, 3>> early_;
  std::atomic<int> delete_failures_{0};
};

}  // namespace bgc::bench

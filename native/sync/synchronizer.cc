#include "sync/synchronizer.h"

#include <algorithm>
#include <atomic>
#include <iterator>
#include <thread>
#include <unordered_map>

#include "core/http.h"
#include "core/json_patch.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/stall.h"
#include "core/trace.h"
#include "kube/ratelimit.h"
#include "core/process.h"

namespace bgc::sync {

using json::Value;
namespace types = kube::types;

Config Config::from_env(const EnvConfig& env) {
  Config c;
  c.listen_addr = env.str("listen_addr");
  c.listen_port = env.u16("listen_port");
  c.google_service_account_json_path = env.str("google_service_account_json_path");
  c.google_file_id = env.str("google_file_id");
  c.sync_interval_secs = env.u64_or("sync_interval_secs", 60);
  c.gpu_server_name = env.str("gpu_server_name");
  c.quota_keys.gpu_resource = env.str_or("gpu_resource_name", "amd.com/gpu");
  c.quota_keys.partition_resource = env.str_or("partition_resource_name", "amd.com/gpu-partition");
  c.watch = env.boolean_or("watch", true);
  c.min_refresh_ms = env.u64_or("min_refresh_ms", 5000);
  c.sheet_poll_ms = env.u64_or("sheet_poll_ms", c.sheet_poll_ms);
  c.exit_on_error = env.boolean_or("exit_on_error", true);
  c.skip_unchanged = env.boolean_or("skip_unchanged", true);
  c.workers = static_cast<int>(env.u64_or("workers", 8));
  c.retry_base_ms = env.u64_or("retry_base_ms", c.retry_base_ms);
  c.retry_max_ms = env.u64_or("retry_max_ms", c.retry_max_ms);
  c.retry_qps = env.f64_or("retry_qps", c.retry_qps);
  c.retry_burst = static_cast<int>(env.u64_or("retry_burst", static_cast<uint64_t>(c.retry_burst)));
  c.lease = kube::LeaseSettings::from_env(env, "bacchus-gpu-synchronizer");
  if (c.sync_interval_secs == 0) throw ConfigError("invalid value for field sync_interval_secs: must be > 0");
  return c;
}

Synchronizer::Synchronizer(kube::KubeClient& client, SheetSource source, Config cfg)
    : client_(client), source_(std::move(source)), cfg_(std::move(cfg)), index_(std::make_shared<RowIndex>()) {}

std::shared_ptr<const RowIndex> Synchronizer::index() const {
  std::lock_guard<std::mutex> lk(mu_);
  return index_;
}

static metrics::Counter& drive_exports(const char* reason) {
  return metrics::Registry::global().counter("bgc_drive_exports_total", "Google Drive sheet exports issued",
                                             {{"reason", reason}});
}

// Readiness ("sheet" check behind /readyz): the last sheet export that succeeded, and how old
// it may get.  Process-wide, like the registry the check lives in.
static std::atomic<int64_t> g_sheet_ok_ns{0};
static std::atomic<int64_t> g_sheet_stale_ms{0};

static bool sheet_ready(std::string* why) {
  const int64_t ok = g_sheet_ok_ns.load();
  if (ok == 0) {
    if (why) *why = "the sheet has not been read yet";
    return false;
  }
  const int64_t age_ms = (metrics::now_ns() - ok) / 1000000;
  if (age_ms > g_sheet_stale_ms.load()) {
    if (why) *why = "last successful sheet read " + std::to_string(age_ms / 1000) + " s ago";
    return false;
  }
  return true;
}

void Synchronizer::refresh() {
  std::lock_guard<std::mutex> rl(refresh_mu_);
  static auto& tick_exports = drive_exports("tick");
  tick_exports.inc();
  refresh_locked();
}

bool Synchronizer::refresh_if_stale() {
  // Single flight: every worker that finds an unknown user queues here, and only the first
  // one past the lock re-downloads; the rest see the fresh timestamp and reuse its index.
  // A burst of unapproved UserBootstraps therefore costs at most one export per
  // min_refresh_ms (the reference exports once per 60 s tick only).
  auto stale = [&] {
    int64_t last = last_refresh_ns_.load();
    return last != 0 && (metrics::now_ns() - last) / 1000000 >= static_cast<int64_t>(cfg_.min_refresh_ms);
  };
  if (!stale()) return false;
  std::lock_guard<std::mutex> rl(refresh_mu_);
  if (!stale()) return false;
  static auto& on_demand = drive_exports("on_demand");
  on_demand.inc();
  refresh_locked();
  return true;
}

void Synchronizer::refresh_locked() {
  // The sheet's Drive version goes with the export it describes, so the version poller's
  // baseline is the version this export read — not whatever its own first poll, one
  // sheet_poll_ms later, finds (an edit in between would otherwise wait for the next tick).
  std::string version;
  if (version_source_) {
    try {
      version = version_source_();
    } catch (const std::exception& e) {
      LOG_WARN("synchronizer") << "sheet version read failed: " << e.what();
    }
  }
  std::string csv = source_();
  LOG_INFO("synchronizer") << "downloaded csv file";
  std::vector<std::string> warnings;
  auto rows = parse_csv(csv, &warnings);
  for (const auto& w : warnings) LOG_WARN("synchronizer") << w;
  auto idx = std::make_shared<RowIndex>(rows, cfg_.gpu_server_name);
  LOG_INFO("synchronizer") << "target rows: " << idx->target_rows();
  metrics::Registry::global().gauge("bgc_sync_rows", "Sheet rows targeting this GPU server").set(static_cast<double>(idx->target_rows()));
  {
    std::lock_guard<std::mutex> lk(mu_);
    index_ = idx;
  }
  last_refresh_ns_.store(metrics::now_ns());
  g_sheet_ok_ns.store(last_refresh_ns_.load());
  // A new generation re-evaluates every UserBootstrap (the echo filter's decisions were made
  // against the old rows); an unchanged sheet (the periodic tick's re-read) keeps them, so
  // a tenant whose own writes have not echoed yet is not written a second time.
  const size_t digest = std::hash<std::string>{}(csv);
  if (digest != csv_digest_.exchange(digest) || index_gen_.load() == 0) index_gen_.fetch_add(1);
  std::lock_guard<std::mutex> lk(mu_);
  known_version_ = version;
}

std::string Synchronizer::known_version() const {
  std::lock_guard<std::mutex> lk(mu_);
  return known_version_;
}

bool Synchronizer::sync_one(const Value& ub, std::vector<std::string>* produced) {
  const std::string name = ub.get("metadata").get_string("name");
  if (name.empty()) return false;
  auto idx = index();
  const Row* row = idx->find(name);
  if (!row) return false;
  Value desired = quota_spec(*row, cfg_.quota_keys);
  const Value& quota = ub.get("spec").get("quota");
  bool has_quota = !quota.is_null();
  bool quota_same = has_quota && quota == desired;
  const Value& st = ub.get("status");
  bool synced = st.is_object() && st.get("synchronized_with_sheet").is_bool() && st.get("synchronized_with_sheet").as_bool();
  if (cfg_.skip_unchanged && quota_same && synced) return false;

  LOG_INFO("synchronizer") << "updating quota id_username=" << row->id_username << " cpu_request=" << row->cpu_request
                           << " memory_request=" << row->memory_request << " gpu_request=" << row->gpu_request
                           << " storage_request=" << row->storage_request << " mig_request=" << row->mig_request;
  LOG_DEBUG("synchronizer") << "row name=" << row->name << " department=" << row->department;
  std::string rv = ub.get("metadata").get_string("resourceVersion");
  // A UserBootstrap deleted while it is being synchronized (its owner onboarded and left,
  // or the cache still showed it) has nothing left to synchronize: NotFound ends this sync
  // without failing it.  Every other error keeps the reference's exit-on-error (Q7).
  try {
    if (!quota_same || !cfg_.skip_unchanged) {
      json::PatchBuilder ops;
      if (!has_quota) ops.add("/spec/quota", Value::object());
      ops.replace("/spec/quota", desired);
      if (trace::armed()) trace::mark(name, "sync.quota.send");
      rv = client_.patch_json_rv(types::UserBootstrap, "", name, ops.ops(), kPatchManager);
      if (trace::armed()) trace::mark(name, "sync.quota.done");
      if (produced) produced->push_back(rv);
      LOG_INFO("synchronizer") << "quota updated";
    }
    if (!synced || !cfg_.skip_unchanged) {
      for (int attempt = 0; attempt < 3; ++attempt) {
        Value body = Value::object({{"apiVersion", "bacchus.io/v1"}, {"kind", "UserBootstrap"}});
        body["metadata"] = Value::object({{"name", name}, {"resourceVersion", rv}});
        body["status"] = Value::object({{"synchronized_with_sheet", true}});
        try {
          LOG_INFO("synchronizer") << "updating status";
          if (trace::armed()) trace::mark(name, "sync.status.send");
          const std::string written_rv = client_.replace_status_rv(types::UserBootstrap, "", name, body);
          if (trace::armed()) trace::mark(name, "sync.status.done");
          if (produced) produced->push_back(written_rv);
          break;
        } catch (const kube::ApiError& e) {
          if (e.code() != 409 || attempt == 2) throw;
          rv = client_.get(types::UserBootstrap, "", name).get("metadata").get_string("resourceVersion");
        }
      }
    }
  } catch (const kube::ApiError& e) {
    if (e.code() != 404) throw;
    static auto& gone = metrics::Registry::global().counter(
        "bgc_sync_deleted_during_sync_total", "UserBootstraps deleted while their synchronization was in flight");
    gone.inc();
    LOG_INFO("synchronizer") << "userbootstrap " << name << " was deleted during synchronization";
    return false;
  }
  static auto& written = metrics::Registry::global().counter("bgc_sync_writes_total", "UserBootstraps written by the synchronizer");
  written.inc();
  return true;
}

TickStats Synchronizer::tick() {
  auto& reg = metrics::Registry::global();
  static auto& hist = reg.histogram("bgc_sync_duration_seconds", "Wall time of one synchronization tick");
  static auto& ring = reg.samples("sync_tick");
  metrics::Timer timer(&hist, &ring);
  LOG_INFO("synchronizer") << "starting synchronization";
  refresh();
  TickStats ts;
  auto idx = index();
  ts.target_rows = idx->target_rows();
  Value list = client_.list(types::UserBootstrap);
  for (const auto& ub : list.get("items").items()) {
    ++ts.userbootstraps;
    if (idx->find(ub.get("metadata").get_string("name"))) ++ts.matched;
    if (sync_one(ub)) ++ts.written;
  }
  return ts;
}

// What sync_one reads from a UserBootstrap watch event (reference synchronizer.rs:218-330:
// the name, the resourceVersion for the status PUT, spec.quota to compare, status): the rest
// of the object (managedFields, annotations, the rest of the spec) is stepped over.
static const json::Projection& ub_watch_projection() {
  using P = json::Projection;
  static const P kMeta[] = {{"name", P::Keep}, {"namespace", P::Keep}, {"uid", P::Keep}, {"resourceVersion", P::Keep}};
  static const P kSpec[] = {{"quota", P::Keep}};
  static const P kObject[] = {{"apiVersion", P::Keep},
                              {"kind", P::Keep},
                              {"metadata", P::Descend, kMeta, std::size(kMeta), true},
                              {"spec", P::Descend, kSpec, std::size(kSpec), true},
                              {"status", P::Keep}};
  static const P kEvent[] = {{"type", P::Keep}, {"object", P::Descend, kObject, std::size(kObject), true}};
  static const P kRoot{"", P::Descend, kEvent, std::size(kEvent), true};
  return kRoot;
}

int Synchronizer::run(CancelToken& stop) {
  // Not ready until a sheet read succeeded, nor after three sync intervals without one (with
  // CONF_EXIT_ON_ERROR=false a synchronizer that cannot reach Google stays up, retrying).
  g_sheet_stale_ms.store(std::max<int64_t>(3000, 3000 * static_cast<int64_t>(cfg_.sync_interval_secs)));
  http::add_readiness_check("sheet", sheet_ready);
  std::unique_ptr<std::thread> watch_thread;
  std::vector<std::thread> workers;
  kube::WorkQueue queue(kube::WorkQueue::shards_for(cfg_.workers));
  kube::Store store(types::UserBootstrap);
  std::atomic<bool> fatal{false};
  auto& ub_latency = metrics::Registry::global().samples("sync_ub");
  // resourceVersion of the UB version we last wrote for: a deferred re-offer of that same
  // version (the watch has not yet delivered our own writes) needs no second look
  std::mutex acted_mu;
  struct Acted {
    uint64_t sheet_gen;                 // a newer sheet re-evaluates every UB
    std::vector<std::string> versions;  // UB versions acted on or produced by our writes
  };
  std::unordered_map<std::string, Acted> acted;
  static auto& tracked = metrics::Registry::global().gauge(
      "bgc_sync_tracked_userbootstraps", "UserBootstraps with a remembered sync (dropped when one is deleted)");
  // CONF_EXIT_ON_ERROR=false only: per-UserBootstrap exponential backoff plus an overall
  // retry budget (client-go's controller rate limiter) instead of a fixed delay
  kube::RetryLimiter retries(std::chrono::milliseconds(cfg_.retry_base_ms), std::chrono::milliseconds(cfg_.retry_max_ms),
                             cfg_.retry_qps, cfg_.retry_burst);
  static auto& retried = metrics::Registry::global().counter("bgc_sync_retries_total",
                                                             "UserBootstrap syncs re-queued after a failure");

  if (cfg_.watch) {
    watch_thread = std::make_unique<std::thread>([&] {
      kube::Watcher w(client_, types::UserBootstrap);
      w.set_projection(&ub_watch_projection());
      w.run(stop, [&](const kube::WatchEvent& ev) {
        // marked before the store applies it: a queued worker may read the store at once
        if (trace::armed() && ev.object && ev.type != kube::WatchEvent::Type::Deleted) {
          trace::mark(kube::meta_name(*ev.object), "sync.ub_event");
        }
        const int64_t t0 = metrics::now_ns();
        store.apply(ev);
        const int64_t t1 = metrics::now_ns();
        stall::note_lock_section("w:userbootstraps store", t0, t1);
        if (ev.type == kube::WatchEvent::Type::Restarted) {
          for (const auto& o : ev.objects) queue.add(kube::meta_name(*o));
        } else if (ev.type != kube::WatchEvent::Type::Deleted) {
          queue.add(kube::meta_name(*ev.object));
          stall::note_lock_section("w:userbootstraps queue", t1, metrics::now_ns());
        } else {
          retries.forget(kube::meta_name(*ev.object));  // a failing UB that is gone retries no more
          std::lock_guard<std::mutex> g(acted_mu);
          acted.erase(kube::meta_name(*ev.object));
          tracked.set(static_cast<double>(acted.size()));
        }
      });
    });
    for (int i = 0; i < std::max(1, cfg_.workers); ++i) {
      workers.emplace_back([&, i] {
        set_thread_name("sync-worker");
        std::string key;
        while (queue.get(key, static_cast<size_t>(i))) {
          kube::ObjPtr ub = store.get(key);
          if (trace::armed()) trace::mark(key, "sync.dequeue");
          if (ub) {
            const std::string ub_rv = kube::meta_rv(*ub);
            {
              std::lock_guard<std::mutex> g(acted_mu);
              auto a = acted.find(key);
              if (a != acted.end() && a->second.sheet_gen == index_gen_.load() &&
                  std::find(a->second.versions.begin(), a->second.versions.end(), ub_rv) != a->second.versions.end()) {
                queue.done(key);
                continue;
              }
            }
            int64_t t0 = metrics::now_ns();
            try {
              auto idx = index();
              // unknown user: the sheet may have changed since the last fetch
              if (!idx->find(key)) refresh_if_stale();
              std::vector<std::string> produced{ub_rv};
              uint64_t gen = index_gen_.load();
              if (sync_one(*ub, &produced)) {
                ub_latency.add(static_cast<double>(metrics::now_ns() - t0) * 1e-9);
                std::lock_guard<std::mutex> g(acted_mu);
                // not for a UB deleted meanwhile: its DELETED event (store first, then
                // this map, under acted_mu) may already have run, and the entry would stay
                if (store.get(key)) acted[key] = Acted{gen, std::move(produced)};
                tracked.set(static_cast<double>(acted.size()));
              }
              retries.forget(key);
            } catch (const std::exception& e) {
              if (cfg_.exit_on_error) {
                // Q7, as the reference: a failed status PUT or spec PATCH returns Err out of
                // synchronize_loop and try_join! ends the process (synchronizer.rs:302-330,
                // 426-430); the kubelet restarts it with crash-loop backoff.
                LOG_ERROR("synchronizer") << "synchronization of " << key << " failed: " << e.what();
                fatal = true;
                stop.cancel();
              } else {
                const auto delay = retries.when(key);
                retried.inc();
                LOG_ERROR("synchronizer") << "sync of " << key << " failed (retry " << retries.failures(key) << " in "
                                          << delay.count() << " ms): " << e.what();
                queue.add_after(key, delay);
              }
            }
          }
          queue.done(key);
        }
      });
    }
  }

  // Sheet change poll (watch mode): a metadata request per sheet_poll_ms, an export only
  // when Drive reports a new version.  Poll errors are logged, never fatal: the periodic
  // tick still re-reads the sheet and keeps the reference's exit-on-error semantics.
  std::unique_ptr<std::thread> poll_thread;
  if (cfg_.watch && cfg_.sheet_poll_ms > 0 && version_source_) {
    poll_thread = std::make_unique<std::thread>([&] {
      static auto& polls = metrics::Registry::global().counter("bgc_drive_version_polls_total",
                                                               "Drive file-version metadata requests");
      static auto& changed = drive_exports("changed");
      while (!stop.wait_for(std::chrono::milliseconds(cfg_.sheet_poll_ms))) {
        try {
          polls.inc();
          std::string v = version_source_();
          // known_version(): what the last export read ("" when that read failed: then
          // any version re-reads, at the cost of one possibly redundant export)
          if (v == known_version()) continue;
          LOG_INFO("synchronizer") << "sheet changed (version " << v << "); re-reading";
          {
            std::lock_guard<std::mutex> rl(refresh_mu_);
            changed.inc();
            refresh_locked();
          }
          for (const auto& o : store.list()) queue.add(kube::meta_name(*o));
        } catch (const std::exception& e) {
          LOG_WARN("synchronizer") << "sheet version poll failed: " << e.what();
        }
      }
    });
  }

  int rc = 0;
  while (!stop.cancelled()) {
    try {
      if (cfg_.watch) {
        // Workers own the writes; a tick refreshes the sheet and re-offers every
        // UserBootstrap so rows approved since the last tick get applied.
        refresh();
        for (const auto& o : store.list()) queue.add(kube::meta_name(*o));
      } else {
        tick();
      }
    } catch (const std::exception& e) {
      LOG_ERROR("synchronizer") << "synchronization failed: " << e.what();
      if (cfg_.exit_on_error) {
        rc = 1;
        fatal = true;
        stop.cancel();
        break;
      }
    }
    if (stop.wait_for(std::chrono::seconds(cfg_.sync_interval_secs))) break;
  }
  if (poll_thread) poll_thread->join();
  queue.shutdown();
  for (auto& t : workers) t.join();
  if (watch_thread) watch_thread->join();
  if (fatal) rc = 1;
  return rc;
}

}  // namespace bgc::sync

#include "kube/runtime.h"

#include <algorithm>

#include "core/http.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/stall.h"
#include "core/trace.h"
#include "core/net.h"
#include "core/process.h"

namespace bgc::kube {

using json::Value;

std::string meta_name(const Value& obj) { return obj.get("metadata").get_string("name"); }
std::string meta_namespace(const Value& obj) { return obj.get("metadata").get_string("namespace"); }
std::string meta_rv(const Value& obj) { return obj.get("metadata").get_string("resourceVersion"); }

// ---------------------------------------------------------------------------
// Watcher

namespace {
std::mutex g_watch_defaults_mu;
Watcher::Defaults g_watch_defaults;

// Liveness of the running watchers, read by the "watches" readiness check.
struct WatchSlot {
  std::string resource;
  int64_t deadline_ms = 0;
  std::atomic<int64_t> last_ns{0};  // last event, bookmark, list or (re)started stream
  std::atomic<bool> synced{false};  // the initial list has been delivered
  // Largest gap seen between two consecutive BOOKMARKs of one stream: the server's
  // heartbeat, once seen (a real apiserver sends one about every minute, kube-lite every
  // --bookmark-ms).  The maximum, not the last gap: the apiserver also sends one bookmark
  // ~2 s before a watch's timeoutSeconds, and that short gap must not make a quiet,
  // healthy watch look stale seconds later.
  std::atomic<int64_t> heartbeat_ns{0};
};

// How long a watch may be silent before it counts as stale for readiness: three missed
// heartbeats once the server's bookmark cadence is known (so a stall shows on /readyz well
// before the idle deadline reconnects it), the idle deadline otherwise.
int64_t stale_after_ms(const WatchSlot& s) {
  const int64_t hb_ms = s.heartbeat_ns.load() / 1000000;
  if (hb_ms <= 0) return s.deadline_ms;
  return std::min(s.deadline_ms, std::max<int64_t>(3 * hb_ms, 2000));
}
std::mutex g_slots_mu;
std::vector<std::shared_ptr<WatchSlot>> g_slots;

bool watches_ready(std::string* why) {
  std::vector<std::shared_ptr<WatchSlot>> slots;
  {
    std::lock_guard<std::mutex> lk(g_slots_mu);
    slots = g_slots;
  }
  const int64_t now = metrics::now_ns();
  bool ok = true;
  for (const auto& s : slots) {
    std::string problem;
    const int64_t age_ms = (now - s->last_ns.load()) / 1000000;
    if (!s->synced.load()) {
      problem = s->resource + ": initial list not complete";
    } else if (s->deadline_ms > 0 && age_ms > stale_after_ms(*s)) {
      problem = s->resource + ": no event or bookmark for " + std::to_string(age_ms) + " ms (stale after " +
                std::to_string(stale_after_ms(*s)) + " ms)";
    }
    if (problem.empty()) continue;
    if (why) *why += (ok ? "" : "; ") + problem;
    ok = false;
  }
  return ok;
}

// Registers a running watcher's slot (and, once per process, the readiness check).
std::shared_ptr<WatchSlot> open_slot(const std::string& resource, int64_t deadline_ms) {
  static std::once_flag registered;
  std::call_once(registered, [] { http::add_readiness_check("watches", watches_ready); });
  auto s = std::make_shared<WatchSlot>();
  s->resource = resource;
  s->deadline_ms = deadline_ms;
  s->last_ns = metrics::now_ns();
  std::lock_guard<std::mutex> lk(g_slots_mu);
  g_slots.push_back(s);
  return s;
}

void close_slot(const std::shared_ptr<WatchSlot>& s) {
  std::lock_guard<std::mutex> lk(g_slots_mu);
  g_slots.erase(std::remove(g_slots.begin(), g_slots.end(), s), g_slots.end());
}
}  // namespace

void Watcher::set_defaults(Defaults d) {
  std::lock_guard<std::mutex> lk(g_watch_defaults_mu);
  g_watch_defaults = d;
}

Watcher::Defaults Watcher::defaults() {
  std::lock_guard<std::mutex> lk(g_watch_defaults_mu);
  return g_watch_defaults;
}

void Watcher::configure_from_env(const EnvConfig& env) {
  Defaults wd;
  wd.page_size = static_cast<int64_t>(env.u64_or("list_page_size", 500));
  wd.streaming_lists = env.boolean_or("streaming_lists", false);
  wd.idle_timeout_ms = static_cast<int64_t>(env.u64_or("watch_idle_timeout_secs", 295)) * 1000;
  set_defaults(wd);
  net::TcpKeepalive k;
  k.idle_s = static_cast<int>(env.u64_or("tcp_keepalive_secs", static_cast<uint64_t>(k.idle_s)));
  k.user_timeout_ms = static_cast<int>(env.u64_or("tcp_user_timeout_secs", 60)) * 1000;
  net::set_tcp_keepalive(k);
}

Watcher::Watcher(KubeClient& client, ResourceType rt, std::string ns, std::string label_selector,
                 std::string field_selector)
    : client_(client),
      rt_(std::move(rt)),
      ns_(std::move(ns)),
      selector_(std::move(label_selector)),
      field_selector_(std::move(field_selector)) {
  const Defaults d = defaults();
  page_size_ = d.page_size;
  streaming_ = d.streaming_lists;
  idle_timeout_ms_ = d.idle_timeout_ms;
}

ObjPtr Watcher::typed(Value obj) const {
  if (metadata_only_) {  // PartialObjectMetadata -> a metadata view of the watched type
    obj["apiVersion"] = rt_.api_version();
    obj["kind"] = rt_.kind;
  }
  if (!obj.contains("apiVersion")) obj["apiVersion"] = rt_.api_version();
  if (!obj.contains("kind")) obj["kind"] = rt_.kind;
  return std::make_shared<const Value>(std::move(obj));
}

std::string Watcher::list_all(std::vector<ObjPtr>& out, CancelToken& stop) {
  for (int attempt = 0;; ++attempt) {
    out.clear();
    ListOptions lo;
    lo.label_selector = selector_;
    lo.field_selector = field_selector_;
    lo.limit = page_size_ > 0 ? page_size_ : 0;
    lo.metadata_only = metadata_only_;
    std::string rv;
    try {
      do {
        Value list = client_.list(rt_, ns_, lo);
        list_pages_.fetch_add(1);
        const Value& meta = list.get("metadata");
        if (rv.empty()) rv = meta.get_string("resourceVersion");  // the first page's snapshot
        lo.continue_token = meta.get_string("continue");
        Value* items = list.find_mut("items");
        if (items && items->is_array()) {
          for (auto& item : items->items_mut()) out.push_back(typed(std::move(item)));
        }
      } while (!lo.continue_token.empty() && !stop.cancelled());
      return rv;
    } catch (const ApiError& e) {
      // 410 on a continue token: the snapshot expired mid-list; start over
      if (e.code() != 410 || lo.continue_token.empty() || attempt >= 3) throw;
      LOG_INFO("kube::watcher") << rt_.plural << ": continue token expired, restarting the list";
    }
  }
}

// ERROR and BOOKMARK watch lines.  The apiserver writes "type" first ({"type":"ADDED",...}),
// so the prefix answers without scanning a multi-kilobyte object; a line in another member
// order falls back to a search of the whole line.
static bool is_control_event(std::string_view line) {
  constexpr std::string_view kPrefix = "{\"type\":\"";
  if (line.substr(0, kPrefix.size()) == kPrefix) {
    const std::string_view t = line.substr(kPrefix.size(), 9);
    return t.substr(0, 6) == "ERROR\"" || t == "BOOKMARK\"";
  }
  return line.find("\"type\":\"ERROR\"") != std::string_view::npos ||
         line.find("\"type\":\"BOOKMARK\"") != std::string_view::npos;
}

void Watcher::run(CancelToken& stop, const std::function<void(const WatchEvent&)>& on_event) {
  set_thread_name("w:" + rt_.plural);
  std::string rv;
  bool need_list = true;
  auto backoff = std::chrono::milliseconds(800);
  const auto max_backoff = std::chrono::milliseconds(30000);
  auto& errors = metrics::Registry::global().counter("bgc_watch_errors_total", "Watch stream failures",
                                                     {{"resource", rt_.plural}});
  auto& idle_expired = metrics::Registry::global().counter(
      "bgc_watch_idle_timeouts_total", "Watch streams closed after their idle deadline passed with no byte received",
      {{"resource", rt_.plural}});
  const std::shared_ptr<WatchSlot> slot = open_slot(rt_.plural + (selector_.empty() ? "" : "{" + selector_ + "}"),
                                                    idle_timeout_ms_);
  struct SlotGuard {
    std::shared_ptr<WatchSlot> s;
    ~SlotGuard() { close_slot(s); }
  } slot_guard{slot};
  auto alive = [&] { slot->last_ns.store(metrics::now_ns(), std::memory_order_relaxed); };
  // sections of this thread that hold up the events queued behind them (stall::note_slow)
  const std::string slow_event = "w:" + rt_.plural + " event", slow_reopen = "w:" + rt_.plural + " reopen";
  int64_t down_ns = 0;  // when the previous stream ended
  while (!stop.cancelled()) {
    // Streaming list: the initial state arrives on this watch; objects collect here until
    // the initial-events-end bookmark.
    bool initial_phase = false;
    std::vector<ObjPtr> initial;
    try {
      if (need_list && !streaming_) {
        WatchEvent ev{WatchEvent::Type::Restarted, nullptr, {}};
        rv = list_all(ev.objects, stop);
        on_event(ev);
        need_list = false;
        relists_.fetch_add(1);
        alive();
        slot->synced.store(true);
      }
      WatchOptions wo;
      wo.label_selector = selector_;
      wo.field_selector = field_selector_;
      wo.metadata_only = metadata_only_;
      if (idle_timeout_ms_ > 0) {
        // the server ends a quiet healthy watch before the client's deadline would (295 s ->
        // the usual 290 s; a short test deadline keeps most of its length)
        const int64_t idle_s = idle_timeout_ms_ / 1000;
        const int64_t margin = std::max<int64_t>(1, std::min<int64_t>(5, idle_s / 10));
        wo.timeout_seconds = static_cast<int>(std::clamp<int64_t>(idle_s - margin, 1, wo.timeout_seconds));
      }
      if (need_list) {  // streaming
        wo.send_initial_events = true;
        initial_phase = true;
      } else {
        wo.resource_version = rv;
      }
      std::unique_ptr<http::StreamingResponse> stream;
      try {
        stream = client_.watch(rt_, ns_, wo);
      } catch (const ApiError& e) {
        if (initial_phase && e.code() >= 400 && e.code() < 500 && e.code() != 410 && e.code() != 429) {
          LOG_WARN("kube::watcher") << rt_.plural << ": streaming lists rejected (" << e.what()
                                    << "); falling back to LIST";
          streaming_ = false;
          continue;
        }
        throw;
      }
      backoff = std::chrono::milliseconds(800);
      if (idle_timeout_ms_ > 0) stream->set_idle_timeout(static_cast<int>(idle_timeout_ms_));
      alive();
      if (down_ns) stall::note_slow(slow_reopen, down_ns, metrics::now_ns());
      down_ns = 0;
      int64_t last_bookmark_ns = 0;
      std::string line;
      while (stream->next_line(line, &stop, 500)) {
        const int64_t read_ns = metrics::now_ns();
        slot->last_ns.store(read_ns, std::memory_order_relaxed);
        if (line.empty()) continue;
        // Events the consumer does not want are dropped before JSON parsing; ERROR and
        // BOOKMARK lines always go through (they drive relists and resumption).  During
        // a streaming list nothing is dropped: the initial state must be complete.
        const bool control = is_control_event(line);
        if (!initial_phase && line_filter_ && !control && !line_filter_(line)) continue;
        // metadata.managedFields is never read from the cache; skipping it while parsing
        // saves most of the allocations of an SSA-managed child's event.
        Value ev = projection_ && !initial_phase && !control ? json::parse_projected(line, *projection_)
                                                            : json::parse(line, "managedFields");
        const std::string type = ev.get_string("type");
        Value* objp = ev.find_mut("object");
        Value obj = objp ? std::move(*objp) : Value();  // no deep copy of the event object
        if (type == "ERROR") {
          int code = obj.get("code").is_int() ? static_cast<int>(obj.get("code").as_int()) : 0;
          if (code == 410) {
            LOG_DEBUG("kube::watcher") << rt_.plural << ": resourceVersion too old, relisting";
          } else {
            LOG_WARN("kube::watcher") << rt_.plural << ": watch error event: " << obj.dump();
          }
          need_list = true;
          break;
        }
        std::string new_rv = meta_rv(obj);
        if (!new_rv.empty()) rv = new_rv;
        if (type == "BOOKMARK") {
          const int64_t now = metrics::now_ns();
          if (last_bookmark_ns) {
            const int64_t gap = now - last_bookmark_ns;
            int64_t cur = slot->heartbeat_ns.load(std::memory_order_relaxed);
            while (gap > cur && !slot->heartbeat_ns.compare_exchange_weak(cur, gap, std::memory_order_relaxed)) {
            }
          }
          last_bookmark_ns = now;
          if (initial_phase &&
              obj.get("metadata").get("annotations").get_string("k8s.io/initial-events-end") == "true") {
            WatchEvent we{WatchEvent::Type::Restarted, nullptr, std::move(initial)};
            initial.clear();
            initial_phase = false;
            need_list = false;
            on_event(we);
            relists_.fetch_add(1);
            slot->synced.store(true);
          }
          continue;
        }
        if (initial_phase) {
          if (type == "ADDED") initial.push_back(typed(std::move(obj)));
          continue;
        }
        WatchEvent we{WatchEvent::Type::Added,
                      metadata_only_ ? typed(std::move(obj)) : std::make_shared<const Value>(std::move(obj)), {},
                      read_ns};
        if (type == "MODIFIED") we.type = WatchEvent::Type::Modified;
        else if (type == "DELETED") we.type = WatchEvent::Type::Deleted;
        else if (type != "ADDED") continue;
        on_event(we);
        stall::note_slow(slow_event, read_ns, metrics::now_ns());
      }
      stream->close();
      down_ns = metrics::now_ns();
      if (stream->idle_timed_out() && !stop.cancelled()) {
        // Nothing arrived for the whole deadline, not even a bookmark: the connection (or the
        // path to the apiserver) is presumed dead.  Pooled request connections share that
        // path, so they go too; the watch resumes from rv on a fresh connection.
        idle_timeouts_.fetch_add(1);
        idle_expired.inc();
        LOG_WARN("kube::watcher") << rt_.plural << ": no event or bookmark for " << idle_timeout_ms_ / 1000
                                  << " s; reconnecting";
        client_.reset_connections();
      }
      if (!stop.cancelled()) reconnects_.fetch_add(1);
    } catch (const ApiError& e) {
      errors.inc();
      if (!down_ns) down_ns = metrics::now_ns();
      if (e.code() == 410) {
        need_list = true;
        continue;
      }
      LOG_WARN("kube::watcher") << rt_.plural << ": " << e.what() << " (retry in " << backoff.count() << "ms)";
      if (stop.wait_for(backoff)) break;
      backoff = std::min(backoff * 2, max_backoff);
      need_list = true;
    } catch (const std::exception& e) {
      errors.inc();
      if (!down_ns) down_ns = metrics::now_ns();
      LOG_WARN("kube::watcher") << rt_.plural << ": " << e.what() << " (retry in " << backoff.count() << "ms)";
      if (stop.wait_for(backoff)) break;
      backoff = std::min(backoff * 2, max_backoff);
    }
  }
}

// ---------------------------------------------------------------------------
// Store

void Store::apply(const WatchEvent& ev) {
  ObjPtr replaced;  // the previous object is freed after the lock is released
  std::lock_guard<std::mutex> lk(mu_);
  struct Count {
    Store* s;
    ~Count() { s->size_.store(s->items_.size(), std::memory_order_relaxed); }
  } count{this};
  switch (ev.type) {
    case WatchEvent::Type::Restarted:
      items_.clear();
      for (const auto& o : ev.objects) items_[rt_.key(meta_namespace(*o), meta_name(*o))] = o;
      synced_.store(true);
      cv_.notify_all();
      break;
    case WatchEvent::Type::Added:
    case WatchEvent::Type::Modified: {
      ObjPtr& slot = items_[rt_.key(meta_namespace(*ev.object), meta_name(*ev.object))];
      replaced = std::move(slot);
      slot = ev.object;
      break;
    }
    case WatchEvent::Type::Deleted: {
      auto it = items_.find(rt_.key(meta_namespace(*ev.object), meta_name(*ev.object)));
      if (it != items_.end()) {
        replaced = std::move(it->second);
        items_.erase(it);
      }
      break;
    }
  }
}

ObjPtr Store::get(const std::string& key) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = items_.find(key);
  return it == items_.end() ? nullptr : it->second;
}

std::vector<ObjPtr> Store::list() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<ObjPtr> out;
  out.reserve(items_.size());
  for (auto& kv : items_) out.push_back(kv.second);
  return out;
}

bool Store::wait_synced(std::chrono::milliseconds timeout) const {
  std::unique_lock<std::mutex> lk(mu_);
  return cv_.wait_for(lk, timeout, [&] { return synced_.load(); });
}

// ---------------------------------------------------------------------------
// WorkQueue

// One shard: the whole queue of round 5, for the keys that hash to it.
//
// Condition variables are signalled after the shard's lock is released (Wake::fire): a
// signal under the lock lengthens every hold by a futex syscall, and the woken worker can
// preempt the signaller on its CPU while the signaller still holds the lock.  A waiter
// re-checks the timeline under the lock before it sleeps, so deciding under the lock and
// signalling after it loses no wake-up.
struct WorkQueue::Shard {
  using Timeline = std::multimap<Clock::time_point, std::string>;
  struct Due {
    Clock::time_point t;
    Timeline::iterator node;
  };
  // Which waiters to signal once the lock is released: one idle worker per item made due
  // (as many as are idle), and the timer waiter at most once.
  struct Wake {
    int workers = 0;
    bool timer = false;
  };

  mutable std::mutex mu;
  // One idle worker (the timer waiter) sleeps until the earliest deadline on timer_cv; the
  // others wait untimed on cv.  A due item wakes one worker, not every idle one.
  std::condition_variable cv;
  std::condition_variable timer_cv;
  int idle = 0;               // workers waiting on cv
  // Signals sent to cv that no waiter has consumed yet.  A woken worker counts as idle
  // until it re-takes the lock, which under CPU contention can be milliseconds.  Without
  // this count, an add in that window signalled cv although every waiter was already woken:
  // the signal reached nobody, the timer waiter was not asked, and the key waited for a busy
  // worker to come back.
  int signaled = 0;
  bool timer_waiter = false;  // a worker is waiting on timer_cv
  Clock::time_point timer_target{};
  // Hash containers: under churn the queue holds a pending 30 s requeue for every live
  // UserBootstrap, and ordered maps paid a chain of string compares per operation.  due and
  // timeline index each other one to one: a key's entry holds its timeline node, so moving
  // or dropping a key erases that node directly, and the common insert, a periodic requeue
  // later than everything queued, goes in at the end with a hint.
  std::unordered_map<std::string, Due> due;  // key -> due time and its timeline node
  Timeline timeline;                         // due time -> key
  std::unordered_set<std::string> processing;
  std::unordered_map<std::string, Clock::time_point> deferred;  // re-added while processing
  std::unordered_set<std::string> forgotten;                    // forgotten while processing
  std::atomic<size_t> pending{0};
  bool shutdown = false;

  void fire(const Wake& w) {
    for (int i = 0; i < w.workers; ++i) cv.notify_one();
    if (w.timer) timer_cv.notify_one();
  }
  void count_locked() { pending.store(due.size() + deferred.size(), std::memory_order_relaxed); }
  void signal_locked(Wake& wake) {
    ++signaled;
    ++wake.workers;
  }

  void schedule_locked(const std::string& key, Clock::time_point t, Wake& wake) {
    auto [d, fresh] = due.try_emplace(key);
    // Moving a key earlier (an event for a key with a pending 30 s requeue) drops its old node.
    if (!fresh) timeline.erase(d->second.node);
    d->second.t = t;
    d->second.node = (timeline.empty() || !(t < timeline.rbegin()->first)) ? timeline.emplace_hint(timeline.end(), t, key)
                                                                           : timeline.emplace(t, key);
    if (t <= Clock::now()) {
      if (idle > signaled) signal_locked(wake);
      else if (timer_waiter) wake.timer = true;
    } else if (timer_waiter) {
      if (t < timer_target) wake.timer = true;  // new earliest deadline
    } else if (idle > signaled) {
      signal_locked(wake);  // someone must become the timer waiter
    }
  }

  void add_after_locked(const std::string& key, Clock::time_point t, Wake& wake) {
    if (shutdown) return;
    if (processing.count(key)) {
      auto it = deferred.find(key);
      if (it == deferred.end() || t < it->second) deferred[key] = t;
      return;
    }
    auto it = due.find(key);
    if (it != due.end() && it->second.t <= t) return;
    schedule_locked(key, t, wake);
  }

  void done_locked(const std::string& key, Wake& wake) {
    processing.erase(key);
    if (!forgotten.empty()) forgotten.erase(key);
    auto it = deferred.find(key);
    if (it != deferred.end()) {
      auto t = it->second;
      deferred.erase(it);
      auto d = due.find(key);
      if (d == due.end() || t < d->second.t) schedule_locked(key, t, wake);
    }
  }
};

WorkQueue::WorkQueue(size_t shards) {
  for (size_t i = 0; i < std::max<size_t>(1, shards); ++i) shards_.push_back(std::make_unique<Shard>());
}

WorkQueue::~WorkQueue() = default;

size_t WorkQueue::shards_for(int workers) {
  // One shard unless BGC_QUEUE_SHARDS says otherwise (at most one per worker, at most 8).
  // The controller's and synchronizer's workers block on API calls, so a shard's few
  // workers queue a burst that the whole pool would have absorbed: sharding cut the lock
  // waits but lengthened event->dequeue tails (profiles/r6_queue_ab/).
  const char* e = std::getenv("BGC_QUEUE_SHARDS");
  const int want = e && *e ? std::atoi(e) : 1;
  return static_cast<size_t>(std::clamp(want, 1, std::clamp(std::max(1, workers), 1, 8)));
}

WorkQueue::Shard& WorkQueue::shard_of(const std::string& key) const {
  return *shards_[shards_.size() == 1 ? 0 : std::hash<std::string>{}(key) % shards_.size()];
}

void WorkQueue::add_after(const std::string& key, std::chrono::milliseconds delay) {
  auto t = Clock::now() + delay;
  Shard& sh = shard_of(key);
  Shard::Wake wake;
  {
    std::lock_guard<std::mutex> lk(sh.mu);
    if (!sh.forgotten.empty()) sh.forgotten.erase(key);
    sh.add_after_locked(key, t, wake);
    sh.count_locked();
  }
  sh.fire(wake);
}

void WorkQueue::requeue(const std::string& key, std::chrono::milliseconds delay) {
  auto t = Clock::now() + delay;
  Shard& sh = shard_of(key);
  Shard::Wake wake;
  {
    std::lock_guard<std::mutex> lk(sh.mu);
    if (!sh.forgotten.empty() && sh.forgotten.count(key)) return;
    sh.add_after_locked(key, t, wake);
    sh.count_locked();
  }
  sh.fire(wake);
}

void WorkQueue::finish(const std::string& key, bool requeue, std::chrono::milliseconds delay) {
  const auto t = Clock::now() + delay;
  Shard& sh = shard_of(key);
  Shard::Wake wake;
  {
    std::lock_guard<std::mutex> lk(sh.mu);
    if (requeue && (sh.forgotten.empty() || !sh.forgotten.count(key))) sh.add_after_locked(key, t, wake);
    sh.done_locked(key, wake);
    sh.count_locked();
  }
  sh.fire(wake);
}

void WorkQueue::forget(const std::string& key) {
  Shard& sh = shard_of(key);
  std::lock_guard<std::mutex> lk(sh.mu);
  sh.deferred.erase(key);
  if (sh.processing.count(key)) sh.forgotten.insert(key);
  auto d = sh.due.find(key);
  if (d != sh.due.end()) {
    sh.timeline.erase(d->second.node);
    sh.due.erase(d);
  }
  sh.count_locked();
}

bool WorkQueue::get(std::string& key, size_t worker) {
  Shard& sh = *shards_[worker % shards_.size()];
  std::unique_lock<std::mutex> lk(sh.mu);
  while (true) {
    if (sh.shutdown) return false;
    auto now = Clock::now();
    if (!sh.timeline.empty() && !(sh.timeline.begin()->first > now)) {
      auto it = sh.timeline.begin();
      key = std::move(it->second);
      sh.timeline.erase(it);
      sh.due.erase(key);
      sh.processing.insert(key);
      sh.count_locked();
      // hand the timer role on if more work is waiting and nobody is timing it
      const bool hand_on = !sh.timeline.empty() && !sh.timer_waiter && sh.idle > sh.signaled;
      if (hand_on) ++sh.signaled;
      lk.unlock();
      if (hand_on) sh.cv.notify_one();
      return true;
    }
    if (!sh.timeline.empty() && !sh.timer_waiter) {
      sh.timer_waiter = true;
      // copy: wait_until re-reads its deadline after re-locking, when another worker may have erased the node
      sh.timer_target = sh.timeline.begin()->first;
      const auto deadline = sh.timer_target;
      sh.timer_cv.wait_until(lk, deadline);
      sh.timer_waiter = false;
    } else {
      ++sh.idle;
      sh.cv.wait(lk);
      --sh.idle;
      if (sh.signaled > 0) --sh.signaled;  // this wake-up consumed one (or was spurious)
    }
  }
}

void WorkQueue::done(const std::string& key) {
  Shard& sh = shard_of(key);
  Shard::Wake wake;
  {
    std::lock_guard<std::mutex> lk(sh.mu);
    sh.done_locked(key, wake);
    sh.count_locked();
  }
  sh.fire(wake);
}

void WorkQueue::shutdown() {
  for (auto& sh : shards_) {
    {
      std::lock_guard<std::mutex> lk(sh->mu);
      sh->shutdown = true;
    }
    sh->cv.notify_all();
    sh->timer_cv.notify_all();
  }
}

size_t WorkQueue::pending() const {
  size_t n = 0;
  for (const auto& sh : shards_) n += sh->pending.load(std::memory_order_relaxed);
  return n;
}

size_t WorkQueue::in_flight() const {
  size_t n = 0;
  for (const auto& sh : shards_) {
    std::lock_guard<std::mutex> lk(sh->mu);
    n += sh->processing.size();
  }
  return n;
}

// ---------------------------------------------------------------------------
// Controller

Controller::Mapper owner_mapper(const ResourceType& owner) {
  std::string api_version = owner.api_version();
  std::string kind = owner.kind;
  return [api_version, kind](const Value& child) {
    std::vector<std::string> keys;
    for (const auto& ref : child.get("metadata").get("ownerReferences").items()) {
      if (ref.get_string("kind") == kind && ref.get_string("apiVersion") == api_version) {
        keys.push_back(ref.get_string("name"));
      }
    }
    return keys;
  };
}

Controller::Controller(KubeClient& client, ResourceType primary, Options opts)
    : client_(client),
      primary_(std::move(primary)),
      opts_(opts),
      primary_store_(std::make_unique<Store>(primary_)),
      queue_(WorkQueue::shards_for(opts.workers)) {}

Controller::~Controller() { queue_.shutdown(); }

void Controller::owns(const ResourceType& child, Mapper mapper, std::string label_selector, bool metadata_only) {
  auto c = std::make_unique<Child>();
  c->rt = child;
  c->selector = std::move(label_selector);
  c->metadata_only = metadata_only;
  c->mapper = mapper ? std::move(mapper) : owner_mapper(primary_);
  c->store = std::make_unique<Store>(child);
  children_.push_back(std::move(c));
}

Store* Controller::child_store(const std::string& plural) {
  for (auto& c : children_) {
    if (c->rt.plural == plural) return c->store.get();
  }
  return nullptr;
}

void Controller::enqueue_all() {
  for (const auto& o : primary_store_->list()) queue_.add(primary_.key(meta_namespace(*o), meta_name(*o)));
}

bool Controller::wait_synced(std::chrono::milliseconds timeout) {
  auto deadline = std::chrono::steady_clock::now() + timeout;
  if (!primary_store_->wait_synced(timeout)) return false;
  for (auto& c : children_) {
    auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
    if (left.count() < 0 || !c->store->wait_synced(left)) return false;
  }
  return true;
}

void Controller::run(CancelToken& stop, Reconciler reconcile, ErrorPolicy error_policy) {
  std::vector<std::thread> threads;
  auto store_gauge = [](const ResourceType& rt) -> metrics::Gauge& {
    return metrics::Registry::global().gauge("bgc_controller_store_objects", "Objects in the controller's watch cache",
                                             {{"resource", rt.plural}});
  };
  auto& primary_gauge = store_gauge(primary_);
  for (auto& cp : children_) cp->gauge = &store_gauge(cp->rt);
  // primary watcher: trigger_self
  threads.emplace_back([&] {
    Watcher w(client_, primary_);
    w.set_projection(opts_.primary_projection);
    // the two shared locks a watch event takes (stall::note_lock_section)
    const std::string store_section = "w:" + primary_.plural + " store", queue_section = "w:" + primary_.plural + " queue";
    w.run(stop, [&](const WatchEvent& ev) {
      // marked before the store applies it: a worker may reconcile from the store at once
      if (trace::armed() && ev.object && ev.type != WatchEvent::Type::Deleted) {
        const std::string name = meta_name(*ev.object);
        trace::mark_at(name, "ctl.primary_read", ev.read_ns);
        trace::mark(name, "ctl.primary_event");
      }
      const int64_t t0 = metrics::now_ns();
      primary_store_->apply(ev);
      const int64_t t1 = metrics::now_ns();
      stall::note_lock_section(store_section, t0, t1);
      primary_gauge.set(static_cast<double>(primary_store_->size()));
      if (ev.type == WatchEvent::Type::Restarted) {
        for (const auto& o : ev.objects) queue_.add(primary_.key(meta_namespace(*o), meta_name(*o)));
      } else if (ev.type != WatchEvent::Type::Deleted) {
        queue_.add_after(primary_.key(meta_namespace(*ev.object), meta_name(*ev.object)), opts_.debounce);
        stall::note_lock_section(queue_section, t1, metrics::now_ns());
      } else {
        // the object is gone: its periodic requeue would only find nothing
        queue_.forget(primary_.key(meta_namespace(*ev.object), meta_name(*ev.object)));
        if (primary_deleted_) primary_deleted_(*ev.object);
      }
    });
  });
  // owned watchers: trigger_owners
  auto ignored = [](const char* why) -> metrics::Counter& {
    return metrics::Registry::global().counter("bgc_controller_child_events_ignored_total",
                                               "Child watch events that queue no reconcile", {{"reason", why}});
  };
  auto& terminating = ignored("terminating");
  auto& ownerless = ignored("owner_not_cached");
  for (auto& cp : children_) {
    Child* c = cp.get();
    threads.emplace_back([&, c] {
      Watcher w(client_, c->rt, "", c->selector);
      w.set_metadata_only(c->metadata_only);
      w.set_projection(opts_.child_projection);
      const std::string store_section = "w:" + c->rt.plural + " store";
      w.run(stop, [&, c](const WatchEvent& ev) {
        if (trace::armed() && ev.object && ev.type != WatchEvent::Type::Deleted) {
          trace::mark(meta_name(*ev.object), "ctl." + c->rt.plural + "_event");
        }
        const int64_t t0 = metrics::now_ns();
        c->store->apply(ev);
        stall::note_lock_section(store_section, t0, metrics::now_ns());
        c->gauge->set(static_cast<double>(c->store->size()));
        if (ev.type == WatchEvent::Type::Restarted) {
          for (const auto& o : ev.objects) {
            for (const auto& k : c->mapper(*o)) queue_.add(k);
          }
        } else {
          if (ev.type == WatchEvent::Type::Deleted) {
            if (child_deleted_) child_deleted_(c->rt, *ev.object);
            // An owner that is already gone (the usual cascade after a UserBootstrap is
            // deleted) has nothing to repair: no trigger.
            for (const auto& k : c->mapper(*ev.object)) {
              if (primary_store_->get(k)) queue_.add_after(k, opts_.child_delete_delay);
            }
            return;
          }
          // A child on its way out (deletionTimestamp: a Namespace turning Terminating after
          // its owner was deleted) queues nothing until its DELETED event.
          if (ev.object->get("metadata").contains("deletionTimestamp")) {
            terminating.inc();
            return;
          }
          if (child_filter_ && !child_filter_(c->rt, *ev.object)) {
            filtered_.fetch_add(1, std::memory_order_relaxed);
            return;
          }
          // Nor does one whose owner is not in the cache: already deleted (the cascade), or
          // not seen yet, in which case the owner's own event queues it.
          for (const auto& k : c->mapper(*ev.object)) {
            if (primary_store_->get(k)) queue_.add_after(k, opts_.debounce);
            else ownerless.inc();
          }
        }
      });
    });
  }
  auto& reg = metrics::Registry::global();
  auto& q_depth = reg.gauge("bgc_controller_queue_depth", "Keys waiting in the work queue");
  std::vector<std::thread> workers;
  for (int i = 0; i < std::max(1, opts_.workers); ++i) {
    workers.emplace_back([&, i] {
      set_thread_name("reconcile");
      std::string key;
      while (queue_.get(key, static_cast<size_t>(i))) {
        q_depth.set(static_cast<double>(queue_.pending()));
        ObjPtr obj = primary_store_->get(key);
        if (!obj) {
          queue_.done(key);
          continue;
        }
        const bool traced = trace::armed();
        if (traced) trace::mark(meta_name(*obj), "ctl.reconcile0");
        Action a;
        try {
          a = reconcile(obj);
        } catch (const std::exception& e) {
          a = error_policy(obj, e);
        }
        if (traced) trace::mark(meta_name(*obj), "ctl.reconcile1");
        const int64_t f0 = metrics::now_ns();
        queue_.finish(key, a.requeue, a.after);
        stall::note_lock_section("reconcile queue", f0, metrics::now_ns());
        q_depth.set(static_cast<double>(queue_.pending()));
      }
    });
  }
  stop.wait();
  queue_.shutdown();
  for (auto& t : workers) t.join();  // in-flight reconciles complete (graceful shutdown)
  for (auto& t : threads) t.join();
}

}  // namespace bgc::kube

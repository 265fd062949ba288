#include "core/stall.h"

#include <pthread.h>
#include <signal.h>
#include <time.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "core/json.h"
#include "core/metrics.h"
#include "core/schedstat.h"
#include "core/process.h"

namespace bgc::stall {

namespace {

struct Stall {
  int64_t t_ns;        // when the late wake-up (or slow malloc) ended
  int64_t over_ns;     // oversleep beyond the 1 ms tick
  int64_t runq_ns;     // the sampler thread's run-queue delay over the tick
  int64_t malloc_ns;   // one malloc+free of 32 KiB
};

struct Slow {
  int64_t t1_ns;
  int64_t dur_ns;
  std::string what;
};

constexpr int64_t kTickNs = 1000000;
constexpr size_t kMaxKept = 1 << 16;
// past the thread cache (tcache_max 16 KiB in the services' tunables), so the malloc takes
// an arena lock like the services' large allocations do
constexpr size_t kMallocBytes = 32 << 10;

std::once_flag g_once;
std::atomic<bool> g_running{false};
std::atomic<uint64_t> g_ticks{0};
// note_slow's threshold: "never" until start() finds that records are kept
std::atomic<int64_t> g_slow_ns{INT64_MAX};
std::atomic<int64_t> g_lock_ns{INT64_MAX};

// Never destroyed: the sampler thread is detached and still runs while static destructors
// run at exit (a ThreadSanitizer race on a global vector, tools/sanitize.sh tsan).
struct State {
  std::mutex mu;
  std::string process;
  std::vector<Stall> kept;
  std::vector<Slow> slow;
  uint64_t dropped = 0;
};
State& state() {
  static State* s = new State();
  return *s;
}

std::vector<double> stall_buckets() {
  return {50e-6, 100e-6, 200e-6, 500e-6, 1e-3, 2e-3, 5e-3, 10e-3, 20e-3, 50e-3, 100e-3, 500e-3, 1.0};
}

int64_t record_threshold_ns() {
  const char* rec = std::getenv("BGC_STALL_RECORD_US");
  return (rec ? std::atoll(rec) : 2000) * 1000;
}

void loop() {
  set_thread_name("stall-sampler");
  sigset_t all;
  sigfillset(&all);
  pthread_sigmask(SIG_BLOCK, &all, nullptr);
  auto& reg = metrics::Registry::global();
  auto& over_h = reg.histogram("bgc_stall_oversleep_seconds",
                               "How late a 1 ms sleep of the stall sampler woke up (CPU unavailable to this process)",
                               {}, stall_buckets());
  auto& malloc_h = reg.histogram("bgc_stall_malloc_seconds", "One 32 KiB malloc+free of the stall sampler (an arena lock)", {},
                                 stall_buckets());
  const int64_t record_ns = record_threshold_ns();
  const bool keep = metrics::debug_endpoints_enabled();
  struct timespec req {0, kTickNs};
  int64_t runq0 = keep ? sched::thread_sched().runq_ns : -1;
  while (true) {
    const int64_t t0 = metrics::now_ns();
    nanosleep(&req, nullptr);
    const int64_t t1 = metrics::now_ns();
    void* volatile p = std::malloc(kMallocBytes);
    std::free(p);
    const int64_t t2 = metrics::now_ns();
    const int64_t over = std::max<int64_t>(0, t1 - t0 - kTickNs);
    const int64_t mal = t2 - t1;
    over_h.observe(static_cast<double>(over) * 1e-9);
    malloc_h.observe(static_cast<double>(mal) * 1e-9);
    g_ticks.fetch_add(1, std::memory_order_relaxed);
    if (!keep) continue;
    const int64_t runq1 = sched::thread_sched().runq_ns;
    const int64_t runq = runq0 >= 0 && runq1 >= 0 ? runq1 - runq0 : -1;
    runq0 = runq1;
    if (over >= record_ns || mal >= record_ns) {
      State& st = state();
      std::lock_guard<std::mutex> lk(st.mu);
      if (st.kept.size() < kMaxKept) st.kept.push_back({t2, over, runq, mal});
      else ++st.dropped;
    }
  }
}

}  // namespace

void start(const std::string& name) {
  const char* e = std::getenv("BGC_STALL_SAMPLER");
  if (e && std::strcmp(e, "0") == 0) return;
  std::call_once(g_once, [&] {
    {
      State& st = state();
      std::lock_guard<std::mutex> lk(st.mu);
      st.process = name;
    }
    g_running.store(true);
    if (metrics::debug_endpoints_enabled()) {
      g_slow_ns.store(record_threshold_ns());
      const char* lk = std::getenv("BGC_LOCK_SECTION_US");
      g_lock_ns.store((lk ? std::atoll(lk) : 200) * 1000);
    }
    std::thread(loop).detach();
  });
}

bool running() { return g_running.load(); }

namespace {
void keep_slow(std::string_view what, int64_t t0_ns, int64_t t1_ns) {
  State& st = state();
  std::lock_guard<std::mutex> lk(st.mu);
  if (st.slow.size() < kMaxKept) st.slow.push_back({t1_ns, t1_ns - t0_ns, std::string(what)});
  else ++st.dropped;
}
}  // namespace

void note_slow(std::string_view what, int64_t t0_ns, int64_t t1_ns) {
  if (t1_ns - t0_ns >= g_slow_ns.load(std::memory_order_relaxed)) keep_slow(what, t0_ns, t1_ns);
}

void note_lock_section(std::string_view what, int64_t t0_ns, int64_t t1_ns) {
  if (t1_ns - t0_ns >= g_lock_ns.load(std::memory_order_relaxed)) keep_slow(what, t0_ns, t1_ns);
}

std::string dump_json(bool take) {
  std::vector<Stall> kept;
  std::vector<Slow> slow;
  json::Value out = json::Value::object();
  {
    State& st = state();
    std::lock_guard<std::mutex> lk(st.mu);
    out["process"] = st.process;
    out["dropped"] = static_cast<unsigned long long>(st.dropped);
    if (take) {
      kept.swap(st.kept);
      slow.swap(st.slow);
      st.dropped = 0;
    } else {
      kept = st.kept;
      slow = st.slow;
    }
  }
  out["running"] = running();
  out["ticks"] = static_cast<unsigned long long>(g_ticks.load());
  json::Value arr = json::Value::array();
  for (const auto& s : kept) {
    json::Value e = json::Value::array();
    e.push_back(static_cast<long long>(s.t_ns));
    e.push_back(static_cast<double>(s.over_ns) * 1e-3);
    e.push_back(s.runq_ns < 0 ? json::Value() : json::Value(static_cast<double>(s.runq_ns) * 1e-3));
    e.push_back(static_cast<double>(s.malloc_ns) * 1e-3);
    arr.push_back(std::move(e));
  }
  out["stalls"] = std::move(arr);
  json::Value sl = json::Value::array();
  for (auto& s : slow) {
    json::Value e = json::Value::array();
    e.push_back(static_cast<long long>(s.t1_ns));
    e.push_back(static_cast<double>(s.dur_ns) * 1e-3);
    e.push_back(std::move(s.what));
    sl.push_back(std::move(e));
  }
  out["slow"] = std::move(sl);
  return out.dump();
}

}  // namespace bgc::stall

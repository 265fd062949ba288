#include "core/process.h"

#include <malloc.h>
#include <openssl/crypto.h>
#include <pthread.h>
#include <signal.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <thread>

#include "core/cpuprof.h"
#include "core/log.h"
#include "core/metrics.h"

namespace bgc {

static long env_long(const char* name, long dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atol(v) : dflt;
}

// The one source of truth for the services' allocator settings.  The container image and
// the test cluster set only the thread-cache tunables through GLIBC_TUNABLES (mallopt has
// no tcache knob); everything below is set here, and an image env var can no longer
// disagree with it (round 5: the image's trim_threshold was dead, this overrode it).
//
//  * M_ARENA_MAX (BGC_MALLOC_ARENA_MAX, default 4): glibc's default is 8 arenas per CPU —
//    2,048 on the MI355X hosts' 256 visible CPUs — and a thread-per-connection server gives
//    nearly every connection thread an arena of its own, each keeping its own free memory:
//    round 5 measured the admission server at 17 MB live in 195 MB RSS with 11 GB of free
//    arena space.  The thread cache (64 chunks per size class up to 16 KiB) serves the
//    hot-path allocations without touching an arena, so 4 arenas are rarely contended.
//  * M_TOP_PAD 4 MiB (BGC_MALLOC_TOP_PAD_KB) and M_TRIM_THRESHOLD 16 MiB
//    (BGC_MALLOC_TRIM_THRESHOLD_KB): a heap grows 4 MiB at a time and hands back a free top
//    above 16 MiB, so bursts do not cycle sbrk per request (the cost the old 64 MiB pad and
//    512 MiB threshold were there to avoid) and a quiet service returns to its live size.
//  * M_MMAP_THRESHOLD 4 MiB fixed: glibc's dynamic threshold would otherwise climb after
//    the first large free and keep multi-MiB list bodies in the arenas.
// BGC_MALLOC_TUNE=0 leaves glibc's defaults; 0 for one knob leaves that one at glibc's.
void tune_malloc() {
  const char* e = std::getenv("BGC_MALLOC_TUNE");
  if (e && std::strcmp(e, "0") == 0) return;
  if (const long a = env_long("BGC_MALLOC_ARENA_MAX", 4); a > 0) mallopt(M_ARENA_MAX, static_cast<int>(a));
  if (const long k = env_long("BGC_MALLOC_TOP_PAD_KB", 4 << 10); k > 0) mallopt(M_TOP_PAD, static_cast<int>(k << 10));
  if (const long k = env_long("BGC_MALLOC_TRIM_THRESHOLD_KB", 16 << 10); k > 0) {
    mallopt(M_TRIM_THRESHOLD, static_cast<int>(k << 10));
  }
  mallopt(M_MMAP_THRESHOLD, 4 << 20);
}

// The trim threshold above keeps freed heap resident between bursts (no madvise churn on
// the hot path).  A trimmer thread hands memory that stayed free back to the OS once the
// resident set has grown: every BGC_MALLOC_TRIM_SECS (default 30; 0 disables) it reads the
// RSS (/proc/self/statm, cheap) and runs malloc_trim only when the RSS exceeds both
// BGC_MALLOC_TRIM_MIN_MB (default 64) and 1.5x the RSS left by the previous trim.
// malloc_trim walks every free chunk under its arena's lock: measured on the MI355X box a
// pass stalled the synchronizer (85 MB RSS) for 13-15 ms and kube-lite (1.5 GB) for
// 110-130 ms, every 30 s, which showed up as apply->Ready tails.  Trimming on growth keeps
// the RSS of a long-running service near its live data after a burst without stalling a
// steady one.  A pass also waits for a quiet interval: the process used at most
// BGC_MALLOC_TRIM_IDLE_PCT (default 5) % of one CPU since the last check, so the stall
// lands between bursts of work, not inside one (the synchronizer's one pass per bench run
// fell into a latency window: a 13-15 ms stall of the path to Ready).  A process that is
// never quiet still trims once its RSS has passed 4x the previous trim's (and 4x the minimum),
// or half its container's memory limit: freed memory that many threads' arenas keep while
// busy (the admission server: 17 MB live at 195 MB RSS after a bench run) must not reach an
// OOM kill.
TrimDecision malloc_trim_decision(long rss, long baseline, long min_bytes, double busy_pct, double idle_pct,
                                  long limit_bytes) {
  if (rss <= min_bytes || rss * 2 <= baseline * 3) return TrimDecision::Skip;
  if (limit_bytes > 0 && rss > limit_bytes / 2) return TrimDecision::Trim;
  if (busy_pct > idle_pct && rss < std::max(baseline, min_bytes) * 4) return TrimDecision::Defer;
  return TrimDecision::Trim;
}

long cgroup_memory_limit_bytes() {
  // BGC_MALLOC_TRIM_LIMIT_MB overrides what the cgroup says (a runtime that enforces memory
  // some other way, or a test of the valve on a machine without a limit)
  if (const char* o = std::getenv("BGC_MALLOC_TRIM_LIMIT_MB")) return std::atol(o) << 20;
  for (const char* path : {"/sys/fs/cgroup/memory.max", "/sys/fs/cgroup/memory/memory.limit_in_bytes"}) {
    FILE* f = std::fopen(path, "r");
    if (!f) continue;
    char buf[64] = {0};
    const bool got = std::fgets(buf, sizeof buf, f) != nullptr;
    std::fclose(f);
    if (!got) continue;
    const long long v = std::atoll(buf);  // "max" (v2, no limit) reads as 0
    // v1 reports "no limit" as a page-rounded LLONG_MAX
    return v > 0 && v < (1LL << 60) ? static_cast<long>(v) : 0;
  }
  return 0;
}

static double cpu_seconds() {
  struct rusage ru {};
  if (getrusage(RUSAGE_SELF, &ru) != 0) return 0;
  return static_cast<double>(ru.ru_utime.tv_sec + ru.ru_stime.tv_sec) +
         static_cast<double>(ru.ru_utime.tv_usec + ru.ru_stime.tv_usec) * 1e-6;
}

static long rss_bytes() {
  long pages_total = 0, pages_rss = 0;
  if (FILE* f = std::fopen("/proc/self/statm", "r")) {
    if (std::fscanf(f, "%ld %ld", &pages_total, &pages_rss) != 2) pages_rss = 0;
    std::fclose(f);
  }
  return pages_rss * sysconf(_SC_PAGESIZE);
}

void start_malloc_trimmer() {
  const char* e = std::getenv("BGC_MALLOC_TRIM_SECS");
  const long secs = e ? std::atol(e) : 30;
  if (secs <= 0) return;
  const char* m = std::getenv("BGC_MALLOC_TRIM_MIN_MB");
  const long min_bytes = (m ? std::atol(m) : 64) << 20;
  const char* ip = std::getenv("BGC_MALLOC_TRIM_IDLE_PCT");
  const double idle_pct = ip ? std::atof(ip) : 5.0;
  std::thread([secs, min_bytes, idle_pct] {
    // Never take process signals here: SIGTERM/SIGINT are collected by the sigwait thread
    // that install_shutdown_signals starts (this thread exists before that mask is set).
    sigset_t all;
    sigfillset(&all);
    pthread_sigmask(SIG_BLOCK, &all, nullptr);
    auto& reg = metrics::Registry::global();
    auto& hist = reg.histogram("bgc_malloc_trim_seconds", "Wall time of one malloc_trim pass");
    auto& last = reg.gauge("bgc_malloc_trim_last_seconds", "Wall time of the last malloc_trim pass");
    auto& skipped = reg.counter("bgc_malloc_trim_skipped_total", "Trim checks that found the RSS below the trigger");
    auto& deferred = reg.counter("bgc_malloc_trim_deferred_total",
                                 "Trim checks that found the RSS grown but the process busy");
    auto& limit_g = reg.gauge("bgc_malloc_trim_memory_limit_bytes",
                              "Container memory limit the trimmer keeps the RSS under half of (0 = none)");
    const long limit = cgroup_memory_limit_bytes();
    limit_g.set(static_cast<double>(limit));
    long baseline = rss_bytes();
    double cpu0 = cpu_seconds();
    while (true) {
      std::this_thread::sleep_for(std::chrono::seconds(secs));
      const long rss = rss_bytes();
      const double cpu = cpu_seconds();
      const double busy_pct = (cpu - cpu0) * 100.0 / static_cast<double>(secs);
      cpu0 = cpu;
      const TrimDecision d = malloc_trim_decision(rss, baseline, min_bytes, busy_pct, idle_pct, limit);
      if (d != TrimDecision::Trim) {
        (d == TrimDecision::Skip ? skipped : deferred).inc();
        continue;
      }
      const int64_t t0 = metrics::now_ns();
      malloc_trim(0);
      const double dt = static_cast<double>(metrics::now_ns() - t0) * 1e-9;
      hist.observe(dt);
      last.set(dt);
      baseline = rss_bytes();
    }
  }).detach();
}

// OpenSSL's default atexit handler (OPENSSL_cleanup) frees its global state and deletes
// the thread-local key whose destructor frees each thread's state (DRBGs, error queue).
// A detached thread that is still finishing while the process exits (an HTTP connection
// thread after Server::stop's grace, an idle HTTP/2 worker) then ends after that cleanup,
// and its state can never be freed: LeakSanitizer's intermittent kube-lite report of round
// 4 (tools/probes/lsan_openssl_exit_race.cc reproduces it).  Without the handler, exit
// leaves OpenSSL's memory to the kernel, like any other process memory.
void init_openssl() { OPENSSL_init_crypto(OPENSSL_INIT_NO_ATEXIT, nullptr); }

// BGC_DIE_WITH_PARENT=<pid> (test harnesses): SIGTERM this process when the process that
// started it dies (PR_SET_PDEATHSIG), so a test run killed by a timeout leaves no service
// behind.  The variable is removed first, so this process's own children (diagnostics
// workers) do not inherit it.  A parent that is not the given PID — already gone, or a
// wrapper (a profiler, a sanitizer script, a shell) between harness and service — ends this
// process at once with status 3 and a line saying why: a misconfigured launch must fail
// loudly, not look like a clean stop.
static void die_with_parent_from_env() {
  const char* v = std::getenv("BGC_DIE_WITH_PARENT");
  if (!v) return;
  const long parent = std::atol(v);
  ::unsetenv("BGC_DIE_WITH_PARENT");
  ::prctl(PR_SET_PDEATHSIG, SIGTERM);
  const pid_t ppid = ::getppid();
  if (parent > 0 && ppid != static_cast<pid_t>(parent)) {
    std::fprintf(stderr, "BGC_DIE_WITH_PARENT=%ld but the parent process is %d (the parent exited, or a wrapper "
                 "started this process); exiting\n", parent, static_cast<int>(ppid));
    std::_Exit(3);
  }
}

void set_thread_name(const std::string& name) {
  ::pthread_setname_np(::pthread_self(), name.substr(0, 15).c_str());
}

void process_init() {
  die_with_parent_from_env();
  init_openssl();
  tune_malloc();
  start_malloc_trimmer();
  log::init_from_env();
  cpuprof::start_from_env();
}

void arm_shutdown_deadline(std::chrono::milliseconds limit, int code) {
  if (limit.count() <= 0) return;
  std::thread([limit, code] {
    std::this_thread::sleep_for(limit);
    // the line is written from a thread of its own: a blocked stderr must not keep the
    // process alive past the deadline
    std::thread([limit] {
      LOG_ERROR("process") << "shutdown did not finish within " << limit.count()
                           << " ms (a thread is stuck, e.g. in a driver call); exiting";
      log::flush();
    }).detach();
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    std::_Exit(code);
  }).detach();
}

}  // namespace bgc

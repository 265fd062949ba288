#include "core/process.h"

#include <malloc.h>
#include <openssl/crypto.h>
#include <pthread.h>
#include <signal.h>
#include <sys/prctl.h>
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
//  * M_ARENA_MAX (BGC_MALLOC_ARENA_MAX; default 4, the controller 16): glibc's default is 8
//    arenas per CPU — 2,048 on the MI355X hosts' 256 visible CPUs — and a thread-per-
//    connection server gives nearly every connection thread an arena of its own, each
//    keeping its own free memory: round 5 measured the admission server at 17 MB live in
//    195 MB RSS with 11 GB of free arena space.  The thread cache (64 chunks per size class
//    up to 16 KiB) serves most hot-path allocations without an arena.  The controller's 16
//    workers and their apply threads allocate hard enough that 4 arenas cost it 10 % CPU per
//    tenant (0.210 against 0.189 ms unbounded, 16: 0.193; profiles/r6_alloc/), so it gets 16.
//  * M_TOP_PAD 1 MiB (BGC_MALLOC_TOP_PAD_KB) and M_TRIM_THRESHOLD 2 MiB
//    (BGC_MALLOC_TRIM_THRESHOLD_KB): a heap grows 1 MiB at a time and hands back a free top
//    above 2 MiB, so a quiet service returns to its live size.  The old 64 MiB pad and
//    512 MiB threshold were there to avoid sbrk churn under bursts; measured on the box the
//    churn costs nothing visible (controller CPU per tenant 0.195 against 0.193 ms with 4 MiB
//    / 16 MiB, admission and controller 0.368 against 0.368 ms at 64 MiB / 512 MiB), while
//    the controller's RSS falls from 50 to 38 MB (profiles/r6_alloc/r6_alloc7, r6_alloc5).
//  * M_MMAP_THRESHOLD 4 MiB fixed: glibc's dynamic threshold would otherwise climb after
//    the first large free and keep multi-MiB list bodies in the arenas.
// BGC_MALLOC_TUNE=0 leaves glibc's defaults; 0 for one knob leaves that one at glibc's.
void tune_malloc(const ProcessDefaults& defaults) {
  const char* e = std::getenv("BGC_MALLOC_TUNE");
  if (e && std::strcmp(e, "0") == 0) return;
  if (const long a = env_long("BGC_MALLOC_ARENA_MAX", defaults.malloc_arena_max); a > 0) {
    mallopt(M_ARENA_MAX, static_cast<int>(a));
  }
  if (const long k = env_long("BGC_MALLOC_TOP_PAD_KB", 1 << 10); k > 0) mallopt(M_TOP_PAD, static_cast<int>(k << 10));
  if (const long k = env_long("BGC_MALLOC_TRIM_THRESHOLD_KB", 2 << 10); k > 0) {
    mallopt(M_TRIM_THRESHOLD, static_cast<int>(k << 10));
  }
  mallopt(M_MMAP_THRESHOLD, 4 << 20);
}

// With the arenas bounded and tops trimmed by glibc itself (tune_malloc above) the services'
// RSS stays within a few MB of their live heap (round 6: admission 40 MB, controller 38 MB,
// profiles/r6_alloc/), so nothing trims on a timer any more.  Round 5's trimmer thread,
// with its growth, quiet-interval and 4x heuristics, compensated for the 64 MiB heap growth
// and 512 MiB trim threshold it replaced; it stalled the process for 13-15 ms per pass
// (malloc_trim walks every free chunk under its arena's lock).  One valve stays: a process
// whose RSS has passed half its container's memory limit (and grown 1.5x since the last
// pass) trims, rather than reach an OOM kill with freed memory still resident.
TrimDecision malloc_trim_decision(long rss, long baseline, long limit_bytes) {
  if (limit_bytes <= 0 || rss <= limit_bytes / 2 || rss * 2 <= baseline * 3) return TrimDecision::Skip;
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
  const long limit = cgroup_memory_limit_bytes();
  if (secs <= 0 || limit <= 0) return;  // no limit to keep under: glibc's own trimming is enough
  std::thread([secs, limit] {
    set_thread_name("malloc-trim");
    // Never take process signals here: SIGTERM/SIGINT are collected by the sigwait thread
    // that install_shutdown_signals starts (this thread exists before that mask is set).
    sigset_t all;
    sigfillset(&all);
    pthread_sigmask(SIG_BLOCK, &all, nullptr);
    auto& reg = metrics::Registry::global();
    auto& hist = reg.histogram("bgc_malloc_trim_seconds", "Wall time of one malloc_trim pass");
    auto& last = reg.gauge("bgc_malloc_trim_last_seconds", "Wall time of the last malloc_trim pass");
    auto& limit_g = reg.gauge("bgc_malloc_trim_memory_limit_bytes",
                              "Container memory limit the trimmer keeps the RSS under half of");
    limit_g.set(static_cast<double>(limit));
    long baseline = 0;
    while (true) {
      std::this_thread::sleep_for(std::chrono::seconds(secs));
      if (malloc_trim_decision(rss_bytes(), baseline, limit) != TrimDecision::Trim) continue;
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

void process_init(const ProcessDefaults& defaults) {
  die_with_parent_from_env();
  init_openssl();
  tune_malloc(defaults);
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

#include "core/cpuprof.h"

#include <dirent.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>
#include <unwind.h>

#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <set>
#include <sstream>
#include <thread>
#include <vector>

namespace bgc::cpuprof {

namespace {

constexpr int kMaxFrames = 40;
constexpr size_t kMaxSamples = size_t(1) << 17;  // ~43 MB at 40 frames; ~2 min of one busy core at 997 Hz

struct Sample {
  uint32_t n;
  uintptr_t pc[kMaxFrames];
};

Sample* g_buf = nullptr;
std::atomic<size_t> g_next{0};
std::atomic<bool> g_on{false};
std::atomic<uint64_t> g_dropped{0};
std::atomic<uint64_t> g_overruns{0};  // timer expirations folded into one signal (si_overrun)
int g_probe[2] = {-1, -1};
// BGC_CPU_PROFILE_UNWIND=eh: walk with the .eh_frame unwinder (libgcc) instead of frame
// pointers.  OpenSSL and glibc are built without frame pointers (they use %rbp as a
// general register), so a frame-pointer walk that starts inside them ends at once and the
// sample cannot be charged to the bgc code that called them; the unwinder follows the CFI
// those libraries ship.  _Unwind_Backtrace is not formally async-signal-safe; glibc's
// dl_iterate_phdr lock it takes is recursive, and the profiler is a diagnostics mode only.
bool g_eh = false;

struct EhWalk {
  Sample* s;
  int skip;  // frames of the signal handler itself
};

_Unwind_Reason_Code eh_frame(struct _Unwind_Context* ctx, void* arg) {
  auto* w = static_cast<EhWalk*>(arg);
  const uintptr_t ip = _Unwind_GetIP(ctx);
  if (ip == 0) return _URC_END_OF_STACK;
  if (w->skip > 0) {
    --w->skip;
    return _URC_NO_REASON;
  }
  if (w->s->n >= kMaxFrames) return _URC_END_OF_STACK;
  w->s->pc[w->s->n] = ip - 1;  // return addresses: attribute to the call instruction
  w->s->n++;
  return _URC_NO_REASON;
}
std::string g_path;
std::mutex g_mu;
bool g_started = false;

// Per-thread CPU timers.  A process-wide ITIMER_PROF fires at most once per scheduler
// tick for the whole process (250-1000 Hz however many threads are busy), so a 16-thread
// service is sampled at a fraction of `hz`.  Instead every thread gets its own
// CLOCK_THREAD_CPUTIME timer delivering SIGPROF to that thread (SIGEV_THREAD_ID); a
// helper thread arms one for each new thread it finds in /proc/self/task every 50 ms.
bool g_per_thread = false;
long g_interval_ns = 0;
std::thread g_arm;
std::atomic<bool> g_arm_stop{false};
std::map<pid_t, timer_t> g_timers;  // under g_timers_mu
std::mutex g_timers_mu;

clockid_t thread_cpu_clock(pid_t tid) {
  // MAKE_THREAD_CPUCLOCK(tid, CPUCLOCK_SCHED): ((~tid) << 3) | CPUCLOCK_PERTHREAD_MASK | CPUCLOCK_SCHED
  return static_cast<clockid_t>((~static_cast<unsigned>(tid) << 3) | 4 | 2);
}

void arm_new_threads() {
  std::set<pid_t> live;
  if (DIR* d = ::opendir("/proc/self/task")) {
    while (dirent* e = ::readdir(d)) {
      if (e->d_name[0] >= '0' && e->d_name[0] <= '9') live.insert(static_cast<pid_t>(std::atoi(e->d_name)));
    }
    ::closedir(d);
  }
  const pid_t self = static_cast<pid_t>(::syscall(SYS_gettid));
  std::lock_guard<std::mutex> lk(g_timers_mu);
  for (auto it = g_timers.begin(); it != g_timers.end();) {
    if (!live.count(it->first)) {
      ::timer_delete(it->second);
      it = g_timers.erase(it);
    } else {
      ++it;
    }
  }
  for (pid_t tid : live) {
    if (tid == self || g_timers.count(tid)) continue;
    struct sigevent sev {};
    sev.sigev_notify = SIGEV_THREAD_ID;
    sev.sigev_signo = SIGPROF;
    sev._sigev_un._tid = tid;
    timer_t t;
    if (::timer_create(thread_cpu_clock(tid), &sev, &t) != 0) continue;  // the thread just exited
    struct itimerspec its {};
    its.it_interval.tv_sec = g_interval_ns / 1000000000L;
    its.it_interval.tv_nsec = g_interval_ns % 1000000000L;
    its.it_value = its.it_interval;
    ::timer_settime(t, 0, &its, nullptr);
    g_timers[tid] = t;
  }
}

// True when [p, p+16) is readable: write() reports EFAULT instead of faulting.
bool readable(uintptr_t p) {
  if (p < 4096) return false;
  ssize_t w = ::write(g_probe[1], reinterpret_cast<const void*>(p), 16);
  if (w != 16) return false;
  char sink[16];
  (void)!::read(g_probe[0], sink, sizeof(sink));
  return true;
}

void on_sigprof(int, siginfo_t* si, void* ucv) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  int saved_errno = errno;
  // A per-thread CPU timer is checked on scheduler ticks: expirations between two checks
  // arrive as one signal with si_overrun counting the rest (coverage = samples /
  // (samples + overruns) of the CPU time at the requested rate).
  if (si && si->si_code == SI_TIMER && si->si_overrun > 0) {
    g_overruns.fetch_add(static_cast<uint64_t>(si->si_overrun), std::memory_order_relaxed);
  }
  size_t i = g_next.fetch_add(1, std::memory_order_relaxed);
  if (i >= kMaxSamples) {
    g_dropped.fetch_add(1, std::memory_order_relaxed);
    errno = saved_errno;
    return;
  }
  auto* uc = static_cast<ucontext_t*>(ucv);
  Sample& s = g_buf[i];
  if (g_eh) {
    // frames: eh_frame's caller chain starts in this handler, then the kernel's signal
    // trampoline (__restore_rt), then the interrupted function
    s.n = 0;
    EhWalk w{&s, 0};
    _Unwind_Backtrace(eh_frame, &w);
    // drop the handler's own frames and the signal trampoline: the unwinder reports the
    // interrupted pc itself (not a return address) right after the trampoline
    const uintptr_t rip = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RIP]);
    uint32_t start = 0;
    for (uint32_t k = 0; k < s.n; ++k) {
      if (s.pc[k] + 1 == rip || s.pc[k] == rip) {
        start = k;
        break;
      }
    }
    if (start > 0) {
      for (uint32_t k = start; k < s.n; ++k) s.pc[k - start] = s.pc[k];
      s.n -= start;
    }
    if (s.n > 0) s.pc[0] = rip;
    errno = saved_errno;
    return;
  }
  uint32_t n = 0;
  s.pc[n++] = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RIP]);
  uintptr_t sp = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RSP]);
  uintptr_t fp = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RBP]);
  // [fp] = caller's fp, [fp + 8] = return address; frames grow toward higher addresses
  while (n < kMaxFrames && fp >= sp && fp - sp < (uintptr_t(64) << 20) && (fp & 7) == 0 && readable(fp)) {
    const uintptr_t* f = reinterpret_cast<const uintptr_t*>(fp);
    uintptr_t next = f[0];
    uintptr_t ret = f[1];
    if (ret < 4096) break;
    s.pc[n++] = ret - 1;  // attribute to the call instruction
    if (next <= fp) break;
    fp = next;
  }
  s.n = n;
  errno = saved_errno;
}

void write_profile() {
  if (g_path.empty() || !g_buf) return;
  size_t n = std::min(g_next.load(), kMaxSamples);
  std::map<std::vector<uintptr_t>, uint64_t> stacks;
  for (size_t i = 0; i < n; ++i) {
    const Sample& s = g_buf[i];
    if (s.n == 0 || s.n > kMaxFrames) continue;  // slot claimed but not filled
    stacks[std::vector<uintptr_t>(s.pc, s.pc + s.n)]++;
  }
  std::ofstream out(g_path);
  if (!out) return;
  std::ifstream maps("/proc/self/maps");
  out << "# bgc cpuprof v1 samples=" << n << " dropped=" << g_dropped.load() << " overruns=" << g_overruns.load()
      << "\n";
  out << "maps\n" << maps.rdbuf() << "end maps\n";
  char buf[32];
  for (const auto& [st, cnt] : stacks) {
    out << cnt;
    for (uintptr_t pc : st) {
      std::snprintf(buf, sizeof(buf), " %lx", static_cast<unsigned long>(pc));
      out << buf;
    }
    out << "\n";
  }
}

}  // namespace

bool start(const std::string& path, int hz) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_started) return true;
  if (::pipe2(g_probe, O_CLOEXEC | O_NONBLOCK) != 0) return false;
  if (const char* u = std::getenv("BGC_CPU_PROFILE_UNWIND"); u && std::string(u) == "eh") {
    g_eh = true;
    Sample warm{};
    EhWalk w{&warm, 0};
    _Unwind_Backtrace(eh_frame, &w);  // first use outside a signal handler: lazy setup
  }
  g_buf = static_cast<Sample*>(std::calloc(kMaxSamples, sizeof(Sample)));
  if (!g_buf) return false;
  g_path = path;
  struct sigaction sa {};
  sa.sa_sigaction = on_sigprof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, nullptr) != 0) return false;
  g_on = true;
  const char* mode = std::getenv("BGC_CPU_PROFILE_TIMER");  // "thread" (default) | "process"
  g_per_thread = !(mode && std::string(mode) == "process");
  if (g_per_thread) {
    g_interval_ns = 1000000000L / std::max(1, hz);
    g_arm_stop = false;
    arm_new_threads();
    // The helper never takes process signals (SIGTERM belongs to the service's sigwait
    // thread): it is created with every signal blocked and inherits that mask.
    sigset_t all, old;
    sigfillset(&all);
    pthread_sigmask(SIG_BLOCK, &all, &old);
    g_arm = std::thread([] {
      while (!g_arm_stop.load()) {
        arm_new_threads();
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
      }
    });
    pthread_sigmask(SIG_SETMASK, &old, nullptr);
  } else {
    struct itimerval it {};
    long us = 1000000L / std::max(1, hz);
    it.it_interval.tv_sec = us / 1000000L;
    it.it_interval.tv_usec = us % 1000000L;
    it.it_value = it.it_interval;
    if (setitimer(ITIMER_PROF, &it, nullptr) != 0) return false;
  }
  g_started = true;
  std::atexit([] { stop(); });
  return true;
}

void start_from_env() {
  const char* p = std::getenv("BGC_CPU_PROFILE");
  if (!p || !*p) return;
  int hz = 997;
  if (const char* h = std::getenv("BGC_CPU_PROFILE_HZ")) hz = std::max(1, std::atoi(h));
  std::string path = p;
  // one file per process: a "%p" in the path becomes the pid
  size_t at = path.find("%p");
  if (at != std::string::npos) path.replace(at, 2, std::to_string(::getpid()));
  if (!start(path, hz)) std::fprintf(stderr, "cpuprof: failed to start (%s)\n", std::strerror(errno));
}

void stop() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_started) return;
  if (g_per_thread) {
    g_arm_stop = true;
    if (g_arm.joinable()) g_arm.join();
    std::lock_guard<std::mutex> tl(g_timers_mu);
    for (auto& kv : g_timers) ::timer_delete(kv.second);
    g_timers.clear();
  } else {
    struct itimerval it {};
    setitimer(ITIMER_PROF, &it, nullptr);
  }
  g_on = false;
  write_profile();
  g_started = false;
}

}  // namespace bgc::cpuprof

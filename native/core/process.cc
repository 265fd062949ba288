#include "core/process.h"

#include <malloc.h>
#include <openssl/crypto.h>
#include <pthread.h>
#include <signal.h>

#include <cstdlib>
#include <cstring>
#include <chrono>
#include <thread>

#include "core/cpuprof.h"
#include "core/log.h"
#include "core/metrics.h"

namespace bgc {

void tune_malloc() {
  const char* e = std::getenv("BGC_MALLOC_TUNE");
  if (e && std::strcmp(e, "0") == 0) return;
  mallopt(M_TRIM_THRESHOLD, 512 << 20);
  mallopt(M_TOP_PAD, 64 << 20);
  mallopt(M_MMAP_THRESHOLD, 4 << 20);
}

// The trim threshold above keeps freed heap resident between bursts (no madvise churn on
// the hot path); a low-frequency malloc_trim hands memory that stayed free back to the OS,
// so a long-running service's RSS follows its live data instead of its historical peak.
// BGC_MALLOC_TRIM_SECS (default 30; 0 disables).
void start_malloc_trimmer() {
  const char* e = std::getenv("BGC_MALLOC_TRIM_SECS");
  const long secs = e ? std::atol(e) : 30;
  if (secs <= 0) return;
  std::thread([secs] {
    // Never take process signals here: SIGTERM/SIGINT are collected by the sigwait thread
    // that install_shutdown_signals starts (this thread exists before that mask is set).
    sigset_t all;
    sigfillset(&all);
    pthread_sigmask(SIG_BLOCK, &all, nullptr);
    // Every trim is timed: it walks the arenas under their locks, so a long one stalls
    // every allocating thread of the process for that long.
    auto& hist = metrics::Registry::global().histogram("bgc_malloc_trim_seconds", "Wall time of one malloc_trim pass");
    auto& last = metrics::Registry::global().gauge("bgc_malloc_trim_last_seconds", "Wall time of the last malloc_trim pass");
    while (true) {
      std::this_thread::sleep_for(std::chrono::seconds(secs));
      const int64_t t0 = metrics::now_ns();
      malloc_trim(0);
      const double dt = static_cast<double>(metrics::now_ns() - t0) * 1e-9;
      hist.observe(dt);
      last.set(dt);
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

void process_init() {
  init_openssl();
  tune_malloc();
  start_malloc_trimmer();
  log::init_from_env();
  cpuprof::start_from_env();
}

}  // namespace bgc

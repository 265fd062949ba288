// Common process start-up for the native services: RUST_LOG-style logging, glibc malloc
// tuning, OpenSSL's exit behaviour and the optional sampling profiler (core/cpuprof.h).
#pragma once

#include <chrono>
#include <string>

namespace bgc {

// Per-binary defaults of the allocator settings (tune_malloc; env overrides them).
struct ProcessDefaults {
  int malloc_arena_max = 4;
};

// Call first thing in main().
void process_init(const ProcessDefaults& defaults = ProcessDefaults());

// Names the calling thread (first 15 bytes; `top -H`, /proc/<pid>/task/<tid>/comm): the
// bench attributes CPU per thread by these names.
void set_thread_name(const std::string& name);

// OpenSSL without its atexit cleanup (see process.cc); part of process_init().
void init_openssl();

// glibc malloc tuning for many short-lived JSON allocations across thread-per-connection
// servers (process.cc): at most 4 arenas (16 in the controller), heaps grown 1 MiB at a time
// and trimmed above 2 MiB free, a fixed 4 MiB mmap threshold.  BGC_MALLOC_TUNE=0 disables it.
void tune_malloc(const ProcessDefaults& defaults = ProcessDefaults());
// The memory-limit valve's rule (process.cc): Trim once the RSS has passed half the
// container's memory limit (limit_bytes, 0 = none: never) and grown 1.5x since the RSS the
// previous pass left (baseline); else Skip.
enum class TrimDecision { Skip, Trim };
TrimDecision malloc_trim_decision(long rss, long baseline, long limit_bytes);
// The cgroup memory limit of this process (v2 memory.max, else v1 limit_in_bytes); 0 = none.
long cgroup_memory_limit_bytes();
// Bounds a graceful shutdown once it has started: after `limit` the process logs, flushes
// the log and exits with `code`.  A thread stuck in a driver call (amdsmi while the driver
// resets a GPU) would otherwise hold the process until the kubelet's SIGKILL, after its
// grace period, with nothing in the log.  limit <= 0: no deadline.
void arm_shutdown_deadline(std::chrono::milliseconds limit, int code = 1);

}  // namespace bgc

// Process stall sampler ("oversleep" detector).
//
// One thread per process sleeps 1 ms at a time and measures how late it wakes up, then
// times one small malloc/free.  A late wake-up means the process's threads could not get a
// CPU (run-queue wait on a saturated CPU share, CFS throttling); a slow malloc means an
// arena was held (malloc_trim, a heap walk).  Either shows as a process-wide pause with
// its owner — the process that reported it — which is what the bench needs to attribute
// an apply->Ready tail to kube-lite, the load driver or one of the product binaries.
//
// Exported on /metrics as bgc_stall_oversleep_seconds and bgc_stall_malloc_seconds
// histograms; with debug endpoints, every stall >= BGC_STALL_RECORD_US (default 2000 us)
// is kept with its monotonic timestamp and the sampler thread's run-queue delay over it
// (/proc/thread-self/schedstat) and served on /debug/stalls (GET, DELETE = take), so the
// harness can line stalls up with its latency windows.  BGC_STALL_SAMPLER=0 disables it.
#pragma once

#include <cstdint>
#include <string>
#include <string_view>

namespace bgc::stall {

// Starts the sampler thread once per process (idempotent); `name` labels the process in
// the dump.
void start(const std::string& name);
bool running();
// One thread's section of work [t0_ns, t1_ns] (monotonic) that may have held up what queued
// behind it: a watch event's handling, a watch write, a watch reconnect.  Kept beside the
// stalls when it lasted >= BGC_STALL_RECORD_US and the sampler keeps records (debug
// endpoints on); otherwise one relaxed load and a return.
void note_slow(std::string_view what, int64_t t0_ns, int64_t t1_ns);
// The same for a short section that takes a shared lock (a watcher's store apply or queue
// add): kept past BGC_LOCK_SECTION_US (default 200 us) instead, when records are kept.
void note_lock_section(std::string_view what, int64_t t0_ns, int64_t t1_ns);
// {"process":..,"ticks":n,"stalls":[[t_ns, oversleep_us, runq_us, malloc_us],...],
//  "slow":[[t1_ns, duration_us, what],...], "dropped":n}; `take` clears what was kept.
std::string dump_json(bool take);

}  // namespace bgc::stall

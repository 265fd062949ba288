// Scheduler accounting of the calling thread (/proc/thread-self/schedstat): time on a CPU
// and time spent runnable but waiting for one (run-queue delay).  The difference of two
// readings splits a wall-clock interval into running, waiting for a CPU, and blocked (the
// rest: sleeping in a syscall, e.g. an amdsmi ioctl waiting for the SMU).  The file stays
// open per thread: a reading is one pread, ~1-2 us.
#pragma once

#include <cstdint>

namespace bgc::sched {

struct ThreadSched {
  int64_t cpu_ns = -1;   // on-CPU time so far, CLOCK_THREAD_CPUTIME_ID (-1: unavailable)
  int64_t runq_ns = -1;  // run-queue delay so far, schedstat (updated as each wait ends)
  bool ok() const { return cpu_ns >= 0 && runq_ns >= 0; }
};

ThreadSched thread_sched();

}  // namespace bgc::sched

// Sampling CPU profiler for the native services (no perf/valgrind on the target images).
//
// SIGPROF (setitimer ITIMER_PROF) is delivered to whichever thread is consuming CPU; the
// handler records the interrupted PC plus the frame-pointer chain (the release build keeps
// frame pointers, -fno-omit-frame-pointer) into a fixed ring without locks or allocation.
// Every frame address is validated with a write() into a pipe (EFAULT instead of a fault),
// so a non-frame-pointer value in RBP (libc, libssl) cannot crash the process.
//
// Enable with BGC_CPU_PROFILE=<path> (optional BGC_CPU_PROFILE_HZ, default 997). The
// profile is written at exit: "maps" (a copy of /proc/self/maps) then one line per unique
// stack, "count pc0 pc1 ...", leaf first. tools/cpuprof_report.py symbolizes it (addr2line)
// into self/inclusive tables and collapsed stacks for flame graphs.
#pragma once

#include <string>

namespace bgc::cpuprof {

// Starts sampling when BGC_CPU_PROFILE is set; registers an atexit writer. Idempotent.
void start_from_env();
bool start(const std::string& path, int hz);
// Stops sampling and writes the profile (also runs at exit).
void stop();

}  // namespace bgc::cpuprof

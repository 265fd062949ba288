#include "core/schedstat.h"

#include <fcntl.h>
#include <unistd.h>

#include <cstdio>
#include <ctime>

namespace bgc::sched {

namespace {
struct Fd {
  int fd = ::open("/proc/thread-self/schedstat", O_RDONLY | O_CLOEXEC);
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};
}  // namespace

ThreadSched thread_sched() {
  thread_local Fd f;
  ThreadSched s;
  // on-CPU time from the thread CPU clock: schedstat's run time of a running thread is only
  // brought up to date at scheduler events, so it reads stale from the thread itself
  struct timespec ts {};
  if (::clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts) == 0) s.cpu_ns = int64_t{ts.tv_sec} * 1000000000 + ts.tv_nsec;
  if (f.fd < 0) return s;
  char buf[128];
  const ssize_t n = ::pread(f.fd, buf, sizeof buf - 1, 0);
  if (n <= 0) return s;
  buf[n] = '\0';
  unsigned long long run = 0, wait = 0;
  if (std::sscanf(buf, "%llu %llu", &run, &wait) != 2) return s;
  (void)run;
  s.runq_ns = static_cast<int64_t>(wait);
  return s;
}

}  // namespace bgc::sched

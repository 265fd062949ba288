#include "core/schedstat.h"

#include <fcntl.h>
#include <unistd.h>

#include <cstdio>

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
  if (f.fd < 0) return s;
  char buf[128];
  const ssize_t n = ::pread(f.fd, buf, sizeof buf - 1, 0);
  if (n <= 0) return s;
  buf[n] = '\0';
  unsigned long long run = 0, wait = 0;
  if (std::sscanf(buf, "%llu %llu", &run, &wait) != 2) return s;
  s.cpu_ns = static_cast<int64_t>(run);
  s.runq_ns = static_cast<int64_t>(wait);
  return s;
}

}  // namespace bgc::sched

#include "core/subprocess.h"

#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>

extern char** environ;

namespace bgc {

RunResult run_command(const std::vector<std::string>& argv, const std::vector<std::pair<std::string, std::string>>& env,
                      int timeout_ms, const CancelToken* cancel, const std::vector<std::string>& unset) {
  RunResult res;
  if (argv.empty()) {
    res.err = "empty command";
    return res;
  }
  if (cancel && cancel->cancelled()) {  // shutting down: start nothing
    res.cancelled = true;
    return res;
  }
  int out_pipe[2], err_pipe[2];
  if (::pipe2(out_pipe, O_CLOEXEC) != 0) {
    res.err = std::string("pipe: ") + std::strerror(errno);
    return res;
  }
  if (::pipe2(err_pipe, O_CLOEXEC) != 0) {
    ::close(out_pipe[0]);
    ::close(out_pipe[1]);
    res.err = std::string("pipe: ") + std::strerror(errno);
    return res;
  }
  // environment: the parent's, overridden by `env`
  std::map<std::string, std::string> merged;
  for (char** e = environ; e && *e; ++e) {
    const char* eq = std::strchr(*e, '=');
    if (eq) merged[std::string(*e, static_cast<size_t>(eq - *e))] = eq + 1;
  }
  for (const auto& [k, v] : env) merged[k] = v;
  for (const auto& k : unset) merged.erase(k);
  std::vector<std::string> env_strs;
  for (const auto& [k, v] : merged) env_strs.push_back(k + "=" + v);
  std::vector<char*> envp, args;
  for (auto& s : env_strs) envp.push_back(s.data());
  envp.push_back(nullptr);
  std::vector<std::string> argv_copy = argv;
  for (auto& s : argv_copy) args.push_back(s.data());
  args.push_back(nullptr);

  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  posix_spawn_file_actions_adddup2(&fa, out_pipe[1], 1);
  posix_spawn_file_actions_adddup2(&fa, err_pipe[1], 2);
  pid_t pid = -1;
  const int rc = ::posix_spawnp(&pid, args[0], &fa, nullptr, args.data(), envp.data());
  posix_spawn_file_actions_destroy(&fa);
  ::close(out_pipe[1]);
  ::close(err_pipe[1]);
  if (rc != 0) {
    ::close(out_pipe[0]);
    ::close(err_pipe[0]);
    res.err = "cannot run " + argv[0] + ": " + std::strerror(rc);
    return res;
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  pollfd fds[2] = {{out_pipe[0], POLLIN, 0}, {err_pipe[0], POLLIN, 0}};
  int open_fds = 2;
  char buf[4096];
  while (open_fds > 0) {
    const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
    if (left.count() <= 0) {
      res.timed_out = true;
      ::kill(pid, SIGKILL);
      break;
    }
    if (cancel && cancel->cancelled()) {
      res.cancelled = true;
      ::kill(pid, SIGKILL);
      break;
    }
    const int n = ::poll(fds, 2, static_cast<int>(std::min<int64_t>(left.count(), cancel ? 100 : left.count())));
    if (n < 0) {
      if (errno == EINTR) continue;
      break;
    }
    for (int i = 0; i < 2; ++i) {
      if (fds[i].fd < 0 || !(fds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      const ssize_t r = ::read(fds[i].fd, buf, sizeof(buf));
      if (r > 0) {
        (i == 0 ? res.out : res.err).append(buf, static_cast<size_t>(r));
      } else if (r == 0 || (r < 0 && errno != EINTR && errno != EAGAIN)) {
        ::close(fds[i].fd);
        fds[i].fd = -1;
        --open_fds;
      }
    }
  }
  for (auto& f : fds)
    if (f.fd >= 0) ::close(f.fd);
  int status = 0;
  while (::waitpid(pid, &status, 0) < 0 && errno == EINTR) {
  }
  if (!res.timed_out && WIFEXITED(status)) res.exit_code = WEXITSTATUS(status);
  return res;
}

}  // namespace bgc

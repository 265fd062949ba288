// Run a helper program as a child process and collect its output (kubeconfig exec
// credential plugins, gcp auth-provider commands).  posix_spawn: the calling process is
// never replaced, and no shell is involved.
#pragma once

#include <string>
#include <utility>
#include <vector>

#include "core/cancel.h"

namespace bgc {

struct RunResult {
  int exit_code = -1;      // -1: did not exit normally (signal, timeout, spawn failure)
  bool timed_out = false;
  bool cancelled = false;
  std::string out, err;
};

// argv[0] is looked up on PATH when it has no '/'.  `env` entries are added to (and
// override) the parent's environment.  The child is killed after timeout_ms, or as soon
// as `cancel` is cancelled (checked every 100 ms); nothing is started when it already is.
// `unset` names parent variables the child must not inherit.
RunResult run_command(const std::vector<std::string>& argv, const std::vector<std::pair<std::string, std::string>>& env,
                      int timeout_ms, const CancelToken* cancel = nullptr, const std::vector<std::string>& unset = {});

}  // namespace bgc

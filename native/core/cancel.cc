#include "core/cancel.h"

#include <signal.h>

#include <thread>

#include "core/log.h"

namespace bgc {

void install_shutdown_signals(std::shared_ptr<CancelToken> token) {
  sigset_t set;
  sigemptyset(&set);
  sigaddset(&set, SIGINT);
  sigaddset(&set, SIGTERM);
  pthread_sigmask(SIG_BLOCK, &set, nullptr);
  // Writing to a closed socket must not kill the process.
  signal(SIGPIPE, SIG_IGN);
  std::thread([set, token]() {
    int sig = 0;
    sigwait(&set, &sig);
    LOG_INFO("signal") << "signal received, starting graceful shutdown";
    token->cancel();
  }).detach();
}

}  // namespace bgc

// Cooperative cancellation (replaces tokio broadcast/`stopper` in the reference:
// src/controller.rs:177-205, src/admission.rs:67-94, src/synchronizer.rs:339-371).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <vector>

namespace bgc {

class CancelToken {
 public:
  void cancel() {
    std::vector<std::function<void()>> cbs;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (cancelled_.exchange(true)) return;
      cbs.swap(callbacks_);
    }
    cv_.notify_all();
    for (auto& cb : cbs) cb();
  }
  bool cancelled() const { return cancelled_.load(std::memory_order_acquire); }
  // Re-arms a cancelled token for another run of what it stops (e.g. a restarted server).
  // Only once every thread that waited on it has returned.
  void reset() {
    std::lock_guard<std::mutex> lk(mu_);
    cancelled_.store(false, std::memory_order_release);
    callbacks_.clear();
  }

  // Sleeps up to `d`; returns true if cancelled (early or already).
  template <typename Rep, typename Period>
  bool wait_for(std::chrono::duration<Rep, Period> d) const {
    std::unique_lock<std::mutex> lk(mu_);
    return cv_.wait_for(lk, d, [&] { return cancelled_.load(); });
  }
  void wait() const {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return cancelled_.load(); });
  }
  // Runs `cb` on cancellation (immediately if already cancelled).
  void on_cancel(std::function<void()> cb) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!cancelled_) {
        callbacks_.push_back(std::move(cb));
        return;
      }
    }
    cb();
  }

 private:
  mutable std::mutex mu_;
  mutable std::condition_variable cv_;
  std::atomic<bool> cancelled_{false};
  std::vector<std::function<void()>> callbacks_;
};

// Blocks SIGINT/SIGTERM in the calling thread (call from main before spawning
// threads) and starts a thread that cancels `token` when one arrives.
void install_shutdown_signals(std::shared_ptr<CancelToken> token);

}  // namespace bgc

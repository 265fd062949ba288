// Minimal reproducer of round 4's intermittent LeakSanitizer report in kube-lite (40 B
// direct + ~6 KB indirect, every frame CRYPTO_zalloc): a thread that used OpenSSL ends
// while the process exits, after OpenSSL's atexit handler (OPENSSL_cleanup) has deleted
// the thread-local key whose destructor would have freed that thread's state, and before
// LeakSanitizer's own exit-time check.  `no-atexit` (what bgc::process_init now does)
// keeps the key alive, and the same run is clean.
//
//   g++ -std=c++17 -g -fsanitize=address tools/probes/lsan_openssl_exit_race.cc -lcrypto -lpthread
//   ASAN_OPTIONS=detect_leaks=1 ./a.out            -> "Direct leak ... CRYPTO_zalloc"
//   ASAN_OPTIONS=detect_leaks=1 ./a.out no-atexit  -> no report
// (tests/unit/test_lsan_exit_race.py runs both.)
#include <openssl/crypto.h>
#include <openssl/err.h>
#include <openssl/rand.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

// Stands in for the process's own exit-time work (static destructors, other atexit
// handlers): registered before OpenSSL's handler, so it runs after OPENSSL_cleanup.
static void slow_exit_work() { std::this_thread::sleep_for(std::chrono::milliseconds(300)); }

int main(int argc, char** argv) {
  std::atexit(slow_exit_work);
  if (argc > 1 && std::strcmp(argv[1], "no-atexit") == 0) OPENSSL_init_crypto(OPENSSL_INIT_NO_ATEXIT, nullptr);
  static std::atomic<bool> used{false};
  std::thread([] {
    unsigned char b[16];
    RAND_bytes(b, sizeof b);                               // the thread's DRBGs
    ERR_put_error(ERR_LIB_SSL, 0, 1, __FILE__, __LINE__);  // its error queue
    used.store(true);
    std::this_thread::sleep_for(std::chrono::milliseconds(100));  // ends while the process exits
  }).detach();
  // exit only once the thread holds its OpenSSL state: on a loaded machine a thread that
  // first runs after OPENSSL_cleanup crashes in RAND_bytes instead of leaking
  while (!used.load()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  return 0;
}

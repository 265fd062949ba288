#include "core/log.h"
#include "core/process.h"

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <cerrno>
#include <csignal>
#include <pthread.h>
#include <sys/eventfd.h>
#include <unistd.h>

namespace bgc::log {

namespace {

struct Directive {
  std::string target;  // empty = default
  Level level;
};

std::mutex g_mu;  // serializes init()
// Directive sets are immutable once published: enabled() reads the current one through
// an atomic pointer with no lock (it runs on every log statement of every thread; the
// mutex it used to take showed up as lock contention in the control-plane profiles).
// Replaced sets are kept alive (init() runs once per process outside tests).
std::atomic<const std::vector<Directive>*> g_directives{nullptr};  // sorted: longest target first
std::vector<std::unique_ptr<const std::vector<Directive>>> g_retired;  // guarded by g_mu
std::atomic<int> g_min_level{static_cast<int>(Level::Info)};
std::atomic<bool> g_initialized{false};
std::atomic<void (*)(const std::string&)> g_sink{nullptr};

// Asynchronous stderr writer: log lines are queued and one thread writes them in batches
// (one write(2) per batch instead of one per line through stdio's stderr lock).  No
// logging thread ever waits — neither for stderr nor for another logging thread:
//
//  * append() pushes the line onto a lock-free stack (one compare-and-swap).  A stderr that
//    blocks (a container runtime's pipe read slowly, a log file under writeback throttling)
//    stalls only the writer thread.  Round 6 also removed the buffer mutex every logging
//    thread used to take: on the bench's 16-CPU share a thread preempted while holding it
//    stopped every thread that logs (the admission server logs each review at INFO) for a
//    scheduler time slice.
//  * An ERROR line wakes the writer at once (no coalescing delay) instead of writing
//    synchronously.
//  * Past kMaxBuffered queued bytes lines are dropped and counted (lines_dropped(), exported
//    as bgc_log_lines_dropped_total); the next batch written ends with one "N log lines
//    dropped" line at the place the gap occurred.
//  * Batches are taken and written under io_mu_ (writer thread and flush() only), so they
//    reach stderr in the order the lines were queued.
//  * flush() (exit, shutdown, tests) writes everything queued; it is the one caller that
//    may wait for stderr.  BGC_LOG_SYNC=1 flushes after every line (debugging only).
class AsyncWriter {
 public:
  static AsyncWriter& instance() {
    static AsyncWriter* w = new AsyncWriter();  // never destroyed: usable from atexit handlers
    return *w;
  }
  void append(const std::string& line, bool urgent) {
    const size_t queued = queued_bytes_.load(std::memory_order_relaxed);
    if (queued > 0 && queued + line.size() > kMaxBuffered) {
      dropped_pending_.fetch_add(1, std::memory_order_relaxed);
      dropped_total_.fetch_add(1, std::memory_order_relaxed);
      return;
    }
    queued_bytes_.fetch_add(line.size(), std::memory_order_relaxed);
    Node* n = new Node{nullptr, line};
    n->next = head_.load(std::memory_order_relaxed);
    // seq_cst: ordered before the sleeping_ exchange below, against the writer's store of
    // sleeping_ and its re-check of head_ (no lost wake-up)
    while (!head_.compare_exchange_weak(n->next, n, std::memory_order_seq_cst, std::memory_order_relaxed)) {
    }
    if (urgent) urgent_.store(true, std::memory_order_relaxed);
    if (!started_.load(std::memory_order_acquire)) start();
    // wake the writer only if it sleeps: no syscall per line while it is busy
    if (sleeping_.exchange(false, std::memory_order_seq_cst)) {
      const uint64_t one = 1;
      ssize_t r = ::write(wake_fd_, &one, sizeof one);
      (void)r;
    }
  }
  // Writes everything queued before the call.  Waits for stderr.
  void flush() { write_batch(); }
  uint64_t dropped() const { return dropped_total_.load(std::memory_order_relaxed); }

 private:
  struct Node {
    Node* next;
    std::string line;
  };
  static constexpr size_t kMaxBuffered = 1 << 20;
  AsyncWriter() {
    wake_fd_ = ::eventfd(0, EFD_CLOEXEC);
    std::atexit([] { AsyncWriter::instance().flush(); });
  }
  void start() {
    std::lock_guard<std::mutex> lk(start_mu_);
    if (started_.load()) return;
    std::thread([this] {
      set_thread_name("log-writer");
      // the writer must not take signals meant for the services' shutdown handling
      sigset_t all;
      sigfillset(&all);
      pthread_sigmask(SIG_BLOCK, &all, nullptr);
      while (true) {
        sleeping_.store(true, std::memory_order_seq_cst);
        if (head_.load(std::memory_order_seq_cst) == nullptr) {
          uint64_t v;
          ssize_t r = ::read(wake_fd_, &v, sizeof v);  // an append that finds sleeping_ set writes it
          (void)r;
        }
        sleeping_.store(false, std::memory_order_relaxed);
        // let a burst of lines from other threads accumulate into one write; an ERROR line
        // is written at once
        if (!urgent_.exchange(false, std::memory_order_relaxed)) {
          std::this_thread::sleep_for(std::chrono::microseconds(500));
        }
        write_batch();
      }
    }).detach();
    started_.store(true, std::memory_order_release);
  }
  // Takes everything queued (in queue order) and writes it with only io_mu_ held.
  void write_batch() {
    std::lock_guard<std::mutex> io(io_mu_);
    Node* n = head_.exchange(nullptr, std::memory_order_acquire);
    if (!n) return;
    Node* rev = nullptr;  // the stack holds the newest line first
    while (n) {
      Node* next = n->next;
      n->next = rev;
      rev = n;
      n = next;
    }
    std::string out;
    size_t bytes = 0;
    for (Node* p = rev; p; p = p->next) bytes += p->line.size();
    out.reserve(bytes + 64);
    while (rev) {
      Node* next = rev->next;
      out += rev->line;
      delete rev;
      rev = next;
    }
    queued_bytes_.fetch_sub(bytes, std::memory_order_relaxed);
    if (const uint64_t d = dropped_pending_.exchange(0, std::memory_order_relaxed)) {
      out += "log: " + std::to_string(d) + " log lines dropped (stderr blocked)\n";
    }
    size_t off = 0;
    while (off < out.size()) {
      ssize_t w = ::write(2, out.data() + off, out.size() - off);
      if (w <= 0) {
        if (w < 0 && errno == EINTR) continue;
        break;
      }
      off += static_cast<size_t>(w);
    }
  }
  std::atomic<Node*> head_{nullptr};
  std::atomic<size_t> queued_bytes_{0};
  std::atomic<uint64_t> dropped_pending_{0};  // dropped since the last batch
  std::atomic<uint64_t> dropped_total_{0};
  std::atomic<bool> urgent_{false};
  std::atomic<bool> sleeping_{false};
  std::atomic<bool> started_{false};
  std::mutex start_mu_;
  std::mutex io_mu_;  // one batch taken and written at a time (writer thread, flush())
  int wake_fd_ = -1;
};

bool g_sync_writes = std::getenv("BGC_LOG_SYNC") && std::string(std::getenv("BGC_LOG_SYNC")) == "1";
// BGC_LOG_FORMAT=json: one JSON object per line in tracing-subscriber's `fmt().json()` layout
// ({"timestamp","level","fields":{"message"},"target"}), for log pipelines that parse it.
bool g_json = std::getenv("BGC_LOG_FORMAT") && std::string(std::getenv("BGC_LOG_FORMAT")) == "json";

void append_json_string(std::string& out, std::string_view s) {
  static const char kHex[] = "0123456789abcdef";
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out.append("\\\""); break;
      case '\\': out.append("\\\\"); break;
      case '\n': out.append("\\n"); break;
      case '\r': out.append("\\r"); break;
      case '\t': out.append("\\t"); break;
      default:
        if (c < 0x20) {
          out.append("\\u00");
          out.push_back(kHex[c >> 4]);
          out.push_back(kHex[c & 15]);
        } else {
          out.push_back(static_cast<char>(c));
        }
    }
  }
  out.push_back('"');
}

bool parse_level(std::string s, Level& out) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  if (s == "trace") out = Level::Trace;
  else if (s == "debug") out = Level::Debug;
  else if (s == "info") out = Level::Info;
  else if (s == "warn" || s == "warning") out = Level::Warn;
  else if (s == "error") out = Level::Error;
  else if (s == "off") out = Level::Off;
  else return false;
  return true;
}

const char* level_name(Level l) {
  switch (l) {
    case Level::Trace: return "TRACE";
    case Level::Debug: return "DEBUG";
    case Level::Info: return " INFO";
    case Level::Warn: return " WARN";
    case Level::Error: return "ERROR";
    default: return "  OFF";
  }
}

}  // namespace

void init(const std::string& spec) {
  std::vector<Directive> ds;
  bool have_default = false;
  size_t start = 0;
  while (start <= spec.size()) {
    size_t comma = spec.find(',', start);
    std::string item = spec.substr(start, comma == std::string::npos ? std::string::npos : comma - start);
    // trim
    while (!item.empty() && item.front() == ' ') item.erase(0, 1);
    while (!item.empty() && item.back() == ' ') item.pop_back();
    if (!item.empty()) {
      size_t eq = item.find('=');
      Level lvl;
      if (eq == std::string::npos) {
        if (parse_level(item, lvl)) {
          ds.push_back({"", lvl});
          have_default = true;
        } else {
          ds.push_back({item, Level::Trace});  // bare target enables everything for it
        }
      } else if (parse_level(item.substr(eq + 1), lvl)) {
        ds.push_back({item.substr(0, eq), lvl});
      }
    }
    if (comma == std::string::npos) break;
    start = comma + 1;
  }
  // tracing Targets: no default directive means "off" for unmatched targets, unless
  // the whole spec was empty/invalid, in which case INFO is the default.
  if (ds.empty()) ds.push_back({"", Level::Info});
  else if (!have_default) ds.push_back({"", Level::Off});
  std::stable_sort(ds.begin(), ds.end(),
                   [](const Directive& a, const Directive& b) { return a.target.size() > b.target.size(); });
  int mn = static_cast<int>(Level::Off);
  for (auto& d : ds) mn = std::min(mn, static_cast<int>(d.level));
  std::lock_guard<std::mutex> lk(g_mu);
  auto next = std::make_unique<const std::vector<Directive>>(std::move(ds));
  g_directives.store(next.get(), std::memory_order_release);
  g_retired.push_back(std::move(next));
  g_min_level.store(mn);
  g_initialized.store(true);
}

void flush() { AsyncWriter::instance().flush(); }

void init_from_env(const char* var) {
  const char* v = std::getenv(var);
  init(v ? v : "info");
}

bool enabled(Level lvl, std::string_view target) {
  if (!g_initialized.load(std::memory_order_relaxed)) init_from_env();
  if (static_cast<int>(lvl) < g_min_level.load(std::memory_order_relaxed)) return false;
  const std::vector<Directive>* ds = g_directives.load(std::memory_order_acquire);
  if (!ds) return false;
  for (const auto& d : *ds) {
    if (d.target.empty() ||
        (target.substr(0, d.target.size()) == d.target &&
         (target.size() == d.target.size() || target.substr(d.target.size(), 2) == "::"))) {
      return static_cast<int>(lvl) >= static_cast<int>(d.level);
    }
  }
  return false;
}

void set_sink(void (*sink)(const std::string&)) {
  flush();
  g_sink.store(sink);
}

void write(Level lvl, std::string_view target, std::string_view msg) {
  auto now = std::chrono::system_clock::now();
  auto secs = std::chrono::time_point_cast<std::chrono::seconds>(now);
  auto micros = std::chrono::duration_cast<std::chrono::microseconds>(now - secs).count();
  // gmtime_r takes glibc's process-wide tz lock on every call: the date part is formatted
  // once per second per thread and reused (the lock showed up in the services' profiles).
  thread_local std::time_t cached_sec = -1;
  thread_local char ts[96];  // "YYYY-MM-DDTHH:MM:SS.uuuuuuZ"
  thread_local int date_len = 0;
  const std::time_t t = std::chrono::system_clock::to_time_t(secs);
  if (t != cached_sec) {
    std::tm tm{};
    gmtime_r(&t, &tm);
    date_len = std::snprintf(ts, 80, "%04d-%02d-%02dT%02d:%02d:%02d.", tm.tm_year + 1900, tm.tm_mon + 1,
                             tm.tm_mday, tm.tm_hour, tm.tm_min, tm.tm_sec);
    cached_sec = t;
  }
  for (int i = date_len + 5; i >= date_len; --i, micros /= 10) ts[i] = static_cast<char>('0' + micros % 10);
  ts[date_len + 6] = 'Z';
  ts[date_len + 7] = '\0';
  std::string line;
  line.reserve(msg.size() + target.size() + 80);
  if (g_json) {
    std::string_view lv = level_name(lvl);
    while (!lv.empty() && lv.front() == ' ') lv.remove_prefix(1);
    line.append("{\"timestamp\":\"").append(ts).append("\",\"level\":\"").append(lv);
    line.append("\",\"fields\":{\"message\":");
    append_json_string(line, msg);
    line.append("},\"target\":");
    append_json_string(line, target);
    line.append("}\n");
  } else {
    line.append(ts).append(" ").append(level_name(lvl)).append(" ");
    line.append(target).append(": ").append(msg).push_back('\n');
  }
  if (auto sink = g_sink.load()) {
    sink(line);
    return;
  }
  auto& w = AsyncWriter::instance();
  w.append(line, lvl >= Level::Error);
  if (g_sync_writes) w.flush();
}

uint64_t lines_dropped() { return AsyncWriter::instance().dropped(); }

}  // namespace bgc::log

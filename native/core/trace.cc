#include "core/trace.h"

#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

#include "core/json.h"
#include "core/metrics.h"

namespace bgc::trace {

namespace {

struct Mark {
  std::string name;
  std::string stage;
  int64_t t;
};

// What arm() set: immutable once published (mark() reads it through an atomic pointer
// without a lock; replaced configurations are kept, arm() runs a few times per bench run).
struct Config {
  std::string prefix;                 // as armed (comma list)
  std::vector<std::string> prefixes;  // its items
  size_t capacity = 0;
};

// Marks are kept per thread: a mark takes only its own thread's buffer lock, which nothing
// else takes except a dump.  One process-wide lock here was itself a source of the tails
// being measured: a thread preempted while holding it (16 CPUs, hundreds of threads) stopped
// every thread that marks — kube-lite's committers hold a store lock when they mark — for a
// scheduler time slice.
struct ThreadBuf {
  std::mutex mu;
  std::vector<Mark> marks;
};

std::atomic<const Config*> g_config{nullptr};  // null: disarmed
std::atomic<size_t> g_count{0};                // marks kept since arm()
std::atomic<uint64_t> g_dropped{0};

// Never destroyed: threads that mark may outlive static destruction at exit.
struct Registry {
  std::mutex mu;  // everything below
  std::vector<std::shared_ptr<ThreadBuf>> bufs;
  std::vector<std::unique_ptr<const Config>> retired;
  std::string last_prefix;
};
Registry& reg() {
  static Registry* r = new Registry();
  return *r;
}

ThreadBuf& thread_buf() {
  thread_local std::shared_ptr<ThreadBuf> buf = [] {
    auto b = std::make_shared<ThreadBuf>();
    std::lock_guard<std::mutex> lk(reg().mu);
    reg().bufs.push_back(b);
    return b;
  }();
  return *buf;
}

}  // namespace

bool armed() { return g_config.load(std::memory_order_acquire) != nullptr; }

void mark_at(std::string_view name, std::string_view stage, int64_t t_ns) {
  const Config* c = g_config.load(std::memory_order_acquire);
  if (!c) return;
  bool match = false;
  for (const auto& p : c->prefixes) match = match || name.substr(0, p.size()) == p;
  if (!match) return;
  if (g_count.fetch_add(1, std::memory_order_relaxed) >= c->capacity) {
    g_dropped.fetch_add(1, std::memory_order_relaxed);
    return;
  }
  ThreadBuf& b = thread_buf();
  std::lock_guard<std::mutex> lk(b.mu);
  b.marks.push_back({std::string(name), std::string(stage), t_ns});
}

void mark(std::string_view name, std::string_view stage) {
  if (!armed()) return;
  mark_at(name, stage, metrics::now_ns());
}

void arm(const std::string& prefix, size_t capacity) {
  auto c = std::make_unique<Config>();
  c->prefix = prefix;
  size_t start = 0;
  while (start <= prefix.size()) {
    const size_t comma = prefix.find(',', start);
    std::string item = prefix.substr(start, comma == std::string::npos ? std::string::npos : comma - start);
    if (!item.empty()) c->prefixes.push_back(std::move(item));
    if (comma == std::string::npos) break;
    start = comma + 1;
  }
  c->capacity = capacity;
  Registry& r = reg();
  std::lock_guard<std::mutex> lk(r.mu);
  g_config.store(nullptr, std::memory_order_release);
  for (auto& b : r.bufs) {
    std::lock_guard<std::mutex> bl(b->mu);
    b->marks.clear();
  }
  g_count.store(0);
  g_dropped.store(0);
  r.last_prefix = prefix;
  if (!c->prefixes.empty()) {
    g_config.store(c.get(), std::memory_order_release);
    r.retired.push_back(std::move(c));
  }
}

void disarm() { g_config.store(nullptr, std::memory_order_release); }

std::string dump_json(bool take) {
  std::vector<Mark> marks;
  json::Value out = json::Value::object();
  {
    Registry& r = reg();
    std::lock_guard<std::mutex> lk(r.mu);
    out["prefix"] = r.last_prefix;
    out["armed"] = armed();
    if (take) g_config.store(nullptr, std::memory_order_release);
    out["dropped"] = static_cast<unsigned long long>(g_dropped.load());
    for (auto& b : r.bufs) {
      std::lock_guard<std::mutex> bl(b->mu);
      if (take) {
        for (auto& m : b->marks) marks.push_back(std::move(m));
        b->marks.clear();
        b->marks.shrink_to_fit();
      } else {
        marks.insert(marks.end(), b->marks.begin(), b->marks.end());
      }
    }
    if (take) {
      // buffers of threads that have exited (only this list still holds them)
      std::vector<std::shared_ptr<ThreadBuf>> live;
      for (auto& b : r.bufs) {
        if (b.use_count() > 1) live.push_back(std::move(b));
      }
      r.bufs.swap(live);
      g_dropped.store(0);
      g_count.store(0);
    }
  }
  json::Value arr = json::Value::array();
  for (auto& m : marks) {
    json::Value e = json::Value::array();
    e.push_back(std::move(m.name));
    e.push_back(std::move(m.stage));
    e.push_back(static_cast<long long>(m.t));
    arr.push_back(std::move(e));
  }
  out["marks"] = std::move(arr);
  return out.dump();
}

}  // namespace bgc::trace

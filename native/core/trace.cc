#include "core/trace.h"

#include <atomic>
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

std::atomic<bool> g_armed{false};
std::mutex g_mu;  // everything below
std::string g_prefix;                // as armed (comma list)
std::vector<std::string> g_prefixes;  // its items
size_t g_capacity = 0;
uint64_t g_dropped = 0;
std::vector<Mark> g_marks;

}  // namespace

bool armed() { return g_armed.load(std::memory_order_relaxed); }

void mark_at(std::string_view name, std::string_view stage, int64_t t_ns) {
  if (!armed()) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_armed.load(std::memory_order_relaxed)) return;
  bool match = false;
  for (const auto& p : g_prefixes) match = match || name.substr(0, p.size()) == p;
  if (!match) return;
  if (g_marks.size() >= g_capacity) {
    ++g_dropped;
    return;
  }
  g_marks.push_back({std::string(name), std::string(stage), t_ns});
}

void mark(std::string_view name, std::string_view stage) {
  if (!armed()) return;
  mark_at(name, stage, metrics::now_ns());
}

void arm(const std::string& prefix, size_t capacity) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_prefix = prefix;
  g_prefixes.clear();
  size_t start = 0;
  while (start <= prefix.size()) {
    const size_t comma = prefix.find(',', start);
    std::string item = prefix.substr(start, comma == std::string::npos ? std::string::npos : comma - start);
    if (!item.empty()) g_prefixes.push_back(std::move(item));
    if (comma == std::string::npos) break;
    start = comma + 1;
  }
  g_capacity = capacity;
  g_dropped = 0;
  g_marks.clear();
  g_marks.reserve(std::min<size_t>(capacity, 1 << 16));
  g_armed.store(!g_prefixes.empty(), std::memory_order_relaxed);
}

void disarm() {
  std::lock_guard<std::mutex> lk(g_mu);
  g_armed.store(false, std::memory_order_relaxed);
}

std::string dump_json(bool take) {
  std::vector<Mark> marks;
  json::Value out = json::Value::object();
  {
    std::lock_guard<std::mutex> lk(g_mu);
    out["prefix"] = g_prefix;
    out["armed"] = g_armed.load(std::memory_order_relaxed);
    out["dropped"] = static_cast<unsigned long long>(g_dropped);
    if (take) {
      marks.swap(g_marks);
      g_armed.store(false, std::memory_order_relaxed);
      g_dropped = 0;
    } else {
      marks = g_marks;
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

#include "core/log.h"

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <mutex>
#include <vector>

namespace bgc::log {

namespace {

struct Directive {
  std::string target;  // empty = default
  Level level;
};

std::mutex g_mu;
std::vector<Directive> g_directives;  // sorted: longest target first
std::atomic<int> g_min_level{static_cast<int>(Level::Info)};
std::atomic<bool> g_initialized{false};
void (*g_sink)(const std::string&) = nullptr;

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
  g_directives = std::move(ds);
  g_min_level.store(mn);
  g_initialized.store(true);
}

void init_from_env(const char* var) {
  const char* v = std::getenv(var);
  init(v ? v : "info");
}

bool enabled(Level lvl, std::string_view target) {
  if (!g_initialized.load(std::memory_order_relaxed)) init_from_env();
  if (static_cast<int>(lvl) < g_min_level.load(std::memory_order_relaxed)) return false;
  std::lock_guard<std::mutex> lk(g_mu);
  for (const auto& d : g_directives) {
    if (d.target.empty() ||
        (target.substr(0, d.target.size()) == d.target &&
         (target.size() == d.target.size() || target.substr(d.target.size(), 2) == "::"))) {
      return static_cast<int>(lvl) >= static_cast<int>(d.level);
    }
  }
  return false;
}

void set_sink(void (*sink)(const std::string&)) { g_sink = sink; }

void write(Level lvl, std::string_view target, std::string_view msg) {
  auto now = std::chrono::system_clock::now();
  auto secs = std::chrono::time_point_cast<std::chrono::seconds>(now);
  auto micros = std::chrono::duration_cast<std::chrono::microseconds>(now - secs).count();
  std::time_t t = std::chrono::system_clock::to_time_t(now);
  std::tm tm{};
  gmtime_r(&t, &tm);
  char ts[64];
  std::snprintf(ts, sizeof(ts), "%04d-%02d-%02dT%02d:%02d:%02d.%06ldZ", tm.tm_year + 1900, tm.tm_mon + 1,
                tm.tm_mday, tm.tm_hour, tm.tm_min, tm.tm_sec, static_cast<long>(micros));
  std::string line;
  line.reserve(msg.size() + target.size() + 48);
  line.append(ts).append(" ").append(level_name(lvl)).append(" ");
  line.append(target).append(": ").append(msg).push_back('\n');
  if (g_sink) {
    g_sink(line);
    return;
  }
  std::fwrite(line.data(), 1, line.size(), stderr);
}

}  // namespace bgc::log

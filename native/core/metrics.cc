#include "core/metrics.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <malloc.h>
#include <unistd.h>
#include <sstream>

#include "core/env_config.h"
#include "core/json.h"
#include "core/log.h"

namespace bgc::metrics {

namespace {
uint64_t to_bits(double d) {
  uint64_t u;
  std::memcpy(&u, &d, sizeof(u));
  return u;
}
double from_bits(uint64_t u) {
  double d;
  std::memcpy(&d, &u, sizeof(d));
  return d;
}
void atomic_add(std::atomic<uint64_t>& a, double v) {
  uint64_t cur = a.load(std::memory_order_relaxed);
  while (!a.compare_exchange_weak(cur, to_bits(from_bits(cur) + v), std::memory_order_relaxed)) {
  }
}
std::string fmt_double(double v) {
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  std::ostringstream os;
  os.precision(17);
  os << v;
  return os.str();
}
}  // namespace

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void Counter::inc(double v) { atomic_add(bits_, v); }
double Counter::value() const { return from_bits(bits_.load(std::memory_order_relaxed)); }
void Gauge::set(double v) { bits_.store(to_bits(v), std::memory_order_relaxed); }
double Gauge::value() const { return from_bits(bits_.load(std::memory_order_relaxed)); }

Histogram::Histogram(std::vector<double> buckets) : bounds_(std::move(buckets)) {
  std::sort(bounds_.begin(), bounds_.end());
  counts_.reset(new std::atomic<uint64_t>[bounds_.size() + 1]);
  for (size_t i = 0; i <= bounds_.size(); ++i) counts_[i].store(0);
}

void Histogram::observe(double v) {
  size_t idx = static_cast<size_t>(std::lower_bound(bounds_.begin(), bounds_.end(), v) - bounds_.begin());
  counts_[idx].fetch_add(1, std::memory_order_relaxed);
  atomic_add(sum_bits_, v);
  count_.fetch_add(1, std::memory_order_relaxed);
}

std::vector<uint64_t> Histogram::bucket_counts() const {
  std::vector<uint64_t> out(bounds_.size() + 1);
  for (size_t i = 0; i <= bounds_.size(); ++i) out[i] = counts_[i].load(std::memory_order_relaxed);
  return out;
}
double Histogram::sum() const { return from_bits(sum_bits_.load(std::memory_order_relaxed)); }
uint64_t Histogram::count() const { return count_.load(std::memory_order_relaxed); }

namespace {
std::atomic<bool> g_samples_enabled{false};
std::atomic<size_t> g_sample_capacity{size_t{1} << 22};
std::atomic<bool> g_debug_endpoints{false};
}  // namespace

void configure_samples(bool enabled, size_t capacity) {
  g_sample_capacity.store(capacity ? capacity : 1);
  g_samples_enabled.store(enabled);
}
bool samples_enabled() { return g_samples_enabled.load(std::memory_order_relaxed); }
size_t sample_capacity() { return g_sample_capacity.load(std::memory_order_relaxed); }

void configure_debug(const EnvConfig& env) {
  const bool on = env.boolean_or("debug_endpoints", false);
  g_debug_endpoints.store(on);
  configure_samples(on, static_cast<size_t>(env.u64_or("debug_sample_capacity", uint64_t{1} << 22)));
}
void set_debug_endpoints(bool on) {
  g_debug_endpoints.store(on);
  configure_samples(on, sample_capacity());
}
bool debug_endpoints_enabled() { return g_debug_endpoints.load(std::memory_order_relaxed); }

// capacity 0: the process-wide setting, read when a sample arrives
SampleLog::SampleLog(size_t capacity) : cap_(capacity) {}

void SampleLog::add(double v, Counter* linked) {
  const bool keep = samples_enabled();
  const size_t cap = cap_ ? cap_ : sample_capacity();
  std::lock_guard<std::mutex> lk(mu_);
  ++lifetime_;
  ++total_;
  if (linked) linked->inc();
  if (keep && buf_.size() < cap) buf_.push_back(v);
  else ++dropped_;
}

void SampleLog::link(const std::string& key, Counter* c) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : linked_) {
    if (kv.first == key) {
      kv.second = c;
      return;
    }
  }
  linked_.emplace_back(key, c);
}

void SampleLog::fill_counts(Snapshot& s) const {
  s.total = total_;
  s.dropped = dropped_;
  s.lifetime = lifetime_;
  s.capacity = cap_ ? cap_ : sample_capacity();
  for (const auto& kv : linked_) s.linked.emplace_back(kv.first, kv.second->value());
}

SampleLog::Snapshot SampleLog::snapshot() const {
  Snapshot s;
  std::lock_guard<std::mutex> lk(mu_);
  s.samples = buf_;
  fill_counts(s);
  return s;
}

SampleLog::Snapshot SampleLog::clear() {
  Snapshot s;
  std::lock_guard<std::mutex> lk(mu_);
  buf_.clear();
  buf_.shrink_to_fit();
  total_ = 0;
  dropped_ = 0;
  fill_counts(s);
  return s;
}

uint64_t SampleLog::total() const {
  std::lock_guard<std::mutex> lk(mu_);
  return total_;
}

double quantile(std::vector<double> v, double q) {
  if (v.empty()) return std::nan("");
  std::sort(v.begin(), v.end());
  // nearest-rank
  double rank = std::ceil(q * static_cast<double>(v.size()));
  size_t idx = rank < 1 ? 0 : static_cast<size_t>(rank) - 1;
  if (idx >= v.size()) idx = v.size() - 1;
  return v[idx];
}

std::vector<double> default_latency_buckets() {
  std::vector<double> b;
  double x = 50e-6;
  while (x < 30.0) {
    b.push_back(x);
    x *= 1.5;
  }
  b.push_back(30.0);
  return b;
}

Registry& Registry::global() {
  static Registry* r = new Registry();
  return *r;
}

std::string render_labels(const Labels& labels, const std::string& extra_key, const std::string& extra_val) {
  if (labels.empty() && extra_key.empty()) return "";
  std::string out = "{";
  bool first = true;
  auto add = [&](const std::string& k, const std::string& v) {
    if (!first) out += ",";
    first = false;
    out += k + "=\"";
    for (char c : v) {
      if (c == '\\' || c == '"') out.push_back('\\');
      if (c == '\n') {
        out += "\\n";
        continue;
      }
      out.push_back(c);
    }
    out += "\"";
  };
  for (auto& kv : labels) add(kv.first, kv.second);
  if (!extra_key.empty()) add(extra_key, extra_val);
  return out + "}";
}

Counter& Registry::counter(const std::string& name, const std::string& help, const Labels& labels) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& f = families_[name];
  f.type = "counter";
  f.help = help;
  auto& slot = f.counters[render_labels(labels)];
  if (!slot) slot = std::make_unique<Counter>();
  return *slot;
}

Gauge& Registry::gauge(const std::string& name, const std::string& help, const Labels& labels) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& f = families_[name];
  f.type = "gauge";
  f.help = help;
  auto& slot = f.gauges[render_labels(labels)];
  if (!slot) slot = std::make_unique<Gauge>();
  return *slot;
}

Histogram& Registry::histogram(const std::string& name, const std::string& help, const Labels& labels,
                               std::vector<double> buckets) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& f = families_[name];
  f.type = "histogram";
  f.help = help;
  auto& slot = f.histograms[render_labels(labels)];
  if (!slot) slot = std::make_unique<Histogram>(std::move(buckets));
  return *slot;
}

SampleLog& Registry::samples(const std::string& name) {
  std::lock_guard<std::mutex> lk(mu_);
  auto& slot = samples_[name];
  if (!slot) slot = std::make_unique<SampleLog>(0);
  return *slot;
}

SampleLog* Registry::find_samples(const std::string& name) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = samples_.find(name);
  return it == samples_.end() ? nullptr : it->second.get();
}

void append_process_memory(std::string& out);

std::string Registry::render() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::string out;
  for (const auto& [name, f] : families_) {
    out += "# HELP " + name + " " + f.help + "\n";
    out += "# TYPE " + name + " " + f.type + "\n";
    for (const auto& [lbl, c] : f.counters) out += name + lbl + " " + fmt_double(c->value()) + "\n";
    for (const auto& [lbl, g] : f.gauges) out += name + lbl + " " + fmt_double(g->value()) + "\n";
    for (const auto& [lbl, h] : f.histograms) {
      // re-open label set to add `le`
      std::string base = lbl.empty() ? "" : lbl.substr(1, lbl.size() - 2);
      auto counts = h->bucket_counts();
      uint64_t cum = 0;
      for (size_t i = 0; i < h->buckets().size(); ++i) {
        cum += counts[i];
        out += name + "_bucket{" + base + (base.empty() ? "" : ",") + "le=\"" + fmt_double(h->buckets()[i]) +
               "\"} " + std::to_string(cum) + "\n";
      }
      cum += counts.back();
      out += name + "_bucket{" + base + (base.empty() ? "" : ",") + "le=\"+Inf\"} " + std::to_string(cum) + "\n";
      out += name + "_sum" + lbl + " " + fmt_double(h->sum()) + "\n";
      out += name + "_count" + lbl + " " + std::to_string(h->count()) + "\n";
    }
  }
  out += "# HELP bgc_debug_sample_logs Latency sample logs in this process (fixed at start-up)\n"
         "# TYPE bgc_debug_sample_logs gauge\nbgc_debug_sample_logs " + std::to_string(samples_.size()) + "\n";
  append_process_memory(out);
  return out;
}

// Process memory next to the registry's families: RSS from /proc/self/statm and the glibc
// heap split into bytes handed out (including chunks parked in per-thread caches) and free
// bytes kept by the arenas (address space, not RSS: malloc_trim returns their pages).
void append_process_memory(std::string& out) {
  long pages_total = 0, pages_rss = 0;
  {
    std::ifstream statm("/proc/self/statm");
    statm >> pages_total >> pages_rss;
  }
  const double page = static_cast<double>(sysconf(_SC_PAGESIZE));
  // mallinfo2 walks every free chunk of every arena with that arena locked: on a large,
  // fragmented heap it stalls the process's allocating threads for milliseconds (274 ms for
  // 1.3 GB of fragmented free memory in a probe).  A scrape therefore reuses a reading up to
  // BGC_HEAP_STATS_SECS old (default 60).
  static std::mutex mi_mu;
  static struct mallinfo2 mi_cached {};
  static int64_t mi_at = 0;
  static const int64_t mi_max_age_ns = [] {
    const char* e = std::getenv("BGC_HEAP_STATS_SECS");
    return static_cast<int64_t>(e ? std::atol(e) : 60) * 1000000000LL;
  }();
  struct mallinfo2 mi;
  {
    std::lock_guard<std::mutex> lk(mi_mu);
    const int64_t now = now_ns();
    if (mi_at == 0 || now - mi_at >= mi_max_age_ns) {
      mi_cached = mallinfo2();
      mi_at = now;
    }
    mi = mi_cached;
  }
  auto gauge = [&out](const char* name, const char* help, double v) {
    out += std::string("# HELP ") + name + " " + help + "\n# TYPE " + name + " gauge\n" + name + " " + fmt_double(v) + "\n";
  };
  gauge("bgc_process_resident_memory_bytes", "Resident set size", static_cast<double>(pages_rss) * page);
  gauge("bgc_heap_allocated_bytes", "malloc bytes in use (arena + mmapped chunks, incl. thread caches)",
        static_cast<double>(mi.uordblks + mi.hblkhd));
  gauge("bgc_heap_free_bytes", "free bytes in malloc arenas (address space; trimmed pages are not resident)",
        static_cast<double>(mi.fordblks));
  out += "# HELP bgc_log_lines_dropped_total Log lines dropped while stderr was blocked (1 MiB already buffered)\n"
         "# TYPE bgc_log_lines_dropped_total counter\nbgc_log_lines_dropped_total " +
         std::to_string(log::lines_dropped()) + "\n";
}

std::vector<std::string> Registry::sample_names() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> out;
  for (auto& kv : samples_) out.push_back(kv.first);
  return out;
}

namespace {
json::Value snapshot_json(const std::string& name, const SampleLog::Snapshot& s) {
  json::Value out = json::Value::object();
  out["name"] = name;
  out["total"] = static_cast<unsigned long long>(s.total);
  out["dropped"] = static_cast<unsigned long long>(s.dropped);
  out["lifetime"] = static_cast<unsigned long long>(s.lifetime);
  out["capacity"] = static_cast<unsigned long long>(s.capacity);
  out["complete"] = s.dropped == 0;
  json::Value linked = json::Value::object();
  for (const auto& kv : s.linked) linked[kv.first] = kv.second;
  out["linked"] = std::move(linked);
  return out;
}
}  // namespace

std::string Registry::render_samples_json(const std::string& name) const {
  const SampleLog* log = find_samples(name);
  if (!log) return "";
  SampleLog::Snapshot s = log->snapshot();
  json::Value out = snapshot_json(name, s);
  json::Value arr = json::Value::array();
  for (double d : s.samples) arr.push_back(d);
  out["samples"] = std::move(arr);
  return out.dump();
}

std::string Registry::clear_samples_json(const std::string& name) const {
  SampleLog* log = find_samples(name);
  if (!log) return "";
  return snapshot_json(name, log->clear()).dump();
}

Timer::Timer(Histogram* h, SampleLog* s) : h_(h), s_(s), start_ns_(now_ns()) {}
Timer::~Timer() {
  double e = elapsed();
  if (h_) h_->observe(e);
  if (s_) s_->add(e);
}
double Timer::elapsed() const { return static_cast<double>(now_ns() - start_ns_) * 1e-9; }

}  // namespace bgc::metrics

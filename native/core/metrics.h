// Prometheus text-format metrics plus an exact-latency sample recorder.
//
// The reference exposes no metrics at all; every binary here serves
// `/metrics` on its health listener.  With CONF_DEBUG_ENDPOINTS=true (tests and the bench
// harness only; off in the binaries and the chart) it also keeps every latency sample of
// a window and serves them on `/debug/samples/<name>`, which the harness turns into exact
// p50/p99 values.
#pragma once

#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace bgc {
class EnvConfig;
}

namespace bgc::metrics {

using Labels = std::vector<std::pair<std::string, std::string>>;

class Counter {
 public:
  void inc(double v = 1.0);
  double value() const;

 private:
  std::atomic<uint64_t> bits_{0};  // double stored as bits for atomic add
};

class Gauge {
 public:
  void set(double v);
  double value() const;

 private:
  std::atomic<uint64_t> bits_{0};
};

class Histogram {
 public:
  explicit Histogram(std::vector<double> buckets);
  void observe(double v);
  std::vector<uint64_t> bucket_counts() const;
  const std::vector<double>& buckets() const { return bounds_; }
  double sum() const;
  uint64_t count() const;

 private:
  std::vector<double> bounds_;
  std::unique_ptr<std::atomic<uint64_t>[]> counts_;
  std::atomic<uint64_t> sum_bits_{0};
  std::atomic<uint64_t> count_{0};
};

// Every observation of a measurement window (seconds), for exact quantiles.
//
// Nothing is overwritten: once `capacity` samples are held, further ones are counted as
// dropped, so a reader can tell a complete window from a truncated one (the bench refuses
// to report a percentile over a truncated window).  Samples are only kept while sample
// recording is enabled (configure_samples); otherwise add() just counts.
//
// Linked counters: a Prometheus counter passed to add() is incremented inside the same
// critical section that records the sample, and snapshot()/clear() read every linked
// counter under that lock.  The samples of a window are then exactly the increments of
// its linked counters between clear() and snapshot(), by construction.
class SampleLog {
 public:
  explicit SampleLog(size_t capacity);
  void add(double v, Counter* linked = nullptr);
  // Registers `c` under `key` (its exposition name + labels) for snapshots.
  void link(const std::string& key, Counter* c);

  struct Snapshot {
    std::vector<double> samples;
    uint64_t total = 0;     // add() calls since the last clear (kept + dropped)
    uint64_t dropped = 0;   // not kept: capacity reached or recording disabled
    uint64_t lifetime = 0;  // add() calls since start
    uint64_t capacity = 0;
    std::vector<std::pair<std::string, double>> linked;  // linked counter values
  };
  Snapshot snapshot() const;
  Snapshot clear();  // returns the counts at the instant of clearing (no samples)
  uint64_t total() const;

 private:
  mutable std::mutex mu_;
  size_t cap_;
  std::vector<double> buf_;
  uint64_t total_ = 0, dropped_ = 0, lifetime_ = 0;
  std::vector<std::pair<std::string, Counter*>> linked_;
  void fill_counts(Snapshot& s) const;  // mu_ held
};

// Sample recording (off by default: production binaries keep no raw samples).
void configure_samples(bool enabled, size_t capacity = size_t{1} << 22);
bool samples_enabled();
size_t sample_capacity();
// Reads CONF_DEBUG_ENDPOINTS (bool, default false) and CONF_DEBUG_SAMPLE_CAPACITY
// (default 4,194,304 samples per log): the /debug/samples routes and sample recording.
void configure_debug(const EnvConfig& env);
void set_debug_endpoints(bool on);  // routes + recording (kube-lite, a test fixture)
bool debug_endpoints_enabled();

double quantile(std::vector<double> v, double q);

std::vector<double> default_latency_buckets();  // 50us .. 30s, log spaced

class Registry {
 public:
  static Registry& global();

  Counter& counter(const std::string& name, const std::string& help, const Labels& labels = {});
  Gauge& gauge(const std::string& name, const std::string& help, const Labels& labels = {});
  Histogram& histogram(const std::string& name, const std::string& help, const Labels& labels = {},
                       std::vector<double> buckets = default_latency_buckets());
  SampleLog& samples(const std::string& name);             // creates the log
  SampleLog* find_samples(const std::string& name) const;  // nullptr if absent

  std::string render() const;  // Prometheus exposition format 0.0.4
  // JSON of one log: {"name","total","dropped","lifetime","capacity","complete",
  // "linked":{...},"samples":[...]}; clear_samples_json() clears it and returns the same
  // fields without samples.  Both return "" for an unknown name (never create one).
  std::string render_samples_json(const std::string& name) const;
  std::string clear_samples_json(const std::string& name) const;
  std::vector<std::string> sample_names() const;

 private:
  struct Family {
    std::string type, help;
    std::map<std::string, std::unique_ptr<Counter>> counters;
    std::map<std::string, std::unique_ptr<Gauge>> gauges;
    std::map<std::string, std::unique_ptr<Histogram>> histograms;
  };
  mutable std::mutex mu_;
  std::map<std::string, Family> families_;
  std::map<std::string, std::unique_ptr<SampleLog>> samples_;
};

std::string render_labels(const Labels& labels, const std::string& extra_key = "",
                          const std::string& extra_val = "");

// RAII timer: observes elapsed seconds into histogram (and optional sample log).
class Timer {
 public:
  Timer(Histogram* h, SampleLog* s = nullptr);
  ~Timer();
  double elapsed() const;
  void cancel() { h_ = nullptr; s_ = nullptr; }

 private:
  Histogram* h_;
  SampleLog* s_;
  int64_t start_ns_;
};

int64_t now_ns();  // steady clock

}  // namespace bgc::metrics

// Prometheus text-format metrics plus an exact-latency sample recorder.
//
// The reference exposes no metrics at all; every binary here serves
// `/metrics` on its health listener and `/debug/samples` with raw latencies, which the
// bench harness turns into exact p50/p99 values.
#pragma once

#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

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

// Keeps the last `capacity` observations (seconds) for exact quantiles.
class SampleRing {
 public:
  explicit SampleRing(size_t capacity = 1 << 16);
  void add(double v);
  std::vector<double> snapshot() const;
  void clear();
  uint64_t total() const;

 private:
  mutable std::mutex mu_;
  size_t cap_;
  std::vector<double> buf_;
  size_t next_ = 0;
  uint64_t total_ = 0;
};

double quantile(std::vector<double> v, double q);

std::vector<double> default_latency_buckets();  // 50us .. 30s, log spaced

class Registry {
 public:
  static Registry& global();

  Counter& counter(const std::string& name, const std::string& help, const Labels& labels = {});
  Gauge& gauge(const std::string& name, const std::string& help, const Labels& labels = {});
  Histogram& histogram(const std::string& name, const std::string& help, const Labels& labels = {},
                       std::vector<double> buckets = default_latency_buckets());
  SampleRing& samples(const std::string& name);

  std::string render() const;  // Prometheus exposition format 0.0.4
  std::string render_samples_json(const std::string& name) const;
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
  std::map<std::string, std::unique_ptr<SampleRing>> samples_;
};

std::string render_labels(const Labels& labels, const std::string& extra_key = "",
                          const std::string& extra_val = "");

// RAII timer: observes elapsed seconds into histogram (and optional sample ring).
class Timer {
 public:
  Timer(Histogram* h, SampleRing* s = nullptr);
  ~Timer();
  double elapsed() const;
  void cancel() { h_ = nullptr; s_ = nullptr; }

 private:
  Histogram* h_;
  SampleRing* s_;
  int64_t start_ns_;
};

int64_t now_ns();  // steady clock

}  // namespace bgc::metrics

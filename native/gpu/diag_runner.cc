#include "gpu/diag_runner.h"

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdio>
#include <map>
#include <mutex>
#include <thread>

#include <fcntl.h>
#include <signal.h>
#include <sys/file.h>
#include <sys/prctl.h>
#include <unistd.h>

#include <cstdlib>

#include "core/log.h"
#include "core/subprocess.h"
#include "gpu/telemetry.h"

namespace bgc::gpu {

using json::Value;

namespace {

// Per-GPU sampler statistics over a burn.
struct BurnStats {
  double max_hot = 0, max_mem = 0, power_sum = 0, power_max = 0, clk_sum = 0;
  uint32_t clk_min = UINT32_MAX;
  int n = 0;
  Telemetry first, last;
  void add(const Telemetry& t) {
    if (!t.ok) return;
    if (n == 0) first = t;
    last = t;
    max_hot = std::max(max_hot, t.temp_hotspot_c);
    max_mem = std::max(max_mem, t.temp_mem_c);
    power_sum += t.power_w;
    power_max = std::max(power_max, t.power_w);
    clk_sum += t.gfxclk_mhz;
    clk_min = std::min(clk_min, t.gfxclk_mhz);
    ++n;
  }
  void fill(Value& out) const {
    out["samples"] = n;
    out["max_hotspot_c"] = max_hot;
    out["max_mem_c"] = max_mem;
    out["power_mean_w"] = n ? power_sum / n : 0.0;
    out["power_max_w"] = power_max;
    out["gfxclk_mean_mhz"] = n ? clk_sum / n : 0.0;
    out["gfxclk_min_mhz"] = n ? static_cast<double>(clk_min) : 0.0;
    Telemetry span = last;
    TelemetryPoller::violation_deltas(first, span);
    out["thermal_violation_pct"] = span.violation_thermal_pct < 0 ? Value() : Value(span.violation_thermal_pct);
    out["ppt_violation_pct"] = span.violation_ppt_pct < 0 ? Value() : Value(span.violation_ppt_pct);
  }
};

// Sleeps in short slices so a sampler notices `done` quickly.
void nap(const std::atomic<bool>& done, int ms) {
  for (int i = 0; i < ms / 10 && !done.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
}

void sleep_until(std::chrono::steady_clock::time_point t) {
  if (t > std::chrono::steady_clock::now()) std::this_thread::sleep_until(t);
}

// flock(2) on a file: PCIe sections of concurrent worker processes take turns.
class FileLock {
 public:
  explicit FileLock(const std::string& path) {
    if (path.empty()) return;
    fd_ = ::open(path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
    if (fd_ >= 0) {
      while (::flock(fd_, LOCK_EX) != 0 && errno == EINTR) {
      }
    }
  }
  ~FileLock() {
    if (fd_ >= 0) ::close(fd_);  // releases the lock
  }
  bool held() const { return fd_ >= 0; }
  FileLock(const FileLock&) = delete;
  FileLock& operator=(const FileLock&) = delete;

 private:
  int fd_ = -1;
};

class HipDiagEngine : public DiagEngine {
 public:
  explicit HipDiagEngine(std::string pcie_lock_path = "") : pcie_lock_path_(std::move(pcie_lock_path)) {}
  std::string name() const override { return "hip"; }
  Value checks(Backend& backend, const GpuInfo& g, int dev, const DiagPlan& plan, uint32_t seed) override {
    Diag& d = Diag::instance();
    (void)d.device_arch(dev);  // HIP up: when this happened tells the agent a worker's start-up time
    Value r = Value::object();
    r["ready_at_ns"] = static_cast<long long>(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count());
    Value timing = Value::object();  // wall ms per section, to see where a pass spends its time
    auto t = std::chrono::steady_clock::now();
    auto lap = [&](const char* name) {
      const auto now = std::chrono::steady_clock::now();
      timing[name] = std::chrono::duration<double, std::milli>(now - t).count();
      t = now;
    };
    r["hbm"] = d.hbm(dev, plan.hbm_bytes, 2, seed);
    lap("hbm");
    if (plan.hbm_walk_fraction > 0) {
      r["hbm_walk"] = d.hbm_walk(dev, plan.hbm_walk_fraction, plan.hbm_walk_chunk_bytes, plan.hbm_walk_budget_ms, seed);
      lap("hbm_walk");
    }
    r["mfma"] = d.mfma(dev, 16, 2048, seed);
    lap("mfma");
    if (plan.lowp) {
      r["lowp"] = d.mfma_lowp(dev, 32, 4096, seed);  // ~5 ms
      lap("lowp");
    }
    r["gemm"] = d.gemm_check(dev, 64, 64, 512, seed);
    lap("gemm");
    if (plan.pcie_bytes > 0) {
      // One GPU at a time: eight concurrent pinned-copy streams share the host's memory
      // bandwidth and root complexes, so concurrent rates would measure the host, not
      // the GPU's link.  ~50 ms per GPU.
      static std::mutex pcie_mu;
      std::lock_guard<std::mutex> lk(pcie_mu);
      FileLock across_processes(pcie_lock_path_);
      r["pcie"] = pcie_check(backend, g, dev, plan.pcie_bytes, seed);
      // false: the lock file could not be opened, so other GPUs' copies may have overlapped
      if (!pcie_lock_path_.empty()) r["pcie"]["serialized"] = across_processes.held();
      lap("pcie");
    }
    if (plan.soak_launches > 0) {
      r["soak"] = d.gemm_soak(dev, plan.soak_size, plan.soak_size, plan.soak_size, plan.soak_launches, seed);
      lap("soak");
    }
    r["timing_ms"] = timing;
    return r;
  }
  Value burn(int dev, int duration_ms, uint32_t seed, int dtype, std::chrono::steady_clock::time_point start_at) override {
    Diag& d = Diag::instance();
    (void)d.device_arch(dev);  // the HIP runtime and the device's context, before the wait
    const auto ready = std::chrono::steady_clock::now();
    sleep_until(start_at);
    Value r = d.burn(dev, duration_ms, 32, seed, dtype);
    r["ready_at_ns"] = static_cast<long long>(std::chrono::duration_cast<std::chrono::nanoseconds>(ready.time_since_epoch()).count());
    r["late_ms"] = ready > start_at ? std::chrono::duration<double, std::milli>(ready - start_at).count() : 0.0;
    return r;
  }

 private:
  std::string pcie_lock_path_;
};

std::string self_exe() {
  char buf[4096];
  const ssize_t n = ::readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  return n > 0 ? std::string(buf, static_cast<size_t>(n)) : std::string();
}

// Runs one worker request; the result JSON, or throws with the worker's error.
Value run_worker(const std::string& exe, const Value& request, int visible_device, int timeout_ms,
                 const CancelToken* cancel = nullptr) {
  std::vector<std::pair<std::string, std::string>> env{{"BGC_DIAG_REQUEST", request.dump()}};
  // Device numbering: `visible_device` is a ROCr index over ALL of the node's GPUs (the
  // "devices" enumeration below runs with nothing hidden, so its HIP order is ROCr's).
  // Visibility variables the agent itself may carry would renumber or hide devices in the
  // worker, so none is inherited; the worker then sees exactly its own GPU (HSA opens no
  // other device, so it leaves no footprint there) and checks its BDF against the request.
  std::vector<std::string> unset{"HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"};
  if (visible_device >= 0) env.emplace_back("ROCR_VISIBLE_DEVICES", std::to_string(visible_device));
  else unset.push_back("ROCR_VISIBLE_DEVICES");
  RunResult r = run_command({exe, "--diag-worker"}, env, timeout_ms, cancel, unset);
  if (r.cancelled) throw std::runtime_error("diagnostics worker stopped: the agent is shutting down");
  if (r.exit_code != 0) {
    throw std::runtime_error("diagnostics worker " +
                             (r.timed_out ? std::string("timed out") : "failed (exit " + std::to_string(r.exit_code) + ")") +
                             (r.err.empty() ? "" : ": " + r.err.substr(r.err.size() > 800 ? r.err.size() - 800 : 0)));
  }
  // the result is the last line (anything a library prints to stdout comes before it)
  std::string_view text(r.out);
  while (!text.empty() && (text.back() == '\n' || text.back() == '\r')) text.remove_suffix(1);
  const size_t nl = text.rfind('\n');
  if (nl != std::string_view::npos) text.remove_prefix(nl + 1);
  Value out;
  std::string perr;
  if (text.empty() || !json::try_parse(text, out, &perr)) {
    throw std::runtime_error("diagnostics worker printed no result: " + perr);
  }
  if (out.get("error").is_string()) throw std::runtime_error(out.get_string("error"));
  return out;
}

class ProcessDiagEngine : public DiagEngine {
 public:
  ProcessDiagEngine(std::string exe, std::string kind, std::string fixture, std::string lock, const CancelToken* cancel)
      : exe_(std::move(exe)), kind_(std::move(kind)), fixture_(std::move(fixture)), lock_(std::move(lock)),
        cancel_(cancel) {}
  std::string name() const override { return "hip"; }
  // A worker's HIP start-up on one visible GPU: 3 s before any worker has been measured,
  // then 1.5x the slowest recent start-up (concurrent start-ups on a full node are slower
  // than one alone), at least 1 s.  The checks workers measure it before the first burn.
  int start_lead_ms() const override {
    const int seen = slowest_ready_ms_.load();
    return seen <= 0 ? 3000 : std::max(1000, seen * 3 / 2 + 200);
  }
  Value checks(Backend&, const GpuInfo& g, int dev, const DiagPlan& plan, uint32_t seed) override {
    Value req = Value::object({{"op", "checks"}, {"backend", kind_}, {"fixture", fixture_}, {"gpu", to_json(g)},
                               {"plan", to_json(plan)}, {"seed", static_cast<unsigned long long>(seed)},
                               {"pcie_lock", lock_}});
    const auto t0 = std::chrono::steady_clock::now();
    // a healthy pass takes ~3 s (8 s with the VRAM clear of a reused GPU); the bound
    // covers the walk's budget, the PCIe copies waiting for the other GPUs' turns and a
    // slow HIP start, so a hung kernel costs the pass at most this long
    const int timeout_ms = std::max(60000, plan.hbm_walk_budget_ms + 90000);
    Value r = run_worker(exe_, req, dev, timeout_ms, cancel_);
    r["worker_ms"] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    note_ready(r, t0);  // so the start-up burn's lead is measured, not guessed
    return r;
  }
  Value burn(int dev, int duration_ms, uint32_t seed, int dtype, std::chrono::steady_clock::time_point start_at) override {
    const int64_t at = std::chrono::duration_cast<std::chrono::nanoseconds>(start_at.time_since_epoch()).count();
    Value req = Value::object({{"op", "burn"}, {"backend", kind_}, {"fixture", fixture_}, {"gpu_hip_device", dev},
                               {"duration_ms", duration_ms}, {"dtype", burn_dtype_name(dtype)},
                               {"seed", static_cast<unsigned long long>(seed)}, {"start_at_ns", static_cast<long long>(at)}});
    if (auto it = bdfs_.find(dev); it != bdfs_.end()) req["expect_bdf"] = it->second;
    const auto spawned = std::chrono::steady_clock::now();
    Value r = run_worker(exe_, req, dev, duration_ms + start_lead_ms() + 60000, cancel_);
    note_ready(r, spawned);
    return r;
  }

 private:
  // A worker's start-up (spawn to HIP ready) from its result's ready_at_ns: the slowest
  // recent one sets the burn lead.  A new maximum counts at once, an old one fades by a
  // quarter per worker, so one cold start does not lengthen every later pass.
  void note_ready(Value& r, std::chrono::steady_clock::time_point spawned) {
    if (!r.get("ready_at_ns").is_int()) return;
    const auto ready = std::chrono::steady_clock::time_point(std::chrono::nanoseconds(r.get("ready_at_ns").as_int()));
    const int ms = static_cast<int>(std::chrono::duration<double, std::milli>(ready - spawned).count());
    r["worker_ready_ms"] = ms;
    int prev = slowest_ready_ms_.load();
    while (!slowest_ready_ms_.compare_exchange_weak(prev, std::max(ms, prev * 3 / 4))) {
    }
  }

 public:

 private:
  void set_device_bdfs(std::map<int, std::string> bdfs) override { bdfs_ = std::move(bdfs); }

 private:
  std::string exe_, kind_, fixture_, lock_;
  std::map<int, std::string> bdfs_;  // ROCr device -> the BDF its worker must find
  const CancelToken* cancel_;
  std::atomic<int> slowest_ready_ms_{0};
};

// Re-reads the script from the backend on every call, so a test can change a running
// agent's diagnostics by rewriting the mock fixture.
class ScriptedDiagEngine : public DiagEngine {
 public:
  explicit ScriptedDiagEngine(Backend& backend) : backend_(backend) {}
  std::string name() const override { return "scripted"; }
  Value checks(Backend&, const GpuInfo& g, int dev, const DiagPlan& plan, uint32_t) override {
    const Value script = backend_.diag_script();
    const Value& e = script.get("gpus").get(std::to_string(g.index));
    std::this_thread::sleep_for(std::chrono::milliseconds(static_cast<int64_t>(num(e, "checks_ms", num(script, "checks_ms", 100)))));
    Value r = Value::object();
    r["hbm"] = Value::object({{"device", dev}, {"bytes", static_cast<unsigned long long>(plan.hbm_bytes)}, {"read_gbps", 6400.0},
                              {"write_gbps", 5200.0}, {"copy_gbps", 5400.0}, {"mismatches", 0}, {"passed", true}});
    if (plan.hbm_walk_fraction > 0) {
      const uint64_t free_b = g.vram_total_mb * (1ULL << 20);
      const uint64_t covered = static_cast<uint64_t>(static_cast<double>(free_b) * plan.hbm_walk_fraction);
      const uint64_t bad = static_cast<uint64_t>(num(e, "walk_mismatches", 0));
      r["hbm_walk"] = Value::object({{"device", dev}, {"free_bytes", static_cast<unsigned long long>(free_b)},
                                     {"bytes_covered", static_cast<unsigned long long>(covered)},
                                     {"coverage_of_free", plan.hbm_walk_fraction}, {"passes", 2},
                                     {"mismatches", static_cast<unsigned long long>(bad)}, {"passed", bad == 0}});
    }
    r["mfma"] = Value::object({{"device", dev}, {"tflops", 2000.0}, {"xcc_balance", 0.96}, {"xccs_seen", 8},
                               {"mismatches", 0}, {"bad_cus", 0}, {"throughput_ok", true}, {"passed", true}});
    if (plan.lowp) {
      r["lowp"] = Value::object({{"device", dev}, {"fp8_tflops", 4000.0}, {"fp4_tflops", 7000.0}, {"mismatches", 0},
                                 {"bad_cus", 0}, {"throughput_ok", true}, {"passed", true}});
    }
    r["gemm"] = Value::object({{"passed", true}});
    if (plan.soak_launches > 0) {
      r["soak"] = Value::object({{"tflops_mean", 1300.0}, {"row_mismatches", 0}, {"col_mismatches", 0}, {"passed", true}});
    }
    if (e.get("fail").is_string()) r["error"] = e.get_string("fail");
    return r;
  }
  Value burn(int dev, int duration_ms, uint32_t, int dtype, std::chrono::steady_clock::time_point start_at) override {
    sleep_until(start_at);
    std::this_thread::sleep_for(std::chrono::milliseconds(duration_ms));
    const Value script = backend_.diag_script();
    // the script's rate is a bf16 rate; an MX burn scales it like the hardware does
    const double tf = num(script.get("gpus").get(std::to_string(dev)), "burn_tflops", num(script, "burn_tflops", 2400)) *
                      burn_dtype_rate_ratio(dtype);
    return Value::object({{"dtype", burn_dtype_name(dtype)}, {"launches", std::max(1, duration_ms / 10)}, {"elapsed_ms", static_cast<double>(duration_ms)},
                          {"tflops_mean", tf}, {"tflops_min", tf}, {"tflops_first", tf}, {"tflops_last", tf},
                          {"tflops_max", tf}, {"sustain", 1.0}, {"mismatches", 0}});
  }

 private:
  static double num(const Value& v, const char* k, double d) { return v.get(k).is_number() ? v.get(k).as_double() : d; }
  Backend& backend_;
};

}  // namespace

std::unique_ptr<DiagEngine> make_hip_diag_engine() { return std::make_unique<HipDiagEngine>(); }

std::unique_ptr<DiagEngine> make_process_diag_engine(std::string exe, std::string backend_kind,
                                                     std::string mock_fixture_path, std::string pcie_lock_path,
                                                     const CancelToken* cancel) {
  if (exe.empty()) exe = self_exe();
  return std::make_unique<ProcessDiagEngine>(std::move(exe), std::move(backend_kind), std::move(mock_fixture_path),
                                             std::move(pcie_lock_path), cancel);
}

std::vector<std::string> worker_device_bdfs(const std::string& exe) {
  const Value r = run_worker(exe.empty() ? self_exe() : exe, Value::object({{"op", "devices"}}), -1, 120000);
  std::vector<std::string> out;
  for (const auto& b : r.get("bdfs").items()) out.push_back(b.as_string());
  return out;
}

Value to_json(const DiagPlan& p) {
  return Value::object({{"hbm_bytes", static_cast<unsigned long long>(p.hbm_bytes)},
                        {"hbm_walk_fraction", p.hbm_walk_fraction},
                        {"hbm_walk_chunk_bytes", static_cast<unsigned long long>(p.hbm_walk_chunk_bytes)},
                        {"hbm_walk_budget_ms", p.hbm_walk_budget_ms},
                        {"pcie_bytes", static_cast<unsigned long long>(p.pcie_bytes)},
                        {"soak_size", p.soak_size},
                        {"soak_launches", p.soak_launches},
                        {"lowp", p.lowp},
                        {"burn_ms", p.burn_ms},
                        {"burn_dtype", burn_dtype_name(p.burn_dtype)}});
}

DiagPlan diag_plan_from_json(const Value& v) {
  DiagPlan p;
  auto u64 = [&](const char* k, uint64_t d) { return v.get(k).is_int() ? v.get(k).as_uint() : d; };
  auto i32 = [&](const char* k, int d) { return v.get(k).is_int() ? static_cast<int>(v.get(k).as_int()) : d; };
  p.hbm_bytes = u64("hbm_bytes", p.hbm_bytes);
  p.hbm_walk_fraction = v.get("hbm_walk_fraction").is_number() ? v.get("hbm_walk_fraction").as_double() : p.hbm_walk_fraction;
  p.hbm_walk_chunk_bytes = u64("hbm_walk_chunk_bytes", p.hbm_walk_chunk_bytes);
  p.hbm_walk_budget_ms = i32("hbm_walk_budget_ms", p.hbm_walk_budget_ms);
  p.pcie_bytes = u64("pcie_bytes", p.pcie_bytes);
  p.soak_size = i32("soak_size", p.soak_size);
  p.soak_launches = i32("soak_launches", p.soak_launches);
  p.lowp = v.get("lowp").is_bool() ? v.get("lowp").as_bool() : p.lowp;
  p.burn_ms = i32("burn_ms", p.burn_ms);
  if (v.get("burn_dtype").is_string()) p.burn_dtype = burn_dtype_code(v.get_string("burn_dtype"));
  return p;
}

int diag_worker_main() {
  // The worker must not outlive the agent (a burn or a walk left running on a GPU the
  // restarted agent is about to diagnose): die with the thread that spawned it, which
  // waits for this process to finish.
  const pid_t parent = ::getppid();
  ::prctl(PR_SET_PDEATHSIG, SIGKILL);
  if (::getppid() != parent) return 1;  // the parent died before the line above
  Value out;
  try {
    const char* req_text = std::getenv("BGC_DIAG_REQUEST");
    if (!req_text) throw std::runtime_error("BGC_DIAG_REQUEST is not set");
    const Value req = json::parse(req_text);
    const std::string op = req.get_string("op");
    // the parent made this worker's GPU the only visible one (ROCR_VISIBLE_DEVICES)
    const int dev = std::getenv("ROCR_VISIBLE_DEVICES") || !req.get("hip_device").is_int()
                        ? 0
                        : static_cast<int>(req.get("hip_device").as_int());
    const uint32_t seed = static_cast<uint32_t>(req.get("seed").is_int() ? req.get("seed").as_uint() : 0x5eed);
    if (op == "devices") {
      Diag& d = Diag::instance();
      Value b = Value::array();
      for (int i = 0, n = d.device_count(); i < n; ++i) b.push_back(d.device_bdf(i));
      out = Value::object({{"bdfs", b}});
    } else if (op == "checks" || op == "burn") {
      auto backend = make_backend(req.get_string("backend", "amdsmi"), req.get_string("fixture"));
      // a mock backend with a diagnostics script (CPU tests of the worker plumbing)
      const bool scripted = backend->diag_script().is_object();
      // the one GPU this worker sees must be the one the agent means (a renumbered or
      // hidden device would put a burn or a verdict on another GPU, maybe a tenant's)
      const std::string expect = op == "checks" ? req.get("gpu").get_string("bdf") : req.get_string("expect_bdf");
      if (!scripted && !expect.empty()) {
        auto lower = [](std::string v) {
          for (auto& c : v) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
          return v;
        };
        Diag& d = Diag::instance();
        const std::string got = d.device_count() > 0 ? d.device_bdf(dev) : std::string("no device");
        if (lower(got) != lower(expect)) {
          throw std::runtime_error("diagnostics worker opened GPU " + got + " (ROCR_VISIBLE_DEVICES=" +
                                   (std::getenv("ROCR_VISIBLE_DEVICES") ? std::getenv("ROCR_VISIBLE_DEVICES") : "") +
                                   "), expected " + expect + ": not diagnosing another GPU");
        }
      }
      std::unique_ptr<DiagEngine> engine = scripted ? make_scripted_diag_engine(*backend)
                                                    : std::make_unique<HipDiagEngine>(req.get_string("pcie_lock"));
      // a script names GPUs by the agent's device number, not the worker's only device 0
      const int script_dev = scripted && req.get("gpu_hip_device").is_int()
                                 ? static_cast<int>(req.get("gpu_hip_device").as_int())
                                 : dev;
      if (op == "checks") {
        out = engine->checks(*backend, gpu_info_from_json(req.get("gpu")), dev, diag_plan_from_json(req.get("plan")), seed);
      } else {
        const auto at = std::chrono::steady_clock::time_point(std::chrono::nanoseconds(req.get("start_at_ns").as_int()));
        out = engine->burn(script_dev, static_cast<int>(req.get("duration_ms").as_int()), seed,
                           burn_dtype_code(req.get_string("dtype", "bf16")), at);
      }
    } else {
      throw std::runtime_error("unknown diagnostics worker op '" + op + "'");
    }
  } catch (const std::exception& e) {
    out = Value::object({{"error", std::string(e.what())}});
  }
  const std::string text = out.dump() + "\n";
  std::fwrite(text.data(), 1, text.size(), stdout);
  std::fflush(stdout);
  return 0;
}

std::unique_ptr<DiagEngine> make_scripted_diag_engine(Backend& backend) {
  return std::make_unique<ScriptedDiagEngine>(backend);
}

Value pcie_check(Backend& backend, const GpuInfo& g, int hip_device, uint64_t bytes, uint32_t seed) {
  const Telemetry before = backend.sample(g.index, SampleLevel::Slow);
  std::atomic<bool> done{false};
  int width = -1, speed = -1;  // highest seen while copying
  std::thread sampler([&] {
    while (!done.load()) {
      Telemetry t = backend.sample(g.index, SampleLevel::Slow);
      if (t.ok) {
        width = std::max(width, t.pcie_width);
        speed = std::max(speed, t.pcie_speed_mts);
      }
      for (int i = 0; i < 5 && !done.load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  });
  Value out;
  try {
    out = Diag::instance().pcie(hip_device, bytes, 5, seed);
  } catch (...) {
    done = true;
    sampler.join();
    throw;
  }
  done = true;
  sampler.join();
  const Telemetry after = backend.sample(g.index, SampleLevel::Slow);
  if (width > 0) out["link_width"] = width;
  if (speed > 0) out["link_speed_mts"] = speed;
  if (g.pcie_max_width > 0) out["max_width"] = g.pcie_max_width;
  if (g.pcie_max_speed_mts > 0) out["max_speed_mts"] = g.pcie_max_speed_mts;
  if (g.pcie_max_gen > 0) out["max_gen"] = g.pcie_max_gen;
  auto delta = [&](int64_t a, int64_t b) { return a >= 0 && b >= a ? Value(static_cast<long long>(b - a)) : Value(); };
  out["replays"] = delta(before.pcie_replays, after.pcie_replays);
  out["recoveries"] = delta(before.pcie_recoveries, after.pcie_recoveries);
  return out;
}

Value burn_in(Backend& backend, int index, int hip_device, int duration_ms, uint32_t seed, DiagEngine* engine,
              int dtype) {
  std::unique_ptr<DiagEngine> own;
  if (!engine) {
    own = make_hip_diag_engine();
    engine = own.get();
  }
  std::atomic<bool> done{false};
  BurnStats st;
  std::thread sampler([&] {
    while (!done.load()) {
      st.add(backend.sample(index, SampleLevel::Fast));
      nap(done, 100);
    }
  });
  Value out;
  try {
    out = engine->burn(hip_device, duration_ms, seed, dtype, std::chrono::steady_clock::time_point());
  } catch (...) {
    done = true;
    sampler.join();
    throw;
  }
  done = true;
  sampler.join();
  st.fill(out);
  return out;
}

NodeBurnResult node_burn(Backend& backend, DiagEngine& engine, const std::vector<GpuInfo>& gpus,
                         const std::vector<int>& hip_devs, const std::vector<size_t>& which, int duration_ms,
                         uint32_t seed, int dtype) {
  const size_t n = which.size();
  NodeBurnResult res;
  res.per_gpu.assign(n, Value());
  std::vector<BurnStats> st(n);
  std::vector<std::string> err(n);
  std::mutex mu;
  std::condition_variable cv;
  size_t ready = 0;
  bool go = false;
  std::atomic<bool> done{false};
  double sum_max = 0, sum_acc = 0, peak_hot = 0;
  int sweeps = 0;
  // Every GPU starts at the same instant: after the engine's start-up lead (a worker
  // process initialises HIP first), not when its thread happens to get there.
  const auto start_at = std::chrono::steady_clock::now() + std::chrono::milliseconds(engine.start_lead_ms());
  // One sampler for the whole node: each sweep reads every GPU under load, so the summed
  // power is the node's draw at one moment rather than a sum of separate peaks.
  std::thread sampler([&] {
    while (!done.load() && std::chrono::steady_clock::now() < start_at) nap(done, 20);
    while (!done.load()) {
      double sum = 0;
      int ok = 0;
      for (size_t k = 0; k < n; ++k) {
        const Telemetry t = backend.sample(gpus[which[k]].index, SampleLevel::Fast);
        if (!t.ok) continue;
        st[k].add(t);
        sum += t.power_w;
        peak_hot = std::max(peak_hot, t.temp_hotspot_c);
        ++ok;
      }
      if (ok) {
        sum_max = std::max(sum_max, sum);
        sum_acc += sum;
        ++sweeps;
      }
      nap(done, 100);
    }
  });
  std::vector<std::thread> workers;
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t k = 0; k < n; ++k) {
    workers.emplace_back([&, k] {
      {
        std::unique_lock<std::mutex> lk(mu);
        if (++ready == n) {
          go = true;
          cv.notify_all();
        }
        cv.wait(lk, [&] { return go; });
      }
      try {
        res.per_gpu[k] = engine.burn(hip_devs[which[k]], duration_ms, seed + static_cast<uint32_t>(which[k]), dtype, start_at);
      } catch (const std::exception& e) {
        err[k] = e.what();
      }
    });
  }
  for (auto& w : workers) w.join();
  const double wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  const double start_lead_ms = std::chrono::duration<double, std::milli>(start_at - t0).count();
  double late_max = 0;  // how long after the common start the slowest GPU began
  for (const auto& r : res.per_gpu) {
    if (r.get("late_ms").is_number()) late_max = std::max(late_max, r.get("late_ms").as_double());
  }
  done = true;
  sampler.join();
  Value per = Value::array();
  for (size_t k = 0; k < n; ++k) {
    if (!err[k].empty()) {
      res.per_gpu[k] = Value::object({{"error", err[k]}});
      continue;
    }
    st[k].fill(res.per_gpu[k]);
  }
  res.node = Value::object({{"gpus", static_cast<unsigned long long>(n)},
                            {"dtype", burn_dtype_name(dtype)},
                            {"duration_ms", duration_ms},
                            {"wall_ms", wall_ms},
                            {"start_lead_ms", start_lead_ms},
                            {"start_late_max_ms", late_max},
                            {"sweeps", sweeps},
                            {"power_sum_max_w", sum_max},
                            {"power_sum_mean_w", sweeps ? sum_acc / sweeps : 0.0},
                            {"peak_hotspot_c", peak_hot}});
  return res;
}

std::vector<std::vector<std::string>> judge_node_burn(NodeBurnResult& r, const DiagFloors& fl) {
  const size_t n = r.per_gpu.size();
  std::vector<std::vector<std::string>> per(n);
  std::vector<std::string> node_fail;
  double best = 0, worst = 0;
  bool any = false;
  for (const auto& b : r.per_gpu) {
    if (!b.get("tflops_mean").is_number()) continue;
    const double tf = b.get("tflops_mean").as_double();
    best = any ? std::max(best, tf) : tf;
    worst = any ? std::min(worst, tf) : tf;
    any = true;
  }
  const double balance = any && best > 0 ? worst / best : 0.0;
  r.node["tflops_best"] = best;
  r.node["tflops_worst"] = worst;
  r.node["balance"] = balance;
  char buf[200];
  if (fl.min_node_burn_balance > 0 && any && n > 1) {
    for (size_t k = 0; k < n; ++k) {
      const Value& b = r.per_gpu[k];
      if (!b.get("tflops_mean").is_number()) continue;
      const double frac = best > 0 ? b.get("tflops_mean").as_double() / best : 0.0;
      if (frac < fl.min_node_burn_balance) {
        std::snprintf(buf, sizeof(buf), "node burn-in: %.0f TF/s is %.2f of the node's fastest GPU under shared load (floor %.2f)",
                      b.get("tflops_mean").as_double(), frac, fl.min_node_burn_balance);
        per[k].push_back(buf);
      }
    }
  }
  const double psum = r.node.get("power_sum_max_w").is_number() ? r.node.get("power_sum_max_w").as_double() : 0.0;
  if (fl.max_node_power_w > 0 && psum > fl.max_node_power_w) {
    std::snprintf(buf, sizeof(buf), "node drew %.0f W with %zu GPUs under burn (limit %.0f W)", psum, n, fl.max_node_power_w);
    node_fail.push_back(buf);
  }
  const double hot = r.node.get("peak_hotspot_c").is_number() ? r.node.get("peak_hotspot_c").as_double() : 0.0;
  if (fl.max_burn_hotspot_c > 0 && hot > fl.max_burn_hotspot_c) {
    std::snprintf(buf, sizeof(buf), "node peak hotspot %.0f C under the node-level burn (limit %.0f C)", hot,
                  fl.max_burn_hotspot_c);
    node_fail.push_back(buf);
  }
  Value nf = Value::array();
  for (const auto& f : node_fail) {
    nf.push_back(f);
    for (auto& p : per) p.push_back(f);  // a node-wide limit: no GPU of the node is trusted
  }
  r.node["failures"] = nf;
  r.node["passed"] = node_fail.empty();
  return per;
}

std::vector<int> hip_devices_for(const std::vector<GpuInfo>& gpus, const std::vector<std::string>& hip_bdfs) {
  auto lower = [](std::string s) {
    for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    return s;
  };
  std::map<std::string, int> bdf_count, hip_by_bdf;
  for (const auto& g : gpus) bdf_count[lower(g.bdf)]++;
  for (size_t d = 0; d < hip_bdfs.size(); ++d) hip_by_bdf.emplace(lower(hip_bdfs[d]), static_cast<int>(d));
  std::vector<int> out;
  for (const auto& g : gpus) {
    const std::string b = lower(g.bdf);
    auto it = hip_by_bdf.find(b);
    // partitions share a BDF: only amdsmi's own enumeration can tell them apart
    if (!b.empty() && bdf_count[b] == 1 && it != hip_by_bdf.end()) out.push_back(it->second);
    else out.push_back(g.hip_id >= 0 ? g.hip_id : g.index);
  }
  return out;
}

}  // namespace bgc::gpu

// GPU bindings: amdsmi/mock discovery, the telemetry side thread, and the HIP
// diagnostic kernels (dlopen of libbgc_gpu_diag.so).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <memory>

#include "core/json.h"
#include "core/roctx.h"
#include "gpu/device.h"
#include "gpu/diag.h"
#include "gpu/node_agent.h"
#include "gpu/telemetry.h"

namespace py = pybind11;
using bgc::json::Value;

namespace bgc_py {

namespace {

struct PyBackend {
  std::unique_ptr<bgc::gpu::Backend> b;
};

struct PyPoller {
  std::shared_ptr<PyBackend> backend;  // keeps the backend alive
  std::unique_ptr<bgc::gpu::TelemetryPoller> poller;
};

std::string snapshot_json(const bgc::gpu::Snapshot& s) {
  Value v = Value::object();
  v["poll_seq"] = static_cast<unsigned long long>(s.poll_seq);
  v["poll_us"] = s.poll_us;
  Value devs = Value::array();
  for (auto& d : s.devices) devs.push_back(bgc::gpu::to_json(d));
  v["devices"] = devs;
  Value hs = Value::array();
  for (auto& h : s.health) {
    hs.push_back(Value::object({{"index", h.index}, {"healthy", h.healthy}, {"reason", h.reason}}));
  }
  v["health"] = hs;
  v["stalled"] = s.stalled;
  return v.dump();
}

bgc::gpu::HealthPolicy policy_from_json(const std::string& js) {
  bgc::gpu::HealthPolicy p;
  Value v = bgc::json::parse(js.empty() ? "{}" : js);
  auto d = [&](const char* k, double& dst) {
    if (v.get(k).is_number()) dst = v.get(k).as_double();
  };
  auto u = [&](const char* k, uint64_t& dst) {
    if (v.get(k).is_int()) dst = v.get(k).as_uint();
  };
  auto i = [&](const char* k, int& dst) {
    if (v.get(k).is_int()) dst = static_cast<int>(v.get(k).as_int());
  };
  d("max_hotspot_c", p.max_hotspot_c);
  d("max_mem_c", p.max_mem_c);
  u("max_new_uncorrectable", p.max_new_uncorrectable);
  u("max_uncorrectable_at_start", p.max_uncorrectable_at_start);
  if (v.get("require_all_xgmi_links").is_bool()) p.require_all_xgmi_links = v.get("require_all_xgmi_links").as_bool();
  u("max_retired_pages", p.max_retired_pages);
  d("max_thermal_violation_pct", p.max_thermal_violation_pct);
  d("max_ppt_violation_pct", p.max_ppt_violation_pct);
  i("violation_sustain_polls", p.violation_sustain_polls);
  i("fail_threshold", p.fail_threshold);
  i("recover_threshold", p.recover_threshold);
  if (v.get("require_full_pcie_width").is_bool()) p.require_full_pcie_width = v.get("require_full_pcie_width").as_bool();
  if (v.get("max_pcie_replays_per_poll").is_int()) p.max_pcie_replays_per_poll = v.get("max_pcie_replays_per_poll").as_int();
  return p;
}

}  // namespace

void register_gpu(py::module_& m) {
  py::class_<PyBackend, std::shared_ptr<PyBackend>>(m, "GpuBackend")
      .def_property_readonly("name", [](PyBackend& b) { return b.b->name(); })
      .def("discover", [](PyBackend& b) {
        Value arr = Value::array();
        {
          py::gil_scoped_release nogil;
          for (auto& g : b.b->discover()) arr.push_back(bgc::gpu::to_json(g));
        }
        return arr.dump();
      })
      .def("sample", [](PyBackend& b, int idx, int level) {
        bgc::gpu::Telemetry t;
        {
          py::gil_scoped_release nogil;
          t = b.b->sample(idx, static_cast<bgc::gpu::SampleLevel>(std::clamp(level, 0, 2)));
        }
        return bgc::gpu::to_json(t).dump();
      }, py::arg("index"), py::arg("level") = 2)
      .def("busy_processes", [](PyBackend& b, int idx) { return b.b->busy_processes(idx); });

  m.def("gpu_backend", [](const std::string& kind, const std::string& fixture_json) {
    auto pb = std::make_shared<PyBackend>();
    if (kind == "mock") {
      pb->b = bgc::gpu::make_mock_backend(fixture_json.empty() ? bgc::gpu::default_mi355x_fixture()
                                                               : bgc::json::parse(fixture_json));
    } else {
      pb->b = bgc::gpu::make_backend(kind, "");
    }
    return pb;
  }, py::arg("kind") = "auto", py::arg("fixture_json") = "");

  m.def("default_mi355x_fixture",
        [](int n, uint64_t hive_id) { return bgc::gpu::default_mi355x_fixture(n, hive_id).dump(); }, py::arg("n") = 8,
        py::arg("hive_id") = 0x1a2b3c4d5e6f7788ULL);

  py::class_<PyPoller>(m, "TelemetryPoller")
      .def(py::init([](std::shared_ptr<PyBackend> b, std::vector<int> idx, int interval_ms, const std::string& policy,
                       int slow_every, int ras_every, std::vector<uint64_t> page_limits, int stall_ms) {
             auto p = std::make_unique<PyPoller>();
             p->backend = b;
             p->poller = std::make_unique<bgc::gpu::TelemetryPoller>(
                 *b->b, idx, std::chrono::milliseconds(interval_ms), policy_from_json(policy), slow_every, ras_every,
                 std::move(page_limits));
             p->poller->set_stall_timeout(std::chrono::milliseconds(stall_ms));
             return p;
           }),
           py::arg("backend"), py::arg("indices"), py::arg("interval_ms") = 1000, py::arg("policy") = "{}",
           py::arg("slow_every") = 10, py::arg("ras_every") = 60, py::arg("page_limits") = std::vector<uint64_t>{},
           py::arg("stall_ms") = 0)
      .def("stalled", [](PyPoller& p) { return p.poller->stalled(); })
      .def("start", [](PyPoller& p) { p.poller->start(); })
      .def("stop", [](PyPoller& p) {
        py::gil_scoped_release nogil;
        p.poller->stop();
      })
      .def("poll_once", [](PyPoller& p) {
        py::gil_scoped_release nogil;
        p.poller->poll_once();
      })
      .def("polls", [](PyPoller& p) { return p.poller->polls(); })
      .def("snapshot", [](PyPoller& p) { return snapshot_json(*p.poller->snapshot()); });

  m.def("health_step", [](const std::string& telemetry_json, int fail_threshold, int recover_threshold,
                          const std::string& policy, uint64_t page_limit) {
    // Runs the health state machine over a sequence of telemetry samples (violation
    // percentages are derived from accumulators when a sample carries acc_counter);
    // returns (healthy, reason) after each step.
    bgc::gpu::HealthPolicy pol = policy_from_json(policy);
    pol.fail_threshold = fail_threshold;
    pol.recover_threshold = recover_threshold;
    bgc::gpu::DeviceHealth h;
    h.page_limit = page_limit ? std::min<uint64_t>(page_limit, pol.max_retired_pages) : pol.max_retired_pages;
    const Value pol_json = bgc::json::parse(policy.empty() ? "{}" : policy);
    if (pol_json.get("pcie_max_width").is_int()) {
      h.pcie_max_width = static_cast<int>(pol_json.get("pcie_max_width").as_int());  // capability (discovery)
    }
    bgc::gpu::Telemetry prev;
    std::vector<py::tuple> out;
    Value seq = bgc::json::parse(telemetry_json);
    for (const auto& tv : seq.items()) {
      bgc::gpu::Telemetry t = bgc::gpu::telemetry_from_json(tv);
      if (t.acc_counter != bgc::gpu::Telemetry::kNoAcc) {
        bgc::gpu::TelemetryPoller::violation_deltas(prev, t);
        prev = t;
      }
      bgc::gpu::TelemetryPoller::evaluate(t, pol, h);
      out.push_back(py::make_tuple(h.healthy, h.reason));
    }
    return out;
  }, py::arg("telemetry_json"), py::arg("fail_threshold") = 3, py::arg("recover_threshold") = 3,
     py::arg("policy") = "{}", py::arg("page_limit") = 0);

  // --- HIP diagnostics ---
  m.def("diag_library_path", [](const std::string& p) { return bgc::gpu::Diag::instance(p).path(); },
        py::arg("explicit_path") = "");
  m.def("diag_device_count", [] { return bgc::gpu::Diag::instance().device_count(); });
  m.def("diag_device_arch", [](int d) { return bgc::gpu::Diag::instance().device_arch(d); });
  m.def("diag_hbm", [](int device, unsigned long long bytes, int iters, unsigned seed) {
    Value v;
    {
      py::gil_scoped_release nogil;
      v = bgc::gpu::Diag::instance().hbm(device, bytes, iters, seed);
    }
    return v.dump();
  }, py::arg("device"), py::arg("bytes") = 2ULL << 30, py::arg("iters") = 3, py::arg("seed") = 0x5eed);
  m.def("diag_mfma", [](int device, int waves_per_cu, int iters, unsigned seed) {
    Value v;
    {
      py::gil_scoped_release nogil;
      v = bgc::gpu::Diag::instance().mfma(device, waves_per_cu, iters, seed);
    }
    return v.dump();
  }, py::arg("device"), py::arg("waves_per_cu") = 32, py::arg("iters") = 4096, py::arg("seed") = 0x5eed);
  m.def("diag_mfma_lowp", [](int device, int waves_per_cu, int iters, unsigned seed) {
    Value v;
    {
      py::gil_scoped_release nogil;
      v = bgc::gpu::Diag::instance().mfma_lowp(device, waves_per_cu, iters, seed);
    }
    return v.dump();
  }, py::arg("device"), py::arg("waves_per_cu") = 32, py::arg("iters") = 4096, py::arg("seed") = 0x5eed);
  m.def("diag_gemm", [](int device, int mm, int nn, int kk, const std::string& a, const std::string& b) {
    if (a.size() != static_cast<size_t>(mm) * kk * 2 || b.size() != static_cast<size_t>(kk) * nn * 2) {
      throw std::invalid_argument("A must be M*K and B K*N bf16 values");
    }
    std::string c(static_cast<size_t>(mm) * nn * 4, '\0');
    {
      py::gil_scoped_release nogil;
      bgc::gpu::Diag::instance().gemm(device, mm, nn, kk, reinterpret_cast<const uint16_t*>(a.data()),
                                      reinterpret_cast<const uint16_t*>(b.data()), reinterpret_cast<float*>(c.data()));
    }
    return py::bytes(c);
  }, py::arg("device"), py::arg("m"), py::arg("n"), py::arg("k"), py::arg("a_bf16"), py::arg("b_bf16"));
  m.def("diag_gemm_tiled", [](int device, int mm, int nn, int kk, const std::string& a, const std::string& bt) {
    if (a.size() != static_cast<size_t>(mm) * kk * 2 || bt.size() != static_cast<size_t>(nn) * kk * 2) {
      throw std::invalid_argument("A must be M*K and Bt N*K bf16 values");
    }
    std::string c(static_cast<size_t>(mm) * nn * 4, '\0');
    {
      py::gil_scoped_release nogil;
      bgc::gpu::Diag::instance().gemm_tiled(device, mm, nn, kk, reinterpret_cast<const uint16_t*>(a.data()),
                                            reinterpret_cast<const uint16_t*>(bt.data()), reinterpret_cast<float*>(c.data()));
    }
    return py::bytes(c);
  }, py::arg("device"), py::arg("m"), py::arg("n"), py::arg("k"), py::arg("a_bf16"), py::arg("bt_bf16"));
  m.def("diag_mx_gemm", [](int device, int fmt, int mm, int nn, int kk, const std::string& a, const std::string& sa,
                           const std::string& bt, const std::string& sb) {
    const size_t per = fmt == 0 ? static_cast<size_t>(kk) : static_cast<size_t>(kk) / 2;
    if ((fmt != 0 && fmt != 4) || kk % 128 || a.size() != static_cast<size_t>(mm) * per ||
        bt.size() != static_cast<size_t>(nn) * per || sa.size() != static_cast<size_t>(mm) * (kk / 32) ||
        sb.size() != static_cast<size_t>(nn) * (kk / 32)) {
      throw std::invalid_argument("fmt 0: A M*K, Bt N*K bytes; fmt 4: M*K/2, N*K/2; scales M*K/32 and N*K/32 bytes");
    }
    std::string c(static_cast<size_t>(mm) * nn * 4, '\0');
    {
      py::gil_scoped_release nogil;
      auto u8 = [](const std::string& x) { return reinterpret_cast<const uint8_t*>(x.data()); };
      bgc::gpu::Diag::instance().mx_gemm(device, fmt, mm, nn, kk, u8(a), u8(sa), u8(bt), u8(sb),
                                         reinterpret_cast<float*>(c.data()));
    }
    return py::bytes(c);
  }, py::arg("device"), py::arg("fmt"), py::arg("m"), py::arg("n"), py::arg("k"), py::arg("a"), py::arg("a_scales"),
     py::arg("bt"), py::arg("bt_scales"));
  m.def("diag_hbm_walk", [](int device, double fraction, unsigned long long chunk_bytes, int budget_ms, unsigned seed) {
    Value v;
    {
      py::gil_scoped_release nogil;
      v = bgc::gpu::Diag::instance().hbm_walk(device, fraction, chunk_bytes, budget_ms, seed);
    }
    return v.dump();
  }, py::arg("device"), py::arg("fraction") = 0.9, py::arg("chunk_bytes") = 4ULL << 30, py::arg("budget_ms") = 20000,
     py::arg("seed") = 0x5eed);
  m.def("diag_device_bdf", [](int d) { return bgc::gpu::Diag::instance().device_bdf(d); });
  m.def("diag_gemm_check", [](int device, int mm, int nn, int kk, unsigned seed) {
    Value v;
    {
      py::gil_scoped_release nogil;
      v = bgc::gpu::Diag::instance().gemm_check(device, mm, nn, kk, seed);
    }
    return v.dump();
  }, py::arg("device"), py::arg("m") = 64, py::arg("n") = 64, py::arg("k") = 512, py::arg("seed") = 0x5eed);
  m.def("diag_burn", [](std::shared_ptr<PyBackend> b, int index, int hip_device, int duration_ms, unsigned seed,
                        const std::string& dtype) {
    const int code = bgc::gpu::burn_dtype_code(dtype);
    Value v;
    {
      py::gil_scoped_release nogil;
      v = bgc::gpu::burn_in(*b->b, index, hip_device, duration_ms, seed, nullptr, code);
    }
    return v.dump();
  }, py::arg("backend"), py::arg("index"), py::arg("hip_device"), py::arg("duration_ms"), py::arg("seed") = 0x5eed,
     py::arg("dtype") = "bf16");
  m.def("diag_pcie", [](int device, unsigned long long bytes, int iters, unsigned seed) {
    Value v;
    {
      py::gil_scoped_release nogil;
      v = bgc::gpu::Diag::instance().pcie(device, bytes, iters, seed);
    }
    return v.dump();
  }, py::arg("device"), py::arg("bytes") = 256ULL << 20, py::arg("iters") = 5, py::arg("seed") = 0x5eed);
  m.def("diag_gemm_soak", [](int device, int mm, int nn, int kk, int launches, unsigned seed) {
    Value v;
    {
      py::gil_scoped_release nogil;
      v = bgc::gpu::Diag::instance().gemm_soak(device, mm, nn, kk, launches, seed);
    }
    return v.dump();
  }, py::arg("device"), py::arg("m") = 8192, py::arg("n") = 8192, py::arg("k") = 8192, py::arg("launches") = 10,
     py::arg("seed") = 0x5eed);
  m.def("pcie_check", [](std::shared_ptr<PyBackend> b, int index, int hip_device, unsigned long long bytes, unsigned seed) {
    Value v;
    {
      py::gil_scoped_release nogil;
      auto gpus = b->b->discover();
      if (index < 0 || static_cast<size_t>(index) >= gpus.size()) throw std::out_of_range("no such GPU");
      v = bgc::gpu::pcie_check(*b->b, gpus[static_cast<size_t>(index)], hip_device, bytes, seed);
    }
    return v.dump();
  }, py::arg("backend"), py::arg("index"), py::arg("hip_device"), py::arg("bytes") = 256ULL << 20, py::arg("seed") = 0x5eed);
  m.def("judge_diag", [](const std::string& result, const std::string& floors_json) {
    bgc::gpu::DiagFloors f = bgc::gpu::DiagFloors::mi355x_defaults();
    Value fj = bgc::json::parse(floors_json);
    auto num = [&](const char* k, double& dst) {
      if (fj.get(k).is_number()) dst = fj.get(k).as_double();
    };
    num("min_read_gbps", f.min_read_gbps);
    num("min_copy_gbps", f.min_copy_gbps);
    num("min_write_gbps", f.min_write_gbps);
    num("min_mfma_tflops", f.min_mfma_tflops);
    num("min_xcc_balance", f.min_xcc_balance);
    num("min_fp8_tflops", f.min_fp8_tflops);
    num("min_fp4_tflops", f.min_fp4_tflops);
    num("min_burn_tflops", f.min_burn_tflops);
    num("min_burn_sustain", f.min_burn_sustain);
    num("max_burn_hotspot_c", f.max_burn_hotspot_c);
    num("max_burn_thermal_violation_pct", f.max_burn_thermal_violation_pct);
    num("min_pcie_h2d_gbps", f.min_pcie_h2d_gbps);
    num("min_pcie_d2h_gbps", f.min_pcie_d2h_gbps);
    num("min_pcie_speed_fraction", f.min_pcie_speed_fraction);
    num("min_soak_tflops", f.min_soak_tflops);
    num("min_hbm_walk_coverage", f.min_hbm_walk_coverage);
    num("min_node_burn_balance", f.min_node_burn_balance);
    num("max_node_power_w", f.max_node_power_w);
    if (fj.get("require_full_pcie_width").is_bool()) f.require_full_pcie_width = fj.get("require_full_pcie_width").as_bool();
    if (fj.get("min_xccs").is_int()) f.min_xccs = static_cast<int>(fj.get("min_xccs").as_int());
    return bgc::gpu::judge_diag(bgc::json::parse(result), f).dump();
  }, py::arg("result"), py::arg("floors") = "{}");
  m.def("roctx_available", &bgc::roctx::available);

  // Node agent rendering (pure functions).
  m.def("node_patches", [](const std::string& gpus_json, int healthy, const std::string& node, bool diag_ran,
                           bool diag_passed, const std::string& reason) {
    bgc::gpu::NodeAgentConfig cfg;
    cfg.node_name = node;
    std::vector<bgc::gpu::GpuInfo> gpus;
    bgc::json::Value parsed = bgc::json::parse(gpus_json);
    for (const auto& g : parsed.items()) gpus.push_back(bgc::gpu::gpu_info_from_json(g));
    bgc::gpu::DiagOutcome d;
    d.ran = diag_ran;
    d.passed = diag_passed;
    return py::make_tuple(bgc::gpu::node_labels_patch(cfg, gpus, healthy, d).dump(),
                          bgc::gpu::node_status_patch(cfg, gpus, healthy, reason).dump());
  }, py::arg("gpus_json"), py::arg("healthy"), py::arg("node") = "node-0", py::arg("diag_ran") = false,
     py::arg("diag_passed") = true, py::arg("reason") = "");
  m.def("sanitize_label_value", &bgc::gpu::sanitize_label_value);
}

}  // namespace bgc_py

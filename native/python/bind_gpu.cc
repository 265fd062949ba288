// GPU bindings: amdsmi/mock discovery, the telemetry side thread, and the HIP
// diagnostic kernels (dlopen of libbgc_gpu_diag.so).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

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
  return v.dump();
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
      .def("sample", [](PyBackend& b, int idx, bool full) {
        bgc::gpu::Telemetry t;
        {
          py::gil_scoped_release nogil;
          t = b.b->sample(idx, full);
        }
        return bgc::gpu::to_json(t).dump();
      }, py::arg("index"), py::arg("full") = true);

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
      .def(py::init([](std::shared_ptr<PyBackend> b, std::vector<int> idx, int interval_ms) {
             auto p = std::make_unique<PyPoller>();
             p->backend = b;
             p->poller = std::make_unique<bgc::gpu::TelemetryPoller>(*b->b, idx, std::chrono::milliseconds(interval_ms));
             return p;
           }),
           py::arg("backend"), py::arg("indices"), py::arg("interval_ms") = 1000)
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
                          std::vector<py::dict> history) {
    // Runs the health state machine over a sequence of telemetry samples; returns the
    // (healthy, reason) after each step.
    bgc::gpu::HealthPolicy pol;
    pol.fail_threshold = fail_threshold;
    pol.recover_threshold = recover_threshold;
    bgc::gpu::DeviceHealth h;
    std::vector<py::tuple> out;
    Value seq = bgc::json::parse(telemetry_json);
    for (const auto& tv : seq.items()) {
      bgc::gpu::Telemetry t;
      t.ok = tv.get("ok").is_bool() ? tv.get("ok").as_bool() : true;
      t.error = tv.get_string("error");
      t.temp_hotspot_c = tv.get("temp_hotspot_c").is_number() ? tv.get("temp_hotspot_c").as_double() : 40;
      t.temp_mem_c = tv.get("temp_mem_c").is_number() ? tv.get("temp_mem_c").as_double() : 40;
      t.ecc_uncorrectable = tv.get("ecc_uncorrectable").is_int() ? tv.get("ecc_uncorrectable").as_uint() : 0;
      t.xgmi_links_up = tv.get("xgmi_links_up").is_int() ? static_cast<int>(tv.get("xgmi_links_up").as_int()) : -1;
      t.xgmi_links_total = tv.get("xgmi_links_total").is_int() ? static_cast<int>(tv.get("xgmi_links_total").as_int()) : -1;
      bgc::gpu::TelemetryPoller::evaluate(t, pol, h);
      out.push_back(py::make_tuple(h.healthy, h.reason));
    }
    (void)history;
    return out;
  }, py::arg("telemetry_json"), py::arg("fail_threshold") = 3, py::arg("recover_threshold") = 3,
     py::arg("history") = std::vector<py::dict>{});

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

// Kube-side bindings: native churn driver (bench), in-process kube-lite, workqueue.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>

#include "apiserver/server.h"
#include "bench/churn.h"
#include "controller/reconcile.h"
#include "kube/events.h"
#include "kube/quantity.h"
#include "kube/ratelimit.h"
#include "kube/runtime.h"

namespace py = pybind11;

namespace bgc_py {

void register_kube(py::module_& m) {
  // The reconciler's pure planning step (controller/reconcile.h): [(plural, ns, name, body)]
  m.def("desired_children", [](const std::string& ub_json, bool label) {
    std::vector<std::tuple<std::string, std::string, std::string, std::string>> out;
    for (auto& c : bgc::controller::desired_children(bgc::json::parse(ub_json), label))
      out.emplace_back(c.rt->plural, c.ns, c.name, std::move(c.body));
    return out;
  }, py::arg("ub_json"), py::arg("label") = false);
  // Kubernetes quantity value (kube/quantity.h): float, or None when not a quantity
  m.def("quantity_value", [](const std::string& s) -> py::object {
    auto v = bgc::kube::parse_quantity(s);
    return v ? py::object(py::float_(static_cast<double>(*v))) : py::none();
  });
  m.def("same_quantity", [](const std::string& a, const std::string& b) { return bgc::kube::same_quantity(a, b); });
  m.def("canonical_quantity", [](const std::string& s) -> py::object {
    auto c = bgc::kube::canonical_quantity(s);
    return c ? py::object(py::str(*c)) : py::object(py::none());
  });
  py::class_<bgc::bench::ChurnDriver>(m, "ChurnDriver")
      .def(py::init([](const std::string& server, const std::string& token, const std::string& prefix,
                       int concurrency, const std::string& gpu_key, const std::string& group,
                       const std::string& ca_pem, const std::string& approve_url, bool http2,
                       bool server_filter) {
             bgc::bench::ChurnOptions o;
             o.server = server;
             o.admin_token = token;
             o.ca_pem = ca_pem;
             o.name_prefix = prefix;
             o.concurrency = concurrency;
             o.gpu_quota_key = gpu_key;
             o.group = group;
             o.approve_url = approve_url;
             o.http2 = http2;
             o.server_filter = server_filter;
             return std::make_unique<bgc::bench::ChurnDriver>(o);
           }),
           py::arg("server"), py::arg("admin_token"), py::arg("name_prefix"), py::arg("concurrency") = 32,
           py::arg("gpu_quota_key") = "requests.amd.com/gpu", py::arg("group") = "gpu", py::arg("ca_pem") = "",
           py::arg("approve_url") = "", py::arg("http2") = false,
           py::arg("server_filter") = false)
      .def("start", &bgc::bench::ChurnDriver::start)
      .def("step", [](bgc::bench::ChurnDriver& d, const std::vector<std::string>& names, double timeout) {
        bgc::json::Value v;
        {
          py::gil_scoped_release nogil;
          v = d.step(names, timeout);
        }
        return v.dump();
      })
      .def("step_with_delete", [](bgc::bench::ChurnDriver& d, const std::vector<std::string>& names,
                                  const std::vector<std::string>& prev, double timeout) {
        bgc::json::Value v;
        {
          py::gil_scoped_release nogil;
          v = d.step_with_delete(names, prev, timeout);
        }
        return v.dump();
      })
      .def("open_loop", [](bgc::bench::ChurnDriver& d, const std::vector<std::string>& names, double duration_s,
                           double timeout, uint64_t seed) {
        bgc::json::Value v;
        {
          py::gil_scoped_release nogil;
          v = d.open_loop(names, duration_s, timeout, seed);
        }
        return v.dump();
      }, py::arg("names"), py::arg("duration_s"), py::arg("timeout") = 60.0, py::arg("seed") = 1)
      .def("remove", [](bgc::bench::ChurnDriver& d, const std::vector<std::string>& names) {
        py::gil_scoped_release nogil;
        return d.remove(names);
      })
      .def("stop", [](bgc::bench::ChurnDriver& d) {
        py::gil_scoped_release nogil;
        d.stop();
      });

  // WorkQueue (unit tests of dedup / delay / exclusivity semantics)
  py::class_<bgc::kube::RetryLimiter>(m, "RetryLimiter")
      .def(py::init([](int64_t base_ms, int64_t cap_ms, double qps, int burst) {
             return std::make_unique<bgc::kube::RetryLimiter>(std::chrono::milliseconds(base_ms),
                                                              std::chrono::milliseconds(cap_ms), qps, burst);
           }),
           py::arg("base_ms") = 5, py::arg("cap_ms") = 60000, py::arg("qps") = 10.0, py::arg("burst") = 100)
      .def("when", [](bgc::kube::RetryLimiter& r, const std::string& k) { return r.when(k).count(); })
      .def("forget", &bgc::kube::RetryLimiter::forget)
      .def("failures", &bgc::kube::RetryLimiter::failures);
  // Event recorder's per-object token bucket; `at_s` is a synthetic clock in seconds
  py::class_<bgc::kube::EventRateLimiter>(m, "EventRateLimiter")
      .def(py::init<double, double, size_t>(), py::arg("burst") = 10.0, py::arg("refill_per_minute") = 6.0,
           py::arg("max_keys") = 4096)
      .def("allow", [](bgc::kube::EventRateLimiter& l, const std::string& key, double at_s) {
        return l.allow(key, std::chrono::steady_clock::time_point(
                                std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                    std::chrono::duration<double>(at_s))));
      })
      .def("size", &bgc::kube::EventRateLimiter::size);
  py::class_<bgc::kube::WorkQueue>(m, "WorkQueue")
      .def(py::init<size_t>(), py::arg("shards") = 1)
      .def("shards", &bgc::kube::WorkQueue::shards)
      .def_static("shards_for", &bgc::kube::WorkQueue::shards_for)
      .def("add", [](bgc::kube::WorkQueue& q, const std::string& k) { q.add(k); })
      .def("add_after", [](bgc::kube::WorkQueue& q, const std::string& k, int ms) { q.add_after(k, std::chrono::milliseconds(ms)); })
      .def("get", [](bgc::kube::WorkQueue& q, size_t worker) {
        std::string k;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = q.get(k, worker);
        }
        return ok ? py::object(py::str(k)) : py::object(py::none());
      }, py::arg("worker") = 0)
      .def("done", &bgc::kube::WorkQueue::done)
      .def("forget", &bgc::kube::WorkQueue::forget)
      .def("requeue", [](bgc::kube::WorkQueue& q, const std::string& k, int ms) { q.requeue(k, std::chrono::milliseconds(ms)); })
      .def("shutdown", &bgc::kube::WorkQueue::shutdown)
      .def("pending", &bgc::kube::WorkQueue::pending)
      .def("in_flight", &bgc::kube::WorkQueue::in_flight);
}

}  // namespace bgc_py

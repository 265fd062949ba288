// Admission policy bindings (unit-test surface for SURVEY §3.2's decision table).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "admission/policy.h"

namespace py = pybind11;

namespace bgc_py {

void register_admission(py::module_& m) {
  using bgc::admission::Config;
  py::class_<Config>(m, "AdmissionConfig")
      .def(py::init<>())
      .def_readwrite("oidc_username_prefix", &Config::oidc_username_prefix)
      .def_readwrite("default_role_name", &Config::default_role_name)
      .def_readwrite("authorized_group_names", &Config::authorized_group_names)
      .def_readwrite("log_full_request", &Config::log_full_request);

  m.def("classify_username", [](const std::string& u, const std::string& prefix) {
    auto n = bgc::admission::Username::classify(u, prefix);
    return py::make_tuple(n.original_username, n.kube_username,
                          n.kind == bgc::admission::UserKind::Normal ? "normal" : "admin");
  });

  // Returns (allowed, invalid, message, patch_json_or_None, rule)
  m.def("admission_mutate", [](const std::string& request_json, const Config& cfg) {
    auto d = bgc::admission::mutate(bgc::json::parse(request_json), cfg);
    py::object patch = d.patch.empty() ? py::object(py::none()) : py::object(py::str(d.patch));
    return py::make_tuple(d.allowed, d.invalid, d.message, patch, d.rule);
  });

  // Full HTTP handling of a /mutate body: (status, body, content_type)
  m.def("admission_handle_review", [](const std::string& body, const std::string& content_type, const Config& cfg) {
    auto r = bgc::admission::handle_review(body, content_type, cfg);
    return py::make_tuple(r.status, r.body, r.content_type);
  });
}

}  // namespace bgc_py

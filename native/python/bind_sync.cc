// Synchronizer bindings: sheet parsing, header inference, quota mapping, JWT assertion.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "core/json.h"
#include "core/unicode.h"
#include "sync/google.h"
#include "sync/sheet.h"

namespace py = pybind11;

namespace bgc_py {

namespace {

py::dict row_to_dict(const bgc::sync::Row& r) {
  py::dict d;
  d["name"] = r.name;
  d["department"] = r.department;
  d["id_username"] = r.id_username;
  d["gpu_server"] = r.gpu_server;
  d["gpu_request"] = r.gpu_request;
  d["cpu_request"] = r.cpu_request;
  d["memory_request"] = r.memory_request;
  d["storage_request"] = r.storage_request;
  d["mig_request"] = r.mig_request;
  d["authorized"] = r.authorized;
  return d;
}

bgc::sync::Row dict_to_row(const py::dict& d) {
  bgc::sync::Row r;
  auto s = [&](const char* k) { return d.contains(k) ? d[k].cast<std::string>() : std::string(); };
  auto n = [&](const char* k) { return d.contains(k) ? d[k].cast<int64_t>() : 0; };
  r.name = s("name");
  r.department = s("department");
  r.id_username = s("id_username");
  r.gpu_server = s("gpu_server");
  r.gpu_request = n("gpu_request");
  r.cpu_request = n("cpu_request");
  r.memory_request = n("memory_request");
  r.storage_request = n("storage_request");
  r.mig_request = n("mig_request");
  r.authorized = s("authorized");
  return r;
}

}  // namespace

void register_sync(py::module_& m) {
  py::register_exception<bgc::sync::CsvHeaderError>(m, "CsvHeaderError", PyExc_ValueError);
  py::register_exception<bgc::sync::CsvParseError>(m, "CsvParseError", PyExc_ValueError);

  m.def("infer_header", &bgc::sync::infer_header);
  m.def("csv_records", &bgc::sync::parse_records);
  m.def("parse_sheet", [](const std::string& csv) {
    std::vector<std::string> warnings;
    auto rows = bgc::sync::parse_csv(csv, &warnings);
    py::list out;
    for (auto& r : rows) out.append(row_to_dict(r));
    return py::make_tuple(out, warnings);
  });
  m.def("is_authorized", [](const std::string& a) {
    bgc::sync::Row r;
    r.authorized = a;
    return bgc::sync::is_authorized(r);
  });
  // Rust str::trim / str::to_lowercase slices (core/unicode.h), on UTF-8 bytes
  m.def("unicode_trim", [](const py::bytes& b) { return py::bytes(std::string(bgc::unicode::trim(std::string(b)))); });
  m.def("unicode_lower", [](const py::bytes& b) { return py::bytes(bgc::unicode::to_lower(std::string(b))); });
  m.def("quota_spec", [](const py::dict& row, const std::string& gpu, const std::string& part) {
    bgc::sync::QuotaKeys k;
    k.gpu_resource = gpu;
    k.partition_resource = part;
    return bgc::sync::quota_spec(dict_to_row(row), k).dump();
  }, py::arg("row"), py::arg("gpu_resource") = "amd.com/gpu", py::arg("partition_resource") = "amd.com/gpu-partition");
  m.def("lookup_row", [](const std::string& csv, const std::string& server, const std::string& user) -> py::object {
    auto rows = bgc::sync::parse_csv(csv, nullptr);
    bgc::sync::RowIndex idx(rows, server);
    const bgc::sync::Row* r = idx.find(user);
    if (!r) return py::none();
    return row_to_dict(*r);
  });
  m.def("google_assertion", [](const std::string& key_json, const std::string& scope, int64_t now) {
    auto key = bgc::sync::ServiceAccountKey::from_json(bgc::json::parse(key_json));
    bgc::sync::GoogleAuth auth(key, scope);
    return auth.make_assertion(now);
  });
  m.def("valid_utf8", [](py::bytes b) { return bgc::sync::valid_utf8(std::string(b)); });
}

}  // namespace bgc_py

// pybind11 surface of the native core: used by the pytest suite (unit tests of every
// C++ component) and by the bench harness (native churn driver).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>

#include "core/crypto.h"
#include "core/env_config.h"
#include "core/json.h"
#include "core/json_patch.h"
#include "core/yaml.h"
#include "crd/schema.h"
#include "core/log.h"
#include "core/metrics.h"
#include "core/process.h"
#include "core/stall.h"
#include "core/trace.h"
#include "kube/client.h"

namespace py = pybind11;
using bgc::json::Value;

namespace bgc_py {
void register_admission(py::module_& m);
void register_sync(py::module_& m);
void register_kube(py::module_& m);
void register_gpu(py::module_& m);
void register_grpc(py::module_& m);
void register_http(py::module_& m);
}  // namespace bgc_py

namespace {

// JSON text is the interchange format with Python: json.loads/dumps on the Python side.
std::string yaml_to_json(const std::string& y) { return bgc::yaml::parse(y).dump(); }
std::string json_to_yaml(const std::string& j) { return bgc::yaml::emit(bgc::json::parse(j)); }

std::string json_roundtrip(const std::string& j, const std::string& drop_key) {
  return (drop_key.empty() ? bgc::json::parse(j) : bgc::json::parse(j, drop_key)).dump();
}

// A json::Projection built from dotted paths ("request.object.spec"): every path is
// Descend along the way and Keep at its end.  Nodes live in `store`.
struct ProjectionTree {
  std::vector<std::string> keys;  // backing storage for the string_views
  struct Node {
    std::string key;
    bool keep = false;
    std::vector<Node> kids;
  };
  Node root;
  std::vector<std::unique_ptr<std::vector<bgc::json::Projection>>> store;
  bool omit_unnamed = false;
  bgc::json::Projection build(const Node& n) {
    bgc::json::Projection p;
    p.key = n.key;
    if (n.keep) {
      p.mode = bgc::json::Projection::Keep;
      return p;
    }
    p.mode = bgc::json::Projection::Descend;
    p.omit_unnamed = omit_unnamed;
    auto v = std::make_unique<std::vector<bgc::json::Projection>>();
    for (const auto& k : n.kids) v->push_back(build(k));
    p.children = v->data();
    p.n_children = v->size();
    store.push_back(std::move(v));
    return p;
  }
};

std::string json_parse_projected(const std::string& text, const std::vector<std::string>& keep, bool omit_unnamed) {
  ProjectionTree t;
  t.omit_unnamed = omit_unnamed;
  for (const auto& path : keep) {
    ProjectionTree::Node* n = &t.root;
    size_t start = 0;
    while (true) {
      size_t dot = path.find('.', start);
      std::string k = path.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
      ProjectionTree::Node* next = nullptr;
      for (auto& c : n->kids)
        if (c.key == k) next = &c;
      if (!next) {
        n->kids.push_back({k, false, {}});
        next = &n->kids.back();
      }
      n = next;
      if (dot == std::string::npos) break;
      start = dot + 1;
    }
    n->keep = true;
  }
  return bgc::json::parse_projected(text, t.build(t.root)).dump();
}

std::string apply_json_patch(const std::string& doc, const std::string& patch) {
  Value d = bgc::json::parse(doc);
  bgc::json::apply_patch(d, bgc::json::parse(patch));
  return d.dump();
}

std::string apply_merge_patch(const std::string& doc, const std::string& patch) {
  Value d = bgc::json::parse(doc);
  bgc::json::apply_merge_patch(d, bgc::json::parse(patch));
  return d.dump();
}

py::dict env_config(const std::map<std::string, std::string>& env, const std::string& kind) {
  bgc::EnvConfig c("CONF_", env);
  py::dict d;
  d["listen_addr"] = c.str("listen_addr");
  d["listen_port"] = c.u16("listen_port");
  if (kind == "admission") {
    d["cert_path"] = c.str("cert_path");
    d["key_path"] = c.str("key_path");
    d["oidc_username_prefix"] = c.str("oidc_username_prefix");
    d["default_role_name"] = c.str("default_role_name");
    d["authorized_group_names"] = c.comma_list("authorized_group_names");
  } else if (kind == "synchronizer") {
    d["google_service_account_json_path"] = c.str("google_service_account_json_path");
    d["google_file_id"] = c.str("google_file_id");
    d["sync_interval_secs"] = c.u64_or("sync_interval_secs", 60);
    d["gpu_server_name"] = c.str("gpu_server_name");
  }
  return d;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "bacchus-gpu-controller (MI355X-native) C++ core bindings";

  py::register_exception<bgc::json::ParseError>(m, "JsonParseError", PyExc_ValueError);
  py::register_exception<bgc::json::PatchError>(m, "JsonPatchError", PyExc_ValueError);
  py::register_exception<bgc::yaml::Error>(m, "YamlError", PyExc_ValueError);
  py::register_exception<bgc::ConfigError>(m, "ConfigError", PyExc_ValueError);

  m.def("json_roundtrip", &json_roundtrip, py::arg("text"), py::arg("drop_key") = "");
  m.def("yaml_to_json", &yaml_to_json);
  m.def("json_to_yaml", &json_to_yaml);
  m.def("json_parse_projected", &json_parse_projected, py::arg("text"), py::arg("keep"),
        py::arg("omit_unnamed") = false);
  m.def("json_raw_member", [](const std::string& text, const std::string& key) {
    return std::string(bgc::json::raw_member(text, key));
  });
  m.def("apply_json_patch", &apply_json_patch);
  m.def("apply_merge_patch", &apply_merge_patch);

  m.def("sha256_hex", [](py::bytes b) { return bgc::crypto::sha256_hex(std::string(b)); });
  m.def("base64_encode", [](py::bytes b, bool url, bool pad) { return bgc::crypto::base64_encode(std::string(b), url, pad); },
        py::arg("data"), py::arg("url") = false, py::arg("pad") = true);
  m.def("base64_decode", [](const std::string& s) { return py::bytes(bgc::crypto::base64_decode(s)); });
  m.def("jwt_rs256", &bgc::crypto::jwt_rs256);
  m.def("rs256_verify", [](const std::string& pem, const std::string& data, py::bytes sig) {
    return bgc::crypto::rs256_verify(pem, data, std::string(sig));
  });
  m.def("generate_rsa", [](int bits) {
    auto k = bgc::crypto::generate_rsa(bits);
    return py::make_tuple(k.private_key_pem, k.public_key_pem);
  }, py::arg("bits") = 2048);
  m.def("make_ca_and_leaf", [](const std::string& cn, const std::vector<std::string>& dns, int days,
                               const std::string& key_type) {
    auto b = bgc::crypto::make_ca_and_leaf(cn, dns, days, key_type);
    py::dict d;
    d["ca_cert"] = b.ca_cert_pem;
    d["ca_key"] = b.ca_key_pem;
    d["cert"] = b.cert_pem;
    d["key"] = b.key_pem;
    return d;
  }, py::arg("common_name"), py::arg("dns_names"), py::arg("valid_days") = 90, py::arg("key_type") = "ec");
  m.def("uuid_v4", &bgc::crypto::uuid_v4);

  m.def("env_config", &env_config, py::arg("env"), py::arg("kind"));

  m.def("log_enabled", [](const std::string& spec, const std::string& level, const std::string& target) {
    bgc::log::init(spec);
    static const std::map<std::string, bgc::log::Level> lv = {
        {"trace", bgc::log::Level::Trace}, {"debug", bgc::log::Level::Debug}, {"info", bgc::log::Level::Info},
        {"warn", bgc::log::Level::Warn}, {"error", bgc::log::Level::Error}};
    bool r = bgc::log::enabled(lv.at(level), target);
    bgc::log::init_from_env();
    return r;
  });
  m.def("malloc_trim_decision", [](long rss, long baseline, long limit_bytes) {
    return bgc::malloc_trim_decision(rss, baseline, limit_bytes) == bgc::TrimDecision::Trim ? "trim" : "skip";
  }, py::arg("rss"), py::arg("baseline"), py::arg("limit_bytes"));
  m.def("cgroup_memory_limit_bytes", &bgc::cgroup_memory_limit_bytes);
  // `threads` threads each log `lines` INFO lines "<tag> <thread> <i> xxx..." of `width` pad
  // bytes; thread 0's line number `error_at` (if >= 0) is an ERROR line instead.  Returns the
  // slowest single LOG_* call in ms (tests of the asynchronous log writer against a blocked
  // stderr).
  m.def("log_burst", [](int threads, int lines, int width, int error_at, const std::string& tag) {
    py::gil_scoped_release nogil;
    bgc::log::init("info");
    std::atomic<int64_t> worst{0};
    std::vector<std::thread> ts;
    const std::string pad(static_cast<size_t>(width), 'x');
    for (int t = 0; t < threads; ++t) {
      ts.emplace_back([&, t] {
        for (int i = 0; i < lines; ++i) {
          const auto t0 = std::chrono::steady_clock::now();
          if (t == 0 && i == error_at) {
            LOG_ERROR("burst") << tag << " " << t << " " << i << " " << pad;
          } else {
            LOG_INFO("burst") << tag << " " << t << " " << i << " " << pad;
          }
          const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
          int64_t cur = worst.load();
          while (ns > cur && !worst.compare_exchange_weak(cur, ns)) {
          }
        }
      });
    }
    for (auto& th : ts) th.join();
    return static_cast<double>(worst.load()) * 1e-6;
  }, py::arg("threads"), py::arg("lines"), py::arg("width"), py::arg("error_at") = -1, py::arg("tag") = "burst");
  m.def("log_flush", [] {
    py::gil_scoped_release nogil;
    bgc::log::flush();
  });
  m.def("log_lines_dropped", [] { return bgc::log::lines_dropped(); });
  // Per-tenant stage marks and the stall sampler of this process (the bench's load driver):
  // the same surface the services serve on /debug/trace and /debug/stalls.
  m.def("trace_arm", [](const std::string& prefix) { bgc::trace::arm(prefix); });
  m.def("trace_take", [] { return bgc::trace::dump_json(true); });
  m.def("stall_start", [](const std::string& name) {
    bgc::metrics::set_debug_endpoints(true);  // the sampler keeps its stalls only then
    bgc::stall::start(name);
  });
  m.def("stall_take", [] { return bgc::stall::dump_json(true); });
  // A KubeClient built from a $KUBECONFIG-style path list, one request per call (tests of
  // credential plugins and multi-file merging).  Returns (status, body, credential refreshes).
  m.def("kube_request", [](const std::string& kubeconfig_list, const std::string& method, const std::string& path,
                           int repeat) {
    std::vector<std::string> paths;
    size_t start = 0;
    while (true) {
      size_t colon = kubeconfig_list.find(':', start);
      paths.push_back(kubeconfig_list.substr(start, colon == std::string::npos ? std::string::npos : colon - start));
      if (colon == std::string::npos) break;
      start = colon + 1;
    }
    py::gil_scoped_release nogil;
    bgc::kube::KubeClient client(bgc::kube::KubeConfig::from_kubeconfigs(paths));
    std::vector<std::pair<int, std::string>> out;
    for (int i = 0; i < std::max(1, repeat); ++i) {
      auto r = client.raw(method, path);
      out.emplace_back(r.status, r.body);
    }
    return std::make_tuple(out, client.credential_refreshes(), client.config().source);
  }, py::arg("kubeconfig"), py::arg("method"), py::arg("path"), py::arg("repeat") = 1);
  m.def("kubeconfig_parse", [](const std::string& path, const std::string& context) {
    auto c = bgc::kube::KubeConfig::from_kubeconfig(path, context);
    py::dict d;
    d["server"] = c.server;
    d["token"] = c.token;
    d["ca_pem"] = c.ca_pem;
    d["client_cert_pem"] = c.client_cert_pem;
    d["insecure"] = c.insecure;
    d["impersonate_user"] = c.impersonate_user;
    d["impersonate_groups"] = c.impersonate_groups;
    d["auth_provider"] = c.auth_provider;
    d["basic_auth"] = c.basic_auth;
    if (c.exec) {
      py::dict e;
      e["api_version"] = c.exec->api_version;
      e["command"] = c.exec->command;
      e["args"] = c.exec->args;
      e["provide_cluster_info"] = c.exec->provide_cluster_info;
      e["interactive_mode"] = c.exec->interactive_mode;
      e["install_hint"] = c.exec->install_hint;
      d["exec"] = e;
    }
    return d;
  }, py::arg("path"), py::arg("context") = "");

  m.def("crd_yaml", &bgc::crd::crd_yaml);
  m.def("crd_json", [] { return bgc::crd::userbootstrap_crd().dump(); });
  m.def("ub_schema_json", [] { return bgc::crd::userbootstrap_schema().dump(); });
  m.def("validate_ub", [](const std::string& obj) {
    std::vector<py::tuple> out;
    for (auto& e : bgc::crd::validate(bgc::json::parse(obj), bgc::crd::userbootstrap_schema())) {
      out.push_back(py::make_tuple(e.path, e.kind, e.detail));
    }
    return out;
  });
  m.def("parse_userbootstrap", [](const std::string& obj) {
    auto ub = bgc::crd::parse_userbootstrap(bgc::json::parse(obj));
    py::dict d;
    d["name"] = ub.name;
    d["kube_username"] = ub.has_kube_username ? py::object(py::str(ub.kube_username)) : py::object(py::none());
    d["has_quota"] = ub.has_quota;
    d["has_role"] = ub.has_role;
    d["has_rolebinding"] = ub.has_rolebinding;
    d["synchronized_with_sheet"] = ub.synchronized_with_sheet;
    return d;
  });

  bgc_py::register_admission(m);
  bgc_py::register_sync(m);
  bgc_py::register_kube(m);
  bgc_py::register_gpu(m);
  bgc_py::register_grpc(m);
  bgc_py::register_http(m);
}

// HTTP/2 + gRPC + kubelet device-plugin bindings (tests cross-check them against
// libnghttp2 and python grpcio/protobuf, which are independent implementations).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <memory>

#include "core/hpack.h"
#include "core/http2.h"
#include "core/json.h"
#include "gpu/device.h"
#include "gpu/device_plugin.h"

namespace py = pybind11;
using bgc::json::Value;
namespace dp = bgc::gpu::dp;

namespace bgc_py {

namespace {

Value strings(const std::vector<std::string>& v) {
  Value a = Value::array();
  for (const auto& s : v) a.push_back(s);
  return a;
}

std::vector<std::string> strings(const Value& v) {
  std::vector<std::string> out;
  for (const auto& s : v.items()) out.push_back(s.as_string());
  return out;
}

Value smap(const std::map<std::string, std::string>& m) {
  Value o = Value::object();
  for (const auto& [k, v] : m) o[k] = v;
  return o;
}

std::map<std::string, std::string> smap(const Value& v) {
  std::map<std::string, std::string> out;
  if (v.is_object())
    for (size_t i = 0; i < v.keys().size(); ++i) out[v.keys()[i]] = v.values()[i].as_string();
  return out;
}

bool flag(const Value& v, const char* key) {
  const Value& x = v.get(key);
  return x.is_bool() && x.as_bool();
}

const std::vector<Value>& list(const Value& v, const char* key) {
  static const std::vector<Value> empty;
  const Value& x = v.get(key);
  return x.is_array() ? x.items() : empty;
}

py::bytes dp_encode(const std::string& kind, const std::string& js) {
  Value v = bgc::json::parse(js);
  std::string out;
  if (kind == "options") {
    out = dp::encode_options(flag(v, "pre_start_required"), flag(v, "get_preferred_allocation_available"));
  } else if (kind == "register_request") {
    dp::RegisterRequest r;
    r.version = v.get_string("version");
    r.endpoint = v.get_string("endpoint");
    r.resource_name = v.get_string("resource_name");
    r.pre_start_required = flag(v, "pre_start_required");
    r.get_preferred_allocation_available = flag(v, "get_preferred_allocation_available");
    out = dp::encode_register_request(r);
  } else if (kind == "list_and_watch") {
    std::vector<dp::Device> ds;
    for (const auto& d : v.items()) {
      dp::Device x;
      x.id = d.get_string("id");
      x.healthy = flag(d, "healthy");
      for (const auto& n : list(d, "numa_nodes")) x.numa_nodes.push_back(n.as_int());
      ds.push_back(std::move(x));
    }
    out = dp::encode_list_and_watch(ds);
  } else if (kind == "allocate_request" || kind == "preferred_response") {
    std::vector<std::vector<std::string>> cs;
    for (const auto& c : v.items()) cs.push_back(strings(c));
    out = kind == "allocate_request" ? dp::encode_allocate_request(cs) : dp::encode_preferred_response(cs);
  } else if (kind == "allocate_response") {
    std::vector<dp::ContainerAllocation> cs;
    for (const auto& c : v.items()) {
      dp::ContainerAllocation a;
      a.envs = smap(c.get("envs"));
      a.annotations = smap(c.get("annotations"));
      for (const auto& m : list(c, "mounts"))
        a.mounts.push_back({m.get_string("container_path"), m.get_string("host_path"), flag(m, "read_only")});
      for (const auto& d : list(c, "devices"))
        a.devices.push_back({d.get_string("container_path"), d.get_string("host_path"), d.get_string("permissions")});
      cs.push_back(std::move(a));
    }
    out = dp::encode_allocate_response(cs);
  } else if (kind == "preferred_request") {
    std::vector<dp::PreferredRequest> qs;
    for (const auto& c : v.items()) {
      dp::PreferredRequest q;
      q.available = strings(c.get("available"));
      q.must_include = strings(c.get("must_include"));
      q.size = static_cast<int32_t>(c.get("size").as_int());
      qs.push_back(std::move(q));
    }
    out = dp::encode_preferred_request(qs);
  } else {
    throw std::invalid_argument("unknown message kind " + kind);
  }
  return py::bytes(out);
}

std::string dp_decode(const std::string& kind, const std::string& buf) {
  Value out;
  if (kind == "register_request") {
    auto r = dp::decode_register_request(buf);
    out = Value::object({{"version", r.version}, {"endpoint", r.endpoint}, {"resource_name", r.resource_name},
                         {"pre_start_required", r.pre_start_required},
                         {"get_preferred_allocation_available", r.get_preferred_allocation_available}});
  } else if (kind == "list_and_watch") {
    out = Value::array();
    for (const auto& d : dp::decode_list_and_watch(buf)) {
      Value n = Value::array();
      for (auto x : d.numa_nodes) n.push_back(static_cast<long long>(x));
      out.push_back(Value::object({{"id", d.id}, {"healthy", d.healthy}, {"numa_nodes", n}}));
    }
  } else if (kind == "allocate_request" || kind == "preferred_response") {
    out = Value::array();
    for (const auto& c : kind == "allocate_request" ? dp::decode_allocate_request(buf) : dp::decode_preferred_response(buf))
      out.push_back(strings(c));
  } else if (kind == "allocate_response") {
    out = Value::array();
    for (const auto& a : dp::decode_allocate_response(buf)) {
      Value ms = Value::array(), ds = Value::array();
      for (const auto& m : a.mounts)
        ms.push_back(Value::object({{"container_path", m.container_path}, {"host_path", m.host_path}, {"read_only", m.read_only}}));
      for (const auto& d : a.devices)
        ds.push_back(Value::object({{"container_path", d.container_path}, {"host_path", d.host_path}, {"permissions", d.permissions}}));
      out.push_back(Value::object({{"envs", smap(a.envs)}, {"annotations", smap(a.annotations)}, {"mounts", ms}, {"devices", ds}}));
    }
  } else if (kind == "preferred_request") {
    out = Value::array();
    for (const auto& q : dp::decode_preferred_request(buf))
      out.push_back(Value::object({{"available", strings(q.available)}, {"must_include", strings(q.must_include)},
                                   {"size", static_cast<long long>(q.size)}}));
  } else {
    throw std::invalid_argument("unknown message kind " + kind);
  }
  return out.dump();
}

std::vector<bgc::gpu::GpuInfo> gpus_from_json(const std::string& js) {
  Value v = bgc::json::parse(js);
  const Value& arr = v.is_object() ? v.get("gpus") : v;
  std::vector<bgc::gpu::GpuInfo> gpus;
  for (const auto& g : arr.items()) gpus.push_back(bgc::gpu::gpu_info_from_json(g));
  return gpus;
}

}  // namespace

void register_grpc(py::module_& m) {
  m.def("huffman_encode", [](const std::string& s) { return py::bytes(bgc::hpack::huffman_encode(s)); });
  m.def("huffman_decode", [](const std::string& s) -> py::object {
    std::string out;
    if (!bgc::hpack::huffman_decode(s, &out)) return py::none();
    return py::bytes(out);
  });
  m.def("hpack_encode", [](const std::vector<std::pair<std::string, std::string>>& hl) {
    return py::bytes(bgc::hpack::encode(hl));
  });
  py::class_<bgc::hpack::Decoder>(m, "HpackDecoder")
      .def(py::init<size_t>(), py::arg("max_table_size") = 4096)
      .def("decode",
           [](bgc::hpack::Decoder& d, const std::string& block) {
             bgc::hpack::HeaderList hl;
             std::string err;
             if (!d.decode(block, &hl, &err)) throw std::runtime_error(err);
             std::vector<std::pair<py::bytes, py::bytes>> out;
             for (auto& [k, v] : hl) out.emplace_back(py::bytes(k), py::bytes(v));
             return out;
           })
      .def_property_readonly("table_size", &bgc::hpack::Decoder::table_size)
      .def_property_readonly("table_entries", &bgc::hpack::Decoder::table_entries);

  m.def("dp_encode", &dp_encode, py::arg("kind"), py::arg("json"));
  m.def("dp_decode", [](const std::string& kind, const std::string& buf) { return dp_decode(kind, buf); });
  m.def("preferred_allocation",
        [](const std::string& gpus_json, const std::vector<std::string>& ids, const std::vector<std::string>& available,
           const std::vector<std::string>& must_include, int size) {
          return bgc::gpu::preferred_allocation(gpus_from_json(gpus_json), ids, available, must_include, size);
        });

  // kubelet pod-resources v1 (List) codec + client
  m.def("pod_resources_encode", [](const std::string& js) {
    std::vector<bgc::gpu::PodDevices> v;
    const bgc::json::Value parsed = bgc::json::parse(js);
    for (const auto& p : parsed.items()) {
      bgc::gpu::PodDevices d{p.get_string("pod"), p.get_string("namespace"), p.get_string("container"),
                             p.get_string("resource"), {}};
      for (const auto& id : p.get("ids").items()) d.ids.push_back(id.as_string());
      v.push_back(std::move(d));
    }
    return py::bytes(bgc::gpu::encode_pod_resources(v));
  });
  m.def("pod_resources_decode", [](const std::string& buf) {
    bgc::json::Value out = bgc::json::Value::array();
    for (const auto& d : bgc::gpu::decode_pod_resources(buf)) {
      bgc::json::Value ids = bgc::json::Value::array();
      for (const auto& id : d.ids) ids.push_back(id);
      out.push_back(bgc::json::Value::object({{"pod", d.pod}, {"namespace", d.ns}, {"container", d.container},
                                              {"resource", d.resource}, {"ids", ids}}));
    }
    return out.dump();
  });
  m.def("allocated_device_ids", [](const std::string& socket, const std::string& resource) {
    py::gil_scoped_release nogil;
    return bgc::gpu::allocated_device_ids(socket, resource);
  });

  py::class_<bgc::grpc::Channel>(m, "GrpcChannel")
      .def(py::init<std::string, int>(), py::arg("target"), py::arg("connect_timeout_ms") = 5000)
      .def("unary",
           [](bgc::grpc::Channel& c, const std::string& method, const std::string& req, int timeout_ms) {
             std::string resp;
             bgc::grpc::Status st;
             {
               py::gil_scoped_release nogil;
               st = c.unary(method, req, &resp, std::chrono::milliseconds(timeout_ms));
             }
             return py::make_tuple(st.code, st.message, py::bytes(resp));
           },
           py::arg("method"), py::arg("request"), py::arg("timeout_ms") = 10000)
      .def("server_stream",
           [](bgc::grpc::Channel& c, const std::string& method, const std::string& req, int max_msgs, int timeout_ms) {
             std::vector<std::string> msgs;
             bgc::grpc::Status st;
             {
               py::gil_scoped_release nogil;
               st = c.server_stream(
                   method, req,
                   [&](const std::string& m) {
                     msgs.push_back(m);
                     return max_msgs <= 0 || static_cast<int>(msgs.size()) < max_msgs;
                   },
                   std::chrono::milliseconds(timeout_ms));
             }
             py::list out;
             for (auto& s : msgs) out.append(py::bytes(s));
             return py::make_tuple(st.code, st.message, out);
           },
           py::arg("method"), py::arg("request"), py::arg("max_msgs") = 0, py::arg("timeout_ms") = 10000)
      .def("close", &bgc::grpc::Channel::close);

  py::class_<bgc::gpu::DevicePlugin>(m, "DevicePlugin")
      .def(py::init([](const std::string& gpus_json, const std::map<std::string, std::string>& cfg) {
             bgc::gpu::DevicePluginConfig c;
             auto get = [&](const char* k, std::string& dst) {
               auto it = cfg.find(k);
               if (it != cfg.end()) dst = it->second;
             };
             get("plugin_dir", c.plugin_dir);
             get("socket_name", c.socket_name);
             get("kubelet_socket", c.kubelet_socket);
             get("resource_name", c.resource_name);
             get("dev_root", c.dev_root);
             get("sysfs_root", c.sysfs_root);
             if (cfg.count("watch_interval_ms")) c.watch_interval_ms = std::stoi(cfg.at("watch_interval_ms"));
             if (cfg.count("register")) c.register_with_kubelet = cfg.at("register") == "true";
             if (cfg.count("cdi")) c.cdi = cfg.at("cdi") == "true";
             get("cdi_dir", c.cdi_dir);
             return std::make_unique<bgc::gpu::DevicePlugin>(gpus_from_json(gpus_json), c);
           }),
           py::arg("gpus_json"), py::arg("config"))
      .def("start", &bgc::gpu::DevicePlugin::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &bgc::gpu::DevicePlugin::stop, py::call_guard<py::gil_scoped_release>())
      .def("set_health", &bgc::gpu::DevicePlugin::set_health)
      .def("set_fenced", &bgc::gpu::DevicePlugin::set_fenced)
      .def("fenced", &bgc::gpu::DevicePlugin::fenced)
      .def("allocation_counts", &bgc::gpu::DevicePlugin::allocation_counts)
      .def("allocate_json", [](bgc::gpu::DevicePlugin& p, const std::vector<std::string>& ids) {
        auto c = p.allocate(ids);
        bgc::json::Value devs = bgc::json::Value::array();
        for (const auto& d : c.devices) {
          devs.push_back(bgc::json::Value::object(
              {{"container_path", d.container_path}, {"host_path", d.host_path}, {"permissions", d.permissions}}));
        }
        bgc::json::Value envs = bgc::json::Value::object();
        for (const auto& [k, v] : c.envs) envs[k] = v;
        bgc::json::Value cdi = bgc::json::Value::array();
        for (const auto& n : c.cdi_devices) cdi.push_back(n);
        return bgc::json::Value::object({{"devices", devs}, {"envs", envs}, {"cdi_devices", cdi}}).dump();
      })
      .def("write_cdi_spec", &bgc::gpu::DevicePlugin::write_cdi_spec)
      .def_property_readonly("ids", &bgc::gpu::DevicePlugin::ids)
      .def_property_readonly("socket_path", &bgc::gpu::DevicePlugin::socket_path)
      .def_property_readonly("registrations", &bgc::gpu::DevicePlugin::registrations)
      .def_property_readonly("server_restarts", &bgc::gpu::DevicePlugin::server_restarts)
      .def("describe", [](const bgc::gpu::DevicePlugin& p) { return p.describe().dump(); });
}

}  // namespace bgc_py

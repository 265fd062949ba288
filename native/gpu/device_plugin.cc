#include "gpu/device_plugin.h"

#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <set>
#include <stdexcept>

#include "core/log.h"
#include "core/metrics.h"
#include "core/net.h"
#include "core/protobuf.h"

namespace bgc::gpu {

// ------------------------------------------------------------------ wire codecs
namespace dp {

using pb::Reader;
using pb::Writer;

std::string encode_options(bool pre_start_required, bool get_preferred_allocation_available) {
  Writer w;
  w.boolean(1, pre_start_required);
  w.boolean(2, get_preferred_allocation_available);
  return w.take();
}

std::string encode_register_request(const RegisterRequest& r) {
  Writer w;
  w.str(1, r.version);
  w.str(2, r.endpoint);
  w.str(3, r.resource_name);
  Writer o;
  o.boolean(1, r.pre_start_required);
  o.boolean(2, r.get_preferred_allocation_available);
  w.message(4, o);
  return w.take();
}

RegisterRequest decode_register_request(std::string_view buf) {
  RegisterRequest r;
  Reader rd(buf);
  while (rd.next()) {
    switch (rd.field()) {
      case 1: r.version = rd.string_value(); break;
      case 2: r.endpoint = rd.string_value(); break;
      case 3: r.resource_name = rd.string_value(); break;
      case 4: {
        Reader o(rd.bytes_value());
        while (o.next()) {
          if (o.field() == 1) r.pre_start_required = o.bool_value();
          else if (o.field() == 2) r.get_preferred_allocation_available = o.bool_value();
        }
        break;
      }
      default: break;
    }
  }
  return r;
}

std::string encode_list_and_watch(const std::vector<Device>& devices) {
  Writer w;
  for (const auto& d : devices) {
    Writer dw;
    dw.str(1, d.id);
    dw.str(2, d.healthy ? kHealthy : kUnhealthy);
    if (!d.numa_nodes.empty()) {
      Writer topo;
      for (int64_t n : d.numa_nodes) {
        Writer node;
        node.i64(1, n);
        topo.message(1, node);
      }
      dw.message(3, topo);
    }
    w.message(1, dw);
  }
  return w.take();
}

std::vector<Device> decode_list_and_watch(std::string_view buf) {
  std::vector<Device> out;
  Reader rd(buf);
  while (rd.next()) {
    if (rd.field() != 1) continue;
    Device d;
    Reader dr(rd.bytes_value());
    while (dr.next()) {
      if (dr.field() == 1) {
        d.id = dr.string_value();
      } else if (dr.field() == 2) {
        d.healthy = dr.string_value() == kHealthy;
      } else if (dr.field() == 3) {
        Reader tr(dr.bytes_value());
        while (tr.next()) {
          if (tr.field() != 1) continue;
          int64_t id = 0;
          Reader nr(tr.bytes_value());
          while (nr.next())
            if (nr.field() == 1) id = nr.int64_value();
          d.numa_nodes.push_back(id);
        }
      }
    }
    out.push_back(std::move(d));
  }
  return out;
}

static std::vector<std::string> read_strings(std::string_view buf, uint32_t field) {
  std::vector<std::string> out;
  Reader r(buf);
  while (r.next())
    if (r.field() == field) out.push_back(r.string_value());
  return out;
}

std::string encode_allocate_request(const std::vector<std::vector<std::string>>& containers) {
  Writer w;
  for (const auto& ids : containers) {
    Writer c;
    for (const auto& id : ids) c.bytes(1, id);
    w.message(1, c);
  }
  return w.take();
}

std::vector<std::vector<std::string>> decode_allocate_request(std::string_view buf) {
  std::vector<std::vector<std::string>> out;
  Reader r(buf);
  while (r.next())
    if (r.field() == 1) out.push_back(read_strings(r.bytes_value(), 1));
  return out;
}

std::string encode_allocate_response(const std::vector<ContainerAllocation>& containers) {
  Writer w;
  for (const auto& c : containers) {
    Writer cw;
    for (const auto& [k, v] : c.envs) cw.map_entry(1, k, v);
    for (const auto& m : c.mounts) {
      Writer mw;
      mw.str(1, m.container_path);
      mw.str(2, m.host_path);
      mw.boolean(3, m.read_only);
      cw.message(2, mw);
    }
    for (const auto& d : c.devices) {
      Writer dw;
      dw.str(1, d.container_path);
      dw.str(2, d.host_path);
      dw.str(3, d.permissions);
      cw.message(3, dw);
    }
    for (const auto& [k, v] : c.annotations) cw.map_entry(4, k, v);
    for (const auto& name : c.cdi_devices) {
      Writer dw;
      dw.str(1, name);
      cw.message(5, dw);
    }
    w.message(1, cw);
  }
  return w.take();
}

std::vector<ContainerAllocation> decode_allocate_response(std::string_view buf) {
  std::vector<ContainerAllocation> out;
  Reader r(buf);
  while (r.next()) {
    if (r.field() != 1) continue;
    ContainerAllocation c;
    Reader cr(r.bytes_value());
    while (cr.next()) {
      switch (cr.field()) {
        case 1: c.envs.insert(pb::read_map_entry(cr.bytes_value())); break;
        case 4: c.annotations.insert(pb::read_map_entry(cr.bytes_value())); break;
        case 5: {
          Reader nr(cr.bytes_value());
          while (nr.next())
            if (nr.field() == 1) c.cdi_devices.push_back(nr.string_value());
          break;
        }
        case 2: {
          Mount m;
          Reader mr(cr.bytes_value());
          while (mr.next()) {
            if (mr.field() == 1) m.container_path = mr.string_value();
            else if (mr.field() == 2) m.host_path = mr.string_value();
            else if (mr.field() == 3) m.read_only = mr.bool_value();
          }
          c.mounts.push_back(std::move(m));
          break;
        }
        case 3: {
          DeviceSpec d;
          Reader dr(cr.bytes_value());
          while (dr.next()) {
            if (dr.field() == 1) d.container_path = dr.string_value();
            else if (dr.field() == 2) d.host_path = dr.string_value();
            else if (dr.field() == 3) d.permissions = dr.string_value();
          }
          c.devices.push_back(std::move(d));
          break;
        }
        default: break;
      }
    }
    out.push_back(std::move(c));
  }
  return out;
}

std::string encode_preferred_request(const std::vector<PreferredRequest>& reqs) {
  Writer w;
  for (const auto& q : reqs) {
    Writer c;
    for (const auto& id : q.available) c.bytes(1, id);
    for (const auto& id : q.must_include) c.bytes(2, id);
    c.i32(3, q.size);
    w.message(1, c);
  }
  return w.take();
}

std::vector<PreferredRequest> decode_preferred_request(std::string_view buf) {
  std::vector<PreferredRequest> out;
  Reader r(buf);
  while (r.next()) {
    if (r.field() != 1) continue;
    PreferredRequest q;
    Reader cr(r.bytes_value());
    while (cr.next()) {
      if (cr.field() == 1) q.available.push_back(cr.string_value());
      else if (cr.field() == 2) q.must_include.push_back(cr.string_value());
      else if (cr.field() == 3) q.size = static_cast<int32_t>(cr.int64_value());
    }
    out.push_back(std::move(q));
  }
  return out;
}

std::string encode_preferred_response(const std::vector<std::vector<std::string>>& per_container) {
  Writer w;
  for (const auto& ids : per_container) {
    Writer c;
    for (const auto& id : ids) c.bytes(1, id);
    w.message(1, c);
  }
  return w.take();
}

std::vector<std::vector<std::string>> decode_preferred_response(std::string_view buf) {
  return decode_allocate_request(buf);  // same shape: repeated {repeated string = 1} = 1
}

}  // namespace dp

// ------------------------------------------------------------------ pod resources
// podresources/v1: ListPodResourcesResponse{1: repeated PodResources}
// PodResources{1: name, 2: namespace, 3: repeated ContainerResources}
// ContainerResources{1: name, 2: repeated ContainerDevices, ...}
// ContainerDevices{1: resource_name, 2: repeated device_ids, 3: TopologyInfo}
std::vector<PodDevices> decode_pod_resources(std::string_view buf) {
  std::vector<PodDevices> out;
  pb::Reader r(buf);
  while (r.next()) {
    if (r.field() != 1) continue;
    std::string pod, ns;
    std::vector<std::string_view> containers;
    pb::Reader pr(r.bytes_value());
    while (pr.next()) {
      if (pr.field() == 1) pod = pr.string_value();
      else if (pr.field() == 2) ns = pr.string_value();
      else if (pr.field() == 3) containers.push_back(pr.bytes_value());
    }
    for (auto c : containers) {
      std::string cname;
      std::vector<std::string_view> devs;
      pb::Reader cr(c);
      while (cr.next()) {
        if (cr.field() == 1) cname = cr.string_value();
        else if (cr.field() == 2) devs.push_back(cr.bytes_value());
      }
      for (auto d : devs) {
        PodDevices pd{pod, ns, cname, "", {}};
        pb::Reader dr(d);
        while (dr.next()) {
          if (dr.field() == 1) pd.resource = dr.string_value();
          else if (dr.field() == 2) pd.ids.push_back(dr.string_value());
        }
        out.push_back(std::move(pd));
      }
    }
  }
  return out;
}

std::string encode_pod_resources(const std::vector<PodDevices>& v) {
  pb::Writer w;
  for (const auto& p : v) {
    pb::Writer d;
    d.str(1, p.resource);
    for (const auto& id : p.ids) d.bytes(2, id);
    pb::Writer c;
    c.str(1, p.container);
    c.message(2, d);
    pb::Writer pr;
    pr.str(1, p.pod);
    pr.str(2, p.ns);
    pr.message(3, c);
    w.message(1, pr);
  }
  return w.take();
}

std::set<std::string> allocated_device_ids(const std::string& socket, const std::string& resource_name) {
  grpc::Channel ch(socket, 2000);
  std::string resp;
  grpc::Status st = ch.unary("/v1.PodResourcesLister/List", "", &resp, std::chrono::seconds(5));
  if (!st.ok()) throw std::runtime_error("PodResourcesLister/List: " + st.message);
  std::set<std::string> out;
  for (const auto& p : decode_pod_resources(resp)) {
    if (p.resource != resource_name) continue;
    out.insert(p.ids.begin(), p.ids.end());
  }
  return out;
}

// ------------------------------------------------------------------ allocation policy
namespace {

// Direct-link score between two GPUs from the amdsmi link map: xGMI bandwidth (or a
// nominal value when only the type is known), PCIe a distant second, 0 = no data.
double link_score(const GpuInfo& a, int peer) {
  for (const auto& l : a.links) {
    if (l.peer != peer) continue;
    if (l.type == "xgmi") return 1.0 + (l.hops <= 1 ? static_cast<double>(l.max_bw_mbps ? l.max_bw_mbps : 50000) : 0.0);
    if (l.type == "pcie") return 0.5;
    return 0.0;
  }
  return 0.0;
}

bool have_link_map(const std::vector<GpuInfo>& gpus, const std::vector<size_t>& cand) {
  for (size_t i : cand)
    if (gpus[i].links.empty()) return false;
  return cand.size() > 1;
}

// Greedy max-bandwidth clique growth: start from `seed` (the must-include GPUs of this
// hive), then repeatedly add the candidate with the highest summed link score to
// everything chosen so far (with nothing chosen yet: to every candidate).  Ties — e.g.
// a healthy full xGMI mesh — fall back to the NUMA rules of the no-link-map path:
// NUMA node of the chosen set, then the NUMA group that best fits the request, then
// xGMI node id and index.
std::vector<size_t> pick_by_links(const std::vector<GpuInfo>& gpus, std::vector<size_t> cand,
                                  const std::vector<size_t>& seed, int need) {
  std::vector<size_t> chosen = seed, out;
  std::map<int, int> numa_count;
  for (size_t i : cand) numa_count[gpus[i].numa_node]++;
  const int want = need;
  auto score_to = [&](size_t i, const std::vector<size_t>& set) {
    double sc = 0;
    for (size_t j : set) sc += link_score(gpus[i], gpus[j].index);
    return std::round(sc);
  };
  auto better = [&](size_t a, size_t b) {
    const double sa = chosen.empty() ? score_to(a, cand) : score_to(a, chosen);
    const double sb = chosen.empty() ? score_to(b, cand) : score_to(b, chosen);
    if (sa != sb) return sa > sb;
    const int na = gpus[a].numa_node, nb = gpus[b].numa_node;
    if (na != nb) {
      int aa = 0, ab = 0;
      for (size_t j : chosen) {
        aa += gpus[j].numa_node == na;
        ab += gpus[j].numa_node == nb;
      }
      if (aa != ab) return aa > ab;
      const bool fa = numa_count[na] >= want, fb = numa_count[nb] >= want;
      if (fa != fb) return fa;
      if (numa_count[na] != numa_count[nb]) return fa ? numa_count[na] < numa_count[nb] : numa_count[na] > numa_count[nb];
      return na < nb;
    }
    if (gpus[a].xgmi_node_id != gpus[b].xgmi_node_id) return gpus[a].xgmi_node_id < gpus[b].xgmi_node_id;
    return gpus[a].index < gpus[b].index;
  };
  while (need > 0 && !cand.empty()) {
    size_t best = 0;
    for (size_t k = 1; k < cand.size(); ++k)
      if (better(cand[k], cand[best])) best = k;
    chosen.push_back(cand[best]);
    out.push_back(cand[best]);
    cand.erase(cand.begin() + static_cast<std::ptrdiff_t>(best));
    --need;
  }
  return out;
}

}  // namespace

std::vector<std::string> preferred_allocation(const std::vector<GpuInfo>& gpus, const std::vector<std::string>& ids,
                                              const std::vector<std::string>& available,
                                              const std::vector<std::string>& must_include, int size) {
  std::map<std::string, size_t> pos;
  for (size_t i = 0; i < ids.size() && i < gpus.size(); ++i) pos[ids[i]] = i;
  std::vector<std::string> out;
  std::set<std::string> taken;
  for (const auto& id : must_include) {
    if (static_cast<int>(out.size()) >= size) break;
    if (taken.insert(id).second) out.push_back(id);
  }
  int need = size - static_cast<int>(out.size());
  if (need <= 0) return out;

  // Candidates grouped by hive; unknown ids (not ours) go last in their given order.
  std::map<uint64_t, std::vector<size_t>> by_hive;
  std::vector<std::string> unknown;
  for (const auto& id : available) {
    if (!taken.insert(id).second) continue;  // must-include, or listed twice
    auto it = pos.find(id);
    if (it == pos.end()) {
      unknown.push_back(id);
      continue;
    }
    by_hive[gpus[it->second].xgmi_hive_id].push_back(it->second);
  }
  // Hive and NUMA of the must-include set pull the rest of the allocation toward them.
  std::map<uint64_t, int> must_hive;
  std::map<int, int> must_numa;
  for (const auto& id : out) {
    auto it = pos.find(id);
    if (it == pos.end()) continue;
    must_hive[gpus[it->second].xgmi_hive_id]++;
    must_numa[gpus[it->second].numa_node]++;
  }
  std::vector<uint64_t> hive_order;
  for (auto& [h, v] : by_hive) hive_order.push_back(h);
  auto fits = [&](uint64_t h) { return static_cast<int>(by_hive[h].size()) >= need; };
  std::stable_sort(hive_order.begin(), hive_order.end(), [&](uint64_t a, uint64_t b) {
    int ma = must_hive.count(a) ? must_hive[a] : 0, mb = must_hive.count(b) ? must_hive[b] : 0;
    if (ma != mb) return ma > mb;                      // the must-include hive first
    if (fits(a) != fits(b)) return fits(a);            // then hives that hold the whole request
    if (fits(a)) return by_hive[a].size() < by_hive[b].size();  // best fit keeps big islands whole
    return by_hive[a].size() > by_hive[b].size();      // else fewest hives: biggest first
  });
  std::vector<size_t> must_idx;
  for (const auto& id : out) {
    auto it = pos.find(id);
    if (it != pos.end()) must_idx.push_back(it->second);
  }
  for (uint64_t h : hive_order) {
    auto& cand = by_hive[h];
    if (have_link_map(gpus, cand)) {
      std::vector<size_t> seed;
      for (size_t i : must_idx)
        if (gpus[i].xgmi_hive_id == h) seed.push_back(i);
      for (size_t i : pick_by_links(gpus, cand, seed, need)) {
        out.push_back(ids[i]);
        --need;
      }
      if (need == 0) break;
      continue;
    }
    // Within a hive: prefer the NUMA node of the must-include set, else the NUMA group that
    // best fits what is still needed, then adjacent xGMI node ids.
    std::map<int, int> numa_count;
    for (size_t i : cand) numa_count[gpus[i].numa_node]++;
    const int want = need;
    std::stable_sort(cand.begin(), cand.end(), [&](size_t a, size_t b) {
      const int na = gpus[a].numa_node, nb = gpus[b].numa_node;
      if (na != nb) {
        int ma = must_numa.count(na) ? must_numa[na] : 0, mb = must_numa.count(nb) ? must_numa[nb] : 0;
        if (ma != mb) return ma > mb;
        bool fa = numa_count[na] >= want, fb = numa_count[nb] >= want;
        if (fa != fb) return fa;
        if (fa && numa_count[na] != numa_count[nb]) return numa_count[na] < numa_count[nb];
        if (!fa && numa_count[na] != numa_count[nb]) return numa_count[na] > numa_count[nb];
        return na < nb;
      }
      if (gpus[a].xgmi_node_id != gpus[b].xgmi_node_id) return gpus[a].xgmi_node_id < gpus[b].xgmi_node_id;
      return gpus[a].index < gpus[b].index;
    });
    for (size_t i : cand) {
      if (need == 0) break;
      out.push_back(ids[i]);
      --need;
    }
    if (need == 0) break;
  }
  for (const auto& id : unknown) {
    if (need == 0) break;
    out.push_back(id);
    --need;
  }
  return out;
}

// ------------------------------------------------------------------ plugin
namespace {

std::string join_path(const std::string& dir, const std::string& name) {
  if (dir.empty()) return name;
  return dir.back() == '/' ? dir + name : dir + "/" + name;
}

uint64_t inode_of(const std::string& path) {
  struct stat st {};
  return ::stat(path.c_str(), &st) == 0 ? static_cast<uint64_t>(st.st_ino) : 0;
}

std::string hex16(uint64_t v) {
  char buf[32];
  std::snprintf(buf, sizeof(buf), "%016llx", static_cast<unsigned long long>(v));
  return buf;
}

// card* / renderD* names of a PCI function's DRM nodes (empty when sysfs lacks them).
void drm_nodes(const std::string& sysfs_root, const std::string& bdf, std::string* card, std::string* render) {
  if (bdf.empty()) return;
  const std::string dir = sysfs_root + "/bus/pci/devices/" + bdf + "/drm";
  DIR* d = ::opendir(dir.c_str());
  if (!d) return;
  while (dirent* e = ::readdir(d)) {
    std::string n = e->d_name;
    if (n.rfind("renderD", 0) == 0) *render = n;
    else if (n.rfind("card", 0) == 0 && n.find('-') == std::string::npos) *card = n;
  }
  ::closedir(d);
}

}  // namespace

DevicePlugin::DevicePlugin(std::vector<GpuInfo> gpus, DevicePluginConfig cfg)
    : gpus_(std::move(gpus)),
      cfg_(std::move(cfg)),
      healthy_(gpus_.size(), true),
      fenced_(gpus_.size(), false),
      alloc_counts_(gpus_.size(), 0) {
  ids_ = device_ids_for(gpus_);
  std::map<std::string, int> seen;
  for (const auto& g : gpus_) seen[g.bdf]++;
  for (const auto& g : gpus_) shared_bdf_.push_back(!g.bdf.empty() && seen[g.bdf] > 1);
}

std::vector<std::string> device_ids_for(const std::vector<GpuInfo>& gpus) {
  // ID = PCI BDF; compute partitions of one GPU can share a BDF, so duplicates get the
  // logical device index appended.
  std::map<std::string, int> seen;
  for (const auto& g : gpus) seen[g.bdf]++;
  std::vector<std::string> ids;
  for (const auto& g : gpus) {
    if (g.bdf.empty()) ids.push_back("gpu-" + std::to_string(g.index));
    else if (seen[g.bdf] > 1) ids.push_back(g.bdf + "-p" + std::to_string(g.index));
    else ids.push_back(g.bdf);
  }
  return ids;
}

std::set<std::string> checkpoint_devices(const std::string& plugin_dir, const std::string& resource, bool* readable) {
  std::set<std::string> out;
  if (readable) *readable = false;
  std::string text;
  try {
    text = net::read_file(join_path(plugin_dir, "kubelet_internal_checkpoint"));
  } catch (const std::exception&) {
    return out;
  }
  json::Value cp;
  if (!json::try_parse(text, cp)) return out;
  if (readable) *readable = true;
  // {"Data":{"PodDeviceEntries":[...],"RegisteredDevices":{"<resource>":["id",...]}},"Checksum":N}
  for (const auto& id : cp.get("Data").get("RegisteredDevices").get(resource).items()) {
    if (id.is_string()) out.insert(id.as_string());
  }
  return out;
}

std::vector<ForeignPlugin> foreign_plugins_for(const std::string& plugin_dir, const std::string& kubelet_socket,
                                               const std::string& own_socket, const std::string& resource,
                                               const std::vector<std::string>& own_ids, int timeout_ms) {
  std::vector<ForeignPlugin> out;
  DIR* d = ::opendir(plugin_dir.c_str());
  if (!d) return out;
  std::vector<std::string> sockets;
  while (dirent* e = ::readdir(d)) {
    const std::string name = e->d_name;
    if (name == "." || name == ".." || name == kubelet_socket || name == own_socket) continue;
    struct stat st{};
    if (::stat(join_path(plugin_dir, name).c_str(), &st) == 0 && S_ISSOCK(st.st_mode)) sockets.push_back(name);
  }
  ::closedir(d);
  std::sort(sockets.begin(), sockets.end());
  if (sockets.empty()) return out;
  bool cp_ok = false;
  const std::set<std::string> registered = checkpoint_devices(plugin_dir, resource, &cp_ok);
  const std::set<std::string> ours(own_ids.begin(), own_ids.end());
  for (const auto& name : sockets) {
    ForeignPlugin fp;
    fp.socket = name;
    bool answered = false;
    try {
      grpc::Channel ch(join_path(plugin_dir, name), timeout_ms);
      grpc::Status st = ch.server_stream(
          "/v1beta1.DevicePlugin/ListAndWatch", "",
          [&](const std::string& msg) {
            for (const auto& dev : dp::decode_list_and_watch(msg)) fp.ids.push_back(dev.id);
            answered = true;
            return false;  // the first list is enough
          },
          std::chrono::milliseconds(timeout_ms));
      (void)st;  // cancelled by us after the first message, or a stale socket / not a device plugin
      ch.close();
    } catch (const std::exception&) {
      continue;  // stale socket: nobody listening
    }
    if (!answered) continue;
    bool serves = false;
    for (const auto& id : fp.ids) {
      if (cp_ok ? registered.count(id) > 0 : ours.count(id) > 0) {
        serves = true;
        break;
      }
    }
    if (!serves) continue;
    fp.via_checkpoint = cp_ok;
    out.push_back(std::move(fp));
  }
  return out;
}

DevicePlugin::~DevicePlugin() { stop(); }

std::string DevicePlugin::socket_path() const { return join_path(cfg_.plugin_dir, cfg_.socket_name); }

std::vector<dp::Device> DevicePlugin::devices() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<dp::Device> out;
  for (size_t i = 0; i < gpus_.size(); ++i) {
    dp::Device d;
    d.id = ids_[i];
    d.healthy = healthy_[i] && !fenced_[i];
    if (gpus_[i].numa_node >= 0) d.numa_nodes.push_back(gpus_[i].numa_node);
    out.push_back(std::move(d));
  }
  return out;
}

void DevicePlugin::set_health(const std::vector<bool>& healthy) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    bool changed = false;
    for (size_t i = 0; i < healthy_.size() && i < healthy.size(); ++i) {
      if (healthy_[i] != healthy[i]) {
        healthy_[i] = healthy[i];
        changed = true;
        LOG_INFO("device_plugin") << cfg_.resource_name << " " << ids_[i] << " -> "
                                  << (healthy[i] ? dp::kHealthy : dp::kUnhealthy);
      }
    }
    if (!changed) return;
    ++version_;
  }
  cv_.notify_all();
}

void DevicePlugin::set_fenced(const std::vector<size_t>& which, bool fenced) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    bool changed = false;
    for (size_t i : which) {
      if (i >= fenced_.size() || fenced_[i] == fenced) continue;
      fenced_[i] = fenced;
      changed = true;
      LOG_INFO("device_plugin") << cfg_.resource_name << " " << ids_[i]
                                << (fenced ? " fenced for diagnostics" : " released from diagnostics");
    }
    if (!changed) return;
    ++version_;
  }
  cv_.notify_all();
}

std::vector<bool> DevicePlugin::fenced() const {
  std::lock_guard<std::mutex> lk(mu_);
  return fenced_;
}

std::vector<uint64_t> DevicePlugin::allocation_counts() const {
  std::lock_guard<std::mutex> lk(mu_);
  return alloc_counts_;
}

std::pair<std::string, std::string> DevicePlugin::drm_node_names(size_t gi) const {
  const GpuInfo& g = gpus_[gi];
  std::string card, render;
  if (shared_bdf_[gi]) {
    // A compute partition: the BDF's DRM nodes belong to partition 0, so only the
    // minors amdsmi reported for this logical device are correct.
    if (g.drm_render <= 0) {
      throw std::invalid_argument(cfg_.resource_name + " device " + ids_[gi] +
                                  " shares its PCI function with another partition and its render node is unknown");
    }
    render = "renderD" + std::to_string(g.drm_render);
    if (g.drm_card >= 0) card = "card" + std::to_string(g.drm_card);
  } else {
    drm_nodes(cfg_.sysfs_root, g.bdf, &card, &render);
    if (render.empty() && g.drm_render > 0) render = "renderD" + std::to_string(g.drm_render);
    if (card.empty() && g.drm_card >= 0) card = "card" + std::to_string(g.drm_card);
  }
  if (card.empty()) card = "card" + std::to_string(g.index);
  if (render.empty()) render = "renderD" + std::to_string(128 + g.index);
  return {card, render};
}

dp::ContainerAllocation DevicePlugin::allocate(const std::vector<std::string>& req_ids) {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<size_t> idx;
  for (const auto& id : req_ids) {
    auto it = std::find(ids_.begin(), ids_.end(), id);
    if (it == ids_.end()) throw std::invalid_argument("unknown " + cfg_.resource_name + " device id " + id);
    idx.push_back(static_cast<size_t>(it - ids_.begin()));
    if (fenced_[idx.back()]) {
      refused_fenced_.fetch_add(1);
      throw std::invalid_argument(cfg_.resource_name + " device " + id + " is under node diagnostics");
    }
  }
  dp::ContainerAllocation c;
  if (!cfg_.cdi) c.devices.push_back({"/dev/kfd", join_path(cfg_.dev_root, "kfd"), "rw"});
  std::set<uint64_t> hives;
  std::string id_list;
  for (const auto& id : req_ids) {
    auto it = std::find(ids_.begin(), ids_.end(), id);
    if (it == ids_.end()) throw std::invalid_argument("unknown " + cfg_.resource_name + " device id " + id);
    const size_t gi = static_cast<size_t>(it - ids_.begin());
    const GpuInfo& g = gpus_[gi];
    if (cfg_.cdi) {
      if (shared_bdf_[gi] && g.drm_render <= 0) (void)drm_node_names(gi);  // same refusal as device specs
      c.cdi_devices.push_back(cfg_.resource_name + "=" + id);
    } else {
      const auto [card, render] = drm_node_names(gi);
      c.devices.push_back({"/dev/dri/" + card, join_path(cfg_.dev_root, "dri/" + card), "rw"});
      c.devices.push_back({"/dev/dri/" + render, join_path(cfg_.dev_root, "dri/" + render), "rw"});
    }
    hives.insert(g.xgmi_hive_id);
    if (!id_list.empty()) id_list += ",";
    id_list += id;
  }
  std::string hive_list;
  for (uint64_t h : hives) hive_list += (hive_list.empty() ? "" : ",") + hex16(h);
  c.envs["BGC_AMD_GPU_IDS"] = id_list;
  c.envs["BGC_AMD_GPU_XGMI_HIVES"] = hive_list;
  c.envs["BGC_AMD_GPU_SINGLE_XGMI_HIVE"] = hives.size() <= 1 ? "true" : "false";
  for (size_t i : idx) alloc_counts_[i]++;
  return c;
}

json::Value cdi_spec(const std::string& kind, const std::vector<GpuInfo>& gpus, const std::vector<std::string>& ids,
                     const std::vector<std::pair<std::string, std::string>>& nodes) {
  json::Value devs = json::Value::array();
  for (size_t i = 0; i < gpus.size() && i < ids.size() && i < nodes.size(); ++i) {
    json::Value dn = json::Value::array();
    dn.push_back(json::Value::object({{"path", "/dev/dri/" + nodes[i].first}}));
    dn.push_back(json::Value::object({{"path", "/dev/dri/" + nodes[i].second}}));
    devs.push_back(json::Value::object({{"name", ids[i]},
                                        {"containerEdits", json::Value::object({{"deviceNodes", dn}})}}));
  }
  return json::Value::object(
      {{"cdiVersion", "0.6.0"},
       {"kind", kind},
       {"devices", devs},
       {"containerEdits",
        json::Value::object({{"deviceNodes", json::Value::array({json::Value::object({{"path", "/dev/kfd"}})})}})}});
}

std::string DevicePlugin::write_cdi_spec() const {
  std::vector<std::pair<std::string, std::string>> nodes;
  std::vector<GpuInfo> gpus;
  std::vector<std::string> ids;
  for (size_t i = 0; i < gpus_.size(); ++i) {
    try {
      nodes.push_back(drm_node_names(i));
      gpus.push_back(gpus_[i]);
      ids.push_back(ids_[i]);
    } catch (const std::invalid_argument& e) {
      LOG_WARN("device_plugin") << "CDI spec: " << e.what();  // left out: Allocate refuses it too
    }
  }
  ::mkdir(cfg_.cdi_dir.c_str(), 0755);
  std::string kind = cfg_.resource_name;
  std::string file = kind;
  std::replace(file.begin(), file.end(), '/', '-');
  const std::string path = join_path(cfg_.cdi_dir, "bgc-" + file + ".json");
  const std::string tmp = path + ".tmp";
  net::write_file(tmp, cdi_spec(kind, gpus, ids, nodes).dump());
  if (::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename " + tmp + " failed");
  return path;
}

grpc::Status DevicePlugin::list_and_watch(grpc::ServerCall& call) {
  uint64_t sent = 0;
  while (!call.cancelled() && !stop_.cancelled()) {
    bool send = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait_for(lk, std::chrono::milliseconds(200), [&] { return version_ != sent || stop_.cancelled(); });
      if (stop_.cancelled()) break;
      if (version_ != sent) {
        sent = version_;
        send = true;
      }
    }
    if (send && !call.send_message(dp::encode_list_and_watch(devices()))) break;
  }
  return grpc::Status::Ok();
}

void DevicePlugin::start_server() {
  auto srv = std::make_unique<grpc::Server>(socket_path());
  srv->add("/v1beta1.DevicePlugin/GetDevicePluginOptions", [](grpc::ServerCall& call) {
    call.send_message(dp::encode_options(false, true));
    return grpc::Status::Ok();
  });
  srv->add("/v1beta1.DevicePlugin/ListAndWatch", [this](grpc::ServerCall& call) { return list_and_watch(call); });
  srv->add("/v1beta1.DevicePlugin/GetPreferredAllocation", [this](grpc::ServerCall& call) {
    std::vector<std::vector<std::string>> resp;
    const std::vector<bool> fenced = this->fenced();
    for (auto q : dp::decode_preferred_request(call.request())) {
      // a fenced GPU is not offered (the kubelet's list may predate the fence)
      std::vector<std::string> avail;
      for (const auto& id : q.available) {
        auto it = std::find(ids_.begin(), ids_.end(), id);
        if (it == ids_.end() || !fenced[static_cast<size_t>(it - ids_.begin())]) avail.push_back(id);
      }
      if (static_cast<int32_t>(avail.size()) < q.size) avail = q.available;  // cannot satisfy otherwise
      resp.push_back(preferred_allocation(gpus_, ids_, avail, q.must_include, q.size));
    }
    call.send_message(dp::encode_preferred_response(resp));
    return grpc::Status::Ok();
  });
  srv->add("/v1beta1.DevicePlugin/Allocate", [this](grpc::ServerCall& call) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<dp::ContainerAllocation> resp;
    try {
      for (const auto& ids : dp::decode_allocate_request(call.request())) resp.push_back(allocate(ids));
    } catch (const std::invalid_argument& e) {
      return grpc::Status{grpc::kInvalidArgument, e.what()};
    }
    call.send_message(dp::encode_allocate_response(resp));
    allocations_.fetch_add(1);
    metrics::Registry::global()
        .histogram("device_plugin_allocate_duration_seconds", "kubelet Allocate RPC handling time")
        .observe(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    return grpc::Status::Ok();
  });
  srv->add("/v1beta1.DevicePlugin/PreStartContainer", [](grpc::ServerCall& call) {
    call.send_message("");
    return grpc::Status::Ok();
  });
  srv->start();
  std::lock_guard<std::mutex> lk(server_mu_);
  server_ = std::move(srv);
}

bool DevicePlugin::register_once() {
  const std::string kubelet = join_path(cfg_.plugin_dir, cfg_.kubelet_socket);
  dp::RegisterRequest r;
  r.version = dp::kVersion;
  r.endpoint = cfg_.socket_name;
  r.resource_name = cfg_.resource_name;
  r.pre_start_required = false;
  r.get_preferred_allocation_available = true;
  grpc::Channel ch(kubelet, 2000);
  std::string resp;
  grpc::Status st = ch.unary("/v1beta1.Registration/Register", dp::encode_register_request(r), &resp,
                             std::chrono::seconds(5));
  if (!st.ok()) {
    LOG_WARN("device_plugin") << "register " << cfg_.resource_name << " with " << kubelet << " failed: " << st.message
                              << " (code " << st.code << ")";
    return false;
  }
  registrations_.fetch_add(1);
  LOG_INFO("device_plugin") << "registered " << cfg_.resource_name << " (" << gpus_.size() << " devices) at "
                            << socket_path();
  return true;
}

void DevicePlugin::watch_loop() {
  const std::string kubelet = join_path(cfg_.plugin_dir, cfg_.kubelet_socket);
  do {
    try {
      bool present;
      {
        std::lock_guard<std::mutex> lk(server_mu_);
        present = server_ && server_->socket_present();
      }
      if (!present) {  // kubelet restart wiped the directory: serve again, then re-register
        LOG_WARN("device_plugin") << socket_path() << " disappeared; restarting the plugin server";
        std::unique_ptr<grpc::Server> old;
        {
          std::lock_guard<std::mutex> lk(server_mu_);
          old = std::move(server_);
        }
        if (old) old->stop();
        start_server();
        server_restarts_.fetch_add(1);
        registered_ = false;
      }
      if (cfg_.register_with_kubelet) {
        uint64_t ino = inode_of(kubelet);
        if (ino && ino != kubelet_inode_) {
          kubelet_inode_ = ino;
          registered_ = false;  // a new kubelet instance
        }
        if (!registered_ && ino) registered_ = register_once();
      }
    } catch (const std::exception& e) {
      LOG_ERROR("device_plugin") << "watch loop: " << e.what();
    }
  } while (!stop_.wait_for(std::chrono::milliseconds(cfg_.watch_interval_ms)));
}

void DevicePlugin::start() {
  // after a stop() (an advertiser conflict that has cleared) the plugin serves and registers anew
  stop_.reset();
  registered_ = false;
  kubelet_inode_ = 0;
  ::mkdir(cfg_.plugin_dir.c_str(), 0755);
  if (cfg_.cdi) LOG_INFO("device_plugin") << "CDI spec written to " << write_cdi_spec();
  start_server();
  watcher_ = std::thread([this] { watch_loop(); });
}

void DevicePlugin::stop() {
  stop_.cancel();
  cv_.notify_all();
  if (watcher_.joinable()) watcher_.join();
  std::unique_ptr<grpc::Server> srv;
  {
    std::lock_guard<std::mutex> lk(server_mu_);
    srv = std::move(server_);
  }
  if (srv) srv->stop();
}

json::Value DevicePlugin::describe() const {
  json::Value devs = json::Value::array();
  for (const auto& d : devices()) {
    devs.push_back(json::Value::object({{"id", d.id}, {"health", d.healthy ? dp::kHealthy : dp::kUnhealthy}}));
  }
  json::Value fenced = json::Value::array();
  {
    const std::vector<bool> f = this->fenced();
    for (size_t i = 0; i < f.size(); ++i)
      if (f[i]) fenced.push_back(ids_[i]);
  }
  return json::Value::object({{"resource", cfg_.resource_name},
                              {"socket", socket_path()},
                              {"registrations", static_cast<unsigned long long>(registrations_.load())},
                              {"server_restarts", static_cast<unsigned long long>(server_restarts_.load())},
                              {"allocations", static_cast<unsigned long long>(allocations_.load())},
                              {"refused_fenced", static_cast<unsigned long long>(refused_fenced_.load())},
                              {"devices", devs},
                              {"fenced", fenced}});
}

}  // namespace bgc::gpu

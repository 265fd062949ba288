// Kubelet device plugin for MI355X (`amd.com/gpu`), API k8s.io/kubelet deviceplugin/v1beta1.
//
// The reference never advertises GPUs itself — it only names `requests.nvidia.com/gpu`
// in the quotas it writes (reference src/synchronizer.rs:268) and leaves the device to
// an NVIDIA plugin.  SURVEY §2.6 N3 makes advertising each MI355X as a schedulable
// `amd.com/gpu` part of this build; the device plugin is how a kubelet actually hands a
// GPU to a container:
//
//   Registration  the plugin serves DevicePlugin on <dir>/<socket> and calls
//                 v1beta1.Registration/Register on <dir>/kubelet.sock.  A kubelet restart
//                 wipes the directory: the watcher notices the missing socket (or a new
//                 kubelet.sock inode), re-creates the server and registers again.
//   ListAndWatch  one Device per GPU, ID = PCI BDF, Healthy/Unhealthy from the telemetry
//                 side thread's health state machine, NUMA topology for the kubelet's
//                 topology manager; every health flip re-sends the list.
//   GetPreferredAllocation  xGMI-aware: an allocation of k GPUs is packed onto one
//                 xGMI hive (best fit, so big islands stay whole for TP=8 jobs), then onto
//                 one NUMA node, then by xGMI node id — RCCL rings then run over xGMI links.
//   Allocate      /dev/kfd plus each GPU's /dev/dri/card* and renderD*: the DRM minors
//                 amdsmi reports per logical device (so each compute partition gets its
//                 own render node), else resolved through sysfs from the BDF; ids that
//                 share a BDF with no known minor are refused rather than handed the
//                 parent's node.  Env/annotations name the GPUs and their hive.
//
// Transport: core/http2.h (h2c gRPC) + core/protobuf.h (wire format).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "core/cancel.h"
#include "core/http2.h"
#include "core/json.h"
#include "gpu/device.h"

namespace bgc::gpu {

namespace dp {

constexpr const char* kVersion = "v1beta1";
constexpr const char* kHealthy = "Healthy";
constexpr const char* kUnhealthy = "Unhealthy";

struct Device {
  std::string id;
  bool healthy = true;
  std::vector<int64_t> numa_nodes;
};

struct DeviceSpec {
  std::string container_path, host_path, permissions;
};

struct Mount {
  std::string container_path, host_path;
  bool read_only = false;
};

struct ContainerAllocation {
  std::map<std::string, std::string> envs;
  std::vector<Mount> mounts;
  std::vector<DeviceSpec> devices;
  std::map<std::string, std::string> annotations;
  std::vector<std::string> cdi_devices;  // fully qualified CDI names, e.g. amd.com/gpu=0000:05:00.0
};

struct PreferredRequest {
  std::vector<std::string> available, must_include;
  int32_t size = 0;
};

struct RegisterRequest {
  std::string version, endpoint, resource_name;
  bool pre_start_required = false;
  bool get_preferred_allocation_available = false;
};

// Wire codecs (message layouts from deviceplugin/v1beta1/api.proto).
std::string encode_options(bool pre_start_required, bool get_preferred_allocation_available);
std::string encode_register_request(const RegisterRequest& r);
RegisterRequest decode_register_request(std::string_view buf);
std::string encode_list_and_watch(const std::vector<Device>& devices);
std::vector<Device> decode_list_and_watch(std::string_view buf);
std::string encode_allocate_request(const std::vector<std::vector<std::string>>& containers);
std::vector<std::vector<std::string>> decode_allocate_request(std::string_view buf);
std::string encode_allocate_response(const std::vector<ContainerAllocation>& containers);
std::vector<ContainerAllocation> decode_allocate_response(std::string_view buf);
std::string encode_preferred_request(const std::vector<PreferredRequest>& reqs);
std::vector<PreferredRequest> decode_preferred_request(std::string_view buf);
std::string encode_preferred_response(const std::vector<std::vector<std::string>>& per_container);
std::vector<std::vector<std::string>> decode_preferred_response(std::string_view buf);

}  // namespace dp

struct DevicePluginConfig {
  std::string plugin_dir = "/var/lib/kubelet/device-plugins";
  std::string socket_name = "bgc-amd-gpu.sock";
  std::string kubelet_socket = "kubelet.sock";
  std::string resource_name = "amd.com/gpu";
  std::string dev_root = "/dev";    // host device nodes handed to containers
  std::string sysfs_root = "/sys";  // bus/pci/devices/<bdf>/drm/{card*,renderD*}
  int watch_interval_ms = 1000;
  bool register_with_kubelet = true;
  // Container Device Interface (k8s >= 1.28 with a CDI-enabled runtime): the plugin writes
  // a CDI spec for its devices into cdi_dir and Allocate answers with CDI device names
  // instead of raw device nodes; the runtime injects /dev/kfd and the DRM nodes.
  bool cdi = false;
  std::string cdi_dir = "/var/run/cdi";
};

// CDI spec (cdiVersion 0.6.0, kind = the resource name) for these devices: per device its
// render and card nodes, /dev/kfd as a spec-wide edit.  `ids[i]` names gpus[i].
json::Value cdi_spec(const std::string& kind, const std::vector<GpuInfo>& gpus, const std::vector<std::string>& ids,
                     const std::vector<std::pair<std::string, std::string>>& nodes);

// Kubelet pod-resources API (k8s.io/kubelet/pkg/apis/podresources/v1,
// PodResourcesLister/List): the device ids of `resource_name` currently assigned to
// containers.  Throws on transport errors.
std::set<std::string> allocated_device_ids(const std::string& socket, const std::string& resource_name);
// Wire codecs for the List response (unit-tested against grpcio/protobuf).
struct PodDevices {
  std::string pod, ns, container, resource;
  std::vector<std::string> ids;
};
std::vector<PodDevices> decode_pod_resources(std::string_view buf);
std::string encode_pod_resources(const std::vector<PodDevices>& v);

// Pure allocation policy (unit-tested): choose `size` ids from `available` (must include
// `must_include`) preferring one xGMI hive (best fit), then — when the amdsmi link map is
// known (GpuInfo::links) — the set with the most direct xGMI bandwidth between its
// members (greedy, seeded by must_include), else one NUMA node and adjacent xGMI node
// ids.  `ids[i]` is the device id of gpus[i].
std::vector<std::string> preferred_allocation(const std::vector<GpuInfo>& gpus, const std::vector<std::string>& ids,
                                              const std::vector<std::string>& available,
                                              const std::vector<std::string>& must_include, int size);

// Device ids a DevicePlugin advertises for `gpus` (PCI BDF; "-p<index>" for partitions
// sharing one, "gpu-<index>" without a BDF).
std::vector<std::string> device_ids_for(const std::vector<GpuInfo>& gpus);

// Coexistence with another advertiser of the same resource (an MI355X node commonly runs
// AMD's GPU Operator, whose device plugin registers amd.com/gpu too).  A foreign plugin
// is any live socket in `plugin_dir` other than the kubelet's and ours that answers
// v1beta1.DevicePlugin/ListAndWatch; it serves `resource` when one of its device ids is
// registered for `resource` in the kubelet's checkpoint (kubelet_internal_checkpoint,
// RegisteredDevices), or, without a readable checkpoint, when it lists one of our ids.
struct ForeignPlugin {
  std::string socket;              // file name in plugin_dir
  std::vector<std::string> ids;    // what its ListAndWatch listed
  bool via_checkpoint = false;     // matched through the kubelet checkpoint
};
std::vector<ForeignPlugin> foreign_plugins_for(const std::string& plugin_dir, const std::string& kubelet_socket,
                                               const std::string& own_socket, const std::string& resource,
                                               const std::vector<std::string>& own_ids, int timeout_ms = 2000);
// RegisteredDevices[resource] of the kubelet checkpoint in `plugin_dir` (empty set when the
// file is missing; `readable` says whether it parsed).
std::set<std::string> checkpoint_devices(const std::string& plugin_dir, const std::string& resource,
                                         bool* readable = nullptr);

class DevicePlugin {
 public:
  DevicePlugin(std::vector<GpuInfo> gpus, DevicePluginConfig cfg);
  ~DevicePlugin();
  void start();
  void stop();
  // Per-GPU health (same order as the gpus passed in); re-sends ListAndWatch on change.
  void set_health(const std::vector<bool>& healthy);
  // Diagnostics fence: a fenced GPU is listed Unhealthy, left out of preferred
  // allocations and refused by Allocate until it is unfenced, so the kubelet cannot hand
  // a tenant a GPU that is under a burn-in.  Re-sends ListAndWatch on change.
  void set_fenced(const std::vector<size_t>& which, bool fenced);
  std::vector<bool> fenced() const;
  // Per GPU: Allocate calls that handed it out (the fence re-checks these for an
  // allocation that raced the fence).
  std::vector<uint64_t> allocation_counts() const;
  // Throws std::invalid_argument on unknown or fenced ids.  Holds the plugin lock
  // throughout, so an allocation either completes before a fence or is refused by it.
  dp::ContainerAllocation allocate(const std::vector<std::string>& ids);
  // Writes the CDI spec (cdi mode); returns its path.
  std::string write_cdi_spec() const;
  std::vector<dp::Device> devices() const;
  const std::vector<std::string>& ids() const { return ids_; }
  std::string socket_path() const;
  uint64_t registrations() const { return registrations_.load(); }
  uint64_t server_restarts() const { return server_restarts_.load(); }
  json::Value describe() const;

 private:
  void start_server();
  bool register_once();
  // card* / renderD* node names of gpus_[i] (throws for a partition with no known render node)
  std::pair<std::string, std::string> drm_node_names(size_t i) const;
  void watch_loop();
  grpc::Status list_and_watch(grpc::ServerCall& call);

  std::vector<GpuInfo> gpus_;
  std::vector<std::string> ids_;
  std::vector<bool> shared_bdf_;  // logical devices (partitions) sharing a PCI function
  DevicePluginConfig cfg_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::vector<bool> healthy_;
  std::vector<bool> fenced_;
  std::vector<uint64_t> alloc_counts_;
  uint64_t version_ = 1;
  std::unique_ptr<grpc::Server> server_;
  std::mutex server_mu_;
  CancelToken stop_;
  std::thread watcher_;
  uint64_t kubelet_inode_ = 0;
  bool registered_ = false;
  std::atomic<uint64_t> registrations_{0};
  std::atomic<uint64_t> server_restarts_{0};
  std::atomic<uint64_t> allocations_{0};
  std::atomic<uint64_t> refused_fenced_{0};
};

}  // namespace bgc::gpu

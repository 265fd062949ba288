"""Fake kubelet for device-plugin tests, built on python grpcio + protobuf.

The v1beta1 device-plugin messages (k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto)
are declared here with descriptor_pb2 — no protoc in the image — so the tests exercise
the native plugin against an independent gRPC/HTTP2/protobuf implementation, the same
way a real kubelet (grpc-go) would.

FakeKubelet:
  * serves v1beta1.Registration/Register on <dir>/kubelet.sock and records requests;
  * after a registration, dials the plugin's endpoint like the kubelet does and keeps a
    ListAndWatch stream open, recording every device list it receives;
  * restart() mimics a kubelet restart: stops, wipes the plugin directory (the real
    kubelet deletes every socket there), and serves a fresh kubelet.sock.
"""
import json
import os
import threading
import time
from concurrent import futures

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto
_PKG = "v1beta1"


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="bgc_deviceplugin_v1beta1.proto", package=_PKG, syntax="proto3")

    def msg(name, *fields, map_entry=False):
        m = fd.message_type.add(name=name)
        if map_entry:
            m.options.map_entry = True
        for num, fname, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m

    opt, rep = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    S, B, I64, I32, M = _F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT64, _F.TYPE_INT32, _F.TYPE_MESSAGE
    msg("DevicePluginOptions", (1, "pre_start_required", B, opt, None),
        (2, "get_preferred_allocation_available", B, opt, None))
    msg("RegisterRequest", (1, "version", S, opt, None), (2, "endpoint", S, opt, None),
        (3, "resource_name", S, opt, None), (4, "options", M, opt, f".{_PKG}.DevicePluginOptions"))
    msg("Empty")
    msg("NUMANode", (1, "ID", I64, opt, None))
    msg("TopologyInfo", (1, "nodes", M, rep, f".{_PKG}.NUMANode"))
    msg("Device", (1, "ID", S, opt, None), (2, "health", S, opt, None),
        (3, "topology", M, opt, f".{_PKG}.TopologyInfo"))
    msg("ListAndWatchResponse", (1, "devices", M, rep, f".{_PKG}.Device"))
    msg("PreStartContainerRequest", (1, "devices_ids", S, rep, None))
    msg("PreStartContainerResponse")
    msg("ContainerPreferredAllocationRequest", (1, "available_deviceIDs", S, rep, None),
        (2, "must_include_deviceIDs", S, rep, None), (3, "allocation_size", I32, opt, None))
    msg("PreferredAllocationRequest", (1, "container_requests", M, rep, f".{_PKG}.ContainerPreferredAllocationRequest"))
    msg("ContainerPreferredAllocationResponse", (1, "deviceIDs", S, rep, None))
    msg("PreferredAllocationResponse",
        (1, "container_responses", M, rep, f".{_PKG}.ContainerPreferredAllocationResponse"))
    msg("ContainerAllocateRequest", (1, "devices_ids", S, rep, None))
    msg("AllocateRequest", (1, "container_requests", M, rep, f".{_PKG}.ContainerAllocateRequest"))
    msg("Mount", (1, "container_path", S, opt, None), (2, "host_path", S, opt, None), (3, "read_only", B, opt, None))
    msg("DeviceSpec", (1, "container_path", S, opt, None), (2, "host_path", S, opt, None),
        (3, "permissions", S, opt, None))
    msg("CDIDevice", (1, "name", S, opt, None))
    car = msg("ContainerAllocateResponse",
              (1, "envs", M, rep, f".{_PKG}.ContainerAllocateResponse.EnvsEntry"),
              (2, "mounts", M, rep, f".{_PKG}.Mount"), (3, "devices", M, rep, f".{_PKG}.DeviceSpec"),
              (4, "annotations", M, rep, f".{_PKG}.ContainerAllocateResponse.AnnotationsEntry"),
              (5, "cdi_devices", M, rep, f".{_PKG}.CDIDevice"))
    for entry in ("EnvsEntry", "AnnotationsEntry"):
        e = car.nested_type.add(name=entry)
        e.options.map_entry = True
        e.field.add(name="key", number=1, type=S, label=opt)
        e.field.add(name="value", number=2, type=S, label=opt)
    msg("AllocateResponse", (1, "container_responses", M, rep, f".{_PKG}.ContainerAllocateResponse"))
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return {m.name: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{_PKG}.{m.name}"))
            for m in fd.message_type}


pb = _build()


def _unary(channel, name, req_cls, resp_cls):
    return channel.unary_unary(name, request_serializer=req_cls.SerializeToString,
                               response_deserializer=resp_cls.FromString)


class PluginClient:
    """kubelet -> plugin calls over the plugin's unix socket (grpcio client)."""

    def __init__(self, socket_path):
        self.channel = grpc.insecure_channel("unix://" + socket_path)
        self.options = _unary(self.channel, "/v1beta1.DevicePlugin/GetDevicePluginOptions", pb["Empty"],
                              pb["DevicePluginOptions"])
        self.allocate = _unary(self.channel, "/v1beta1.DevicePlugin/Allocate", pb["AllocateRequest"],
                               pb["AllocateResponse"])
        self.preferred = _unary(self.channel, "/v1beta1.DevicePlugin/GetPreferredAllocation",
                                pb["PreferredAllocationRequest"], pb["PreferredAllocationResponse"])
        self.prestart = _unary(self.channel, "/v1beta1.DevicePlugin/PreStartContainer",
                               pb["PreStartContainerRequest"], pb["PreStartContainerResponse"])
        self.list_and_watch = self.channel.unary_stream(
            "/v1beta1.DevicePlugin/ListAndWatch", request_serializer=pb["Empty"].SerializeToString,
            response_deserializer=pb["ListAndWatchResponse"].FromString)

    def close(self):
        self.channel.close()


class FakeKubelet:
    def __init__(self, plugin_dir):
        self.dir = plugin_dir
        self.registrations = []
        self.device_lists = []  # [(endpoint, [(id, health, [numa...])...])]
        self.cv = threading.Condition()
        self.server = None
        self._watchers = []
        self._stopping = False
        self.registered_devices = {}  # resource -> device ids (the kubelet checkpoint's RegisteredDevices)

    def _write_checkpoint(self):
        """The kubelet's device-manager checkpoint (<dir>/kubelet_internal_checkpoint), which
        records the device ids each registered resource listed."""
        doc = {"Data": {"PodDeviceEntries": None, "RegisteredDevices": self.registered_devices}, "Checksum": 0}
        tmp = os.path.join(self.dir, ".checkpoint.tmp")
        with open(tmp, "w") as f:
            json.dump(doc, f)
        os.replace(tmp, os.path.join(self.dir, "kubelet_internal_checkpoint"))

    # -- Registration service
    def _register(self, req, ctx):
        with self.cv:
            self.registrations.append(req)
            self.cv.notify_all()
        t = threading.Thread(target=self._watch_plugin, args=(req.endpoint,), daemon=True)
        t.start()
        self._watchers.append(t)
        return pb["Empty"]()

    def _watch_plugin(self, endpoint):
        # like kubelet's endpoint.run(): ListAndWatch until the stream breaks
        client = PluginClient(os.path.join(self.dir, endpoint))
        try:
            for resp in client.list_and_watch(pb["Empty"]()):
                devs = [(d.ID, d.health, [n.ID for n in d.topology.nodes]) for d in resp.devices]
                with self.cv:
                    self.device_lists.append((endpoint, devs))
                    resource = next((r.resource_name for r in reversed(self.registrations) if r.endpoint == endpoint),
                                    None)
                    if resource:
                        self.registered_devices[resource] = [d[0] for d in devs]
                        self._write_checkpoint()
                    self.cv.notify_all()
                if self._stopping:
                    break
        except grpc.RpcError:
            pass
        finally:
            client.close()

    def start(self):
        os.makedirs(self.dir, exist_ok=True)
        self._stopping = False
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        handler = grpc.method_handlers_generic_handler("v1beta1.Registration", {
            "Register": grpc.unary_unary_rpc_method_handler(
                self._register, request_deserializer=pb["RegisterRequest"].FromString,
                response_serializer=pb["Empty"].SerializeToString)})
        self.server.add_generic_rpc_handlers((handler,))
        self.server.add_insecure_port("unix://" + os.path.join(self.dir, "kubelet.sock"))
        self.server.start()
        return self

    def stop(self):
        self._stopping = True
        if self.server is not None:
            self.server.stop(grace=None)
            self.server = None

    def restart(self):
        """Kubelet restart: the device-plugin directory is wiped and kubelet.sock re-created."""
        self.stop()
        for name in os.listdir(self.dir):
            try:
                os.unlink(os.path.join(self.dir, name))
            except OSError:
                pass
        time.sleep(0.05)
        return self.start()

    def wait(self, pred, timeout=10.0):
        deadline = time.time() + timeout
        with self.cv:
            while not pred():
                left = deadline - time.time()
                if left <= 0:
                    return False
                self.cv.wait(left)
        return True


class FakeDevicePlugin:
    """Another vendor's device plugin (e.g. the GPU Operator's): serves ListAndWatch and
    GetDevicePluginOptions on <dir>/<socket> with fixed device ids, and registers
    `resource` with the kubelet when asked to."""

    def __init__(self, plugin_dir, socket_name, device_ids):
        self.dir, self.socket, self.ids = plugin_dir, socket_name, list(device_ids)
        self.server = None
        self._stop = threading.Event()

    def _list_and_watch(self, req, ctx):
        resp = pb["ListAndWatchResponse"]()
        for i in self.ids:
            resp.devices.add(ID=i, health="Healthy")
        yield resp
        while not self._stop.is_set() and ctx.is_active():
            self._stop.wait(0.2)

    def _options(self, req, ctx):
        return pb["DevicePluginOptions"]()

    def start(self):
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        handler = grpc.method_handlers_generic_handler("v1beta1.DevicePlugin", {
            "ListAndWatch": grpc.unary_stream_rpc_method_handler(
                self._list_and_watch, request_deserializer=pb["Empty"].FromString,
                response_serializer=pb["ListAndWatchResponse"].SerializeToString),
            "GetDevicePluginOptions": grpc.unary_unary_rpc_method_handler(
                self._options, request_deserializer=pb["Empty"].FromString,
                response_serializer=pb["DevicePluginOptions"].SerializeToString)})
        self.server.add_generic_rpc_handlers((handler,))
        self.server.add_insecure_port("unix://" + os.path.join(self.dir, self.socket))
        self.server.start()
        return self

    def register(self, resource):
        ch = grpc.insecure_channel("unix://" + os.path.join(self.dir, "kubelet.sock"))
        try:
            reg = _unary(ch, "/v1beta1.Registration/Register", pb["RegisterRequest"], pb["Empty"])
            reg(pb["RegisterRequest"](version="v1beta1", endpoint=self.socket, resource_name=resource), timeout=5)
        finally:
            ch.close()

    def stop(self):
        self._stop.set()
        if self.server is not None:
            self.server.stop(grace=None)
            self.server = None
        try:
            os.unlink(os.path.join(self.dir, self.socket))
        except OSError:
            pass


def _build_podresources():
    """k8s.io/kubelet/pkg/apis/podresources/v1 (List only)."""
    fd = descriptor_pb2.FileDescriptorProto(name="bgc_podresources_v1.proto", package="v1", syntax="proto3")
    opt, rep = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    S, I64, M = _F.TYPE_STRING, _F.TYPE_INT64, _F.TYPE_MESSAGE

    def msg(name, *fields):
        m = fd.message_type.add(name=name)
        for num, fname, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname

    msg("ListPodResourcesRequest")
    msg("NUMANode", (1, "ID", I64, opt, None))
    msg("TopologyInfo", (1, "nodes", M, rep, ".v1.NUMANode"))
    msg("ContainerDevices", (1, "resource_name", S, opt, None), (2, "device_ids", S, rep, None),
        (3, "topology", M, opt, ".v1.TopologyInfo"))
    msg("ContainerResources", (1, "name", S, opt, None), (2, "devices", M, rep, ".v1.ContainerDevices"),
        (3, "cpu_ids", I64, rep, None))
    msg("PodResources", (1, "name", S, opt, None), (2, "namespace", S, opt, None),
        (3, "containers", M, rep, ".v1.ContainerResources"))
    msg("ListPodResourcesResponse", (1, "pod_resources", M, rep, ".v1.PodResources"))
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return {m.name: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"v1.{m.name}"))
            for m in fd.message_type}


podres_pb = _build_podresources()


class FakePodResources:
    """The kubelet's pod-resources endpoint (v1.PodResourcesLister/List) on a unix socket.
    `assign(pod, resource, ids)` sets what a pod's container holds; `lists` counts calls."""

    def __init__(self, socket_path):
        self.path = socket_path
        self.pods = {}  # pod -> (resource, [ids])
        self.lists = 0
        self.server = None

    def assign(self, pod, resource, ids):
        self.pods[pod] = (resource, list(ids))

    def release(self, pod):
        self.pods.pop(pod, None)

    def _list(self, req, ctx):
        self.lists += 1
        r = podres_pb["ListPodResourcesResponse"]()
        for pod, (res, ids) in sorted(self.pods.items()):
            p = r.pod_resources.add(name=pod, namespace="default")
            c = p.containers.add(name="main")
            c.devices.add(resource_name=res, device_ids=ids)
        return r

    def start(self):
        os.makedirs(os.path.dirname(self.path), exist_ok=True)
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        handler = grpc.method_handlers_generic_handler("v1.PodResourcesLister", {
            "List": grpc.unary_unary_rpc_method_handler(
                self._list, request_deserializer=podres_pb["ListPodResourcesRequest"].FromString,
                response_serializer=podres_pb["ListPodResourcesResponse"].SerializeToString)})
        self.server.add_generic_rpc_handlers((handler,))
        self.server.add_insecure_port("unix://" + self.path)
        self.server.start()
        return self

    def stop(self):
        if self.server is not None:
            self.server.stop(grace=None)
            self.server = None

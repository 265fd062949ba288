"""Native kubelet device plugin (native/gpu/device_plugin.cc over core/http2.cc) against a
fake kubelet written with python grpcio — an independent HTTP/2 + gRPC + protobuf stack,
as grpc-go is in a real kubelet.

Covers: registration, ListAndWatch (initial list, health flips), Allocate (device nodes
from sysfs, envs), GetPreferredAllocation (xGMI packing), errors as gRPC statuses, kubelet
restart (directory wipe -> re-serve + re-register), concurrent calls, responses larger
than the peer's flow-control window, and the node agent running the plugin."""
import json
import os
import threading
import time

import grpc
import pytest

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for
from bacchus_gpu_controller_amd.testing.kubelet import FakeKubelet, PluginClient, pb

pytestmark = pytest.mark.slow


@pytest.fixture
def plugin_env(nat, tmp_path):
    d = str(tmp_path / "dp")
    os.makedirs(d)
    kubelet = FakeKubelet(d).start()
    fixture = nat.default_mi355x_fixture(8)
    plugin = nat.DevicePlugin(fixture, {"plugin_dir": d, "watch_interval_ms": "50",
                                        "sysfs_root": str(tmp_path / "sys"), "dev_root": "/dev"})
    yield kubelet, plugin, json.loads(fixture)["gpus"]
    plugin.stop()
    kubelet.stop()


def test_register_list_allocate(plugin_env, tmp_path):
    kubelet, plugin, gpus = plugin_env
    # sysfs for gpu 2: the plugin must hand out *these* DRM nodes, not index-derived ones
    drm = tmp_path / "sys" / "bus" / "pci" / "devices" / gpus[2]["bdf"] / "drm"
    os.makedirs(drm / "card7")
    os.makedirs(drm / "renderD135")
    plugin.start()
    assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists)
    reg = kubelet.registrations[0]
    assert (reg.version, reg.endpoint, reg.resource_name) == ("v1beta1", "bgc-amd-gpu.sock", "amd.com/gpu")
    assert reg.options.get_preferred_allocation_available and not reg.options.pre_start_required
    endpoint, devs = kubelet.device_lists[-1]
    assert [d[0] for d in devs] == [g["bdf"] for g in gpus]
    assert all(d[1] == "Healthy" for d in devs)
    assert [d[2] for d in devs] == [[g["numa_node"]] for g in gpus]

    c = PluginClient(plugin.socket_path)
    try:
        opts = c.options(pb["Empty"](), timeout=5)
        assert opts.get_preferred_allocation_available and not opts.pre_start_required
        req = pb["AllocateRequest"]()
        req.container_requests.add().devices_ids.extend([gpus[0]["bdf"], gpus[2]["bdf"]])
        req.container_requests.add().devices_ids.extend([gpus[5]["bdf"]])
        resp = c.allocate(req, timeout=5)
        assert len(resp.container_responses) == 2
        r0 = resp.container_responses[0]
        paths = [(d.container_path, d.host_path, d.permissions) for d in r0.devices]
        assert paths[0] == ("/dev/kfd", "/dev/kfd", "rw")
        assert ("/dev/dri/card7", "/dev/dri/card7", "rw") in paths
        assert ("/dev/dri/renderD135", "/dev/dri/renderD135", "rw") in paths
        assert ("/dev/dri/renderD128", "/dev/dri/renderD128", "rw") in paths  # no sysfs entry: index-derived
        assert r0.envs["BGC_AMD_GPU_IDS"] == f"{gpus[0]['bdf']},{gpus[2]['bdf']}"
        assert r0.envs["BGC_AMD_GPU_SINGLE_XGMI_HIVE"] == "true"
        assert r0.envs["BGC_AMD_GPU_XGMI_HIVES"] == gpus[0]["xgmi_hive_id"]

        q = pb["PreferredAllocationRequest"]()
        cq = q.container_requests.add()
        cq.available_deviceIDs.extend([g["bdf"] for g in gpus])
        cq.must_include_deviceIDs.append(gpus[6]["bdf"])
        cq.allocation_size = 4
        pref = c.preferred(q, timeout=5).container_responses[0].deviceIDs
        assert pref[0] == gpus[6]["bdf"] and set(pref) == {g["bdf"] for g in gpus[4:8]}  # NUMA 1 quad

        c.prestart(pb["PreStartContainerRequest"](devices_ids=[gpus[0]["bdf"]]), timeout=5)

        bad = pb["AllocateRequest"]()
        bad.container_requests.add().devices_ids.append("0000:ff:00.0")
        with pytest.raises(grpc.RpcError) as ei:
            c.allocate(bad, timeout=5)
        assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        assert "0000:ff:00.0" in ei.value.details()
    finally:
        c.close()


def test_health_flip_resends_list(plugin_env):
    kubelet, plugin, gpus = plugin_env
    plugin.start()
    assert kubelet.wait(lambda: kubelet.device_lists)
    n0 = len(kubelet.device_lists)
    plugin.set_health([i != 3 for i in range(8)])
    assert kubelet.wait(lambda: len(kubelet.device_lists) > n0)
    devs = kubelet.device_lists[-1][1]
    assert [d[1] for d in devs] == ["Healthy"] * 3 + ["Unhealthy"] + ["Healthy"] * 4
    plugin.set_health([True] * 8)
    assert kubelet.wait(lambda: all(d[1] == "Healthy" for d in kubelet.device_lists[-1][1]))


def test_kubelet_restart_reregisters(plugin_env):
    kubelet, plugin, gpus = plugin_env
    plugin.start()
    assert kubelet.wait(lambda: len(kubelet.registrations) == 1)
    wait_for(lambda: plugin.registrations == 1, timeout=10, desc="first registration acknowledged")
    kubelet.restart()  # wipes the directory, including the plugin's socket
    assert kubelet.wait(lambda: len(kubelet.registrations) >= 2, timeout=15)
    wait_for(lambda: plugin.registrations >= 2, timeout=10, desc="plugin saw its re-registration succeed")
    assert plugin.server_restarts >= 1
    n = len(kubelet.device_lists)
    assert kubelet.wait(lambda: len(kubelet.device_lists) > n or n > 0)
    assert os.path.exists(plugin.socket_path)


def test_registration_retries_until_kubelet_appears(nat, tmp_path):
    d = str(tmp_path / "dp")
    os.makedirs(d)
    plugin = nat.DevicePlugin(nat.default_mi355x_fixture(2), {"plugin_dir": d, "watch_interval_ms": "50"})
    plugin.start()
    try:
        time.sleep(0.3)
        assert plugin.registrations == 0
        kubelet = FakeKubelet(d).start()
        try:
            assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists)
            assert len(kubelet.device_lists[-1][1]) == 2
        finally:
            kubelet.stop()
    finally:
        plugin.stop()


def test_concurrent_calls_and_large_responses(plugin_env, nat):
    kubelet, plugin, gpus = plugin_env
    plugin.start()
    ids = [g["bdf"] for g in gpus]
    errors = []

    def worker(k):
        c = PluginClient(plugin.socket_path)
        try:
            for i in range(40):
                req = pb["AllocateRequest"]()
                req.container_requests.add().devices_ids.append(ids[(k + i) % 8])
                r = c.allocate(req, timeout=10)
                assert r.container_responses[0].envs["BGC_AMD_GPU_IDS"] == ids[(k + i) % 8]
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
        finally:
            c.close()

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errors, errors[:3]

    # ~500 KB response: far beyond the 64 KiB default window, so our sender must honour
    # the peer's WINDOW_UPDATEs (unknown ids are allowed in `available` and fill the tail)
    many = [f"extra-device-{i:06d}" for i in range(30000)]
    q = pb["PreferredAllocationRequest"]()
    cq = q.container_requests.add()
    cq.available_deviceIDs.extend(ids + many)
    cq.allocation_size = len(ids) + len(many)
    c = PluginClient(plugin.socket_path)
    try:
        got = list(c.preferred(q, timeout=20).container_responses[0].deviceIDs)
    finally:
        c.close()
    assert len(got) == 30008 and set(got[:8]) == set(ids) and got[8:] == many


def test_native_channel_against_grpcio_server(nat, tmp_path):
    """Our gRPC client (used for Registration) against grpcio's server: unary, server
    streaming with many messages, status propagation, deadline."""
    from concurrent import futures

    sock = str(tmp_path / "echo.sock")
    srv = grpc.server(futures.ThreadPoolExecutor(max_workers=4))

    def echo(req, ctx):
        return req

    def fail(req, ctx):
        ctx.abort(grpc.StatusCode.FAILED_PRECONDITION, "nope: ünïcode")

    def stream(req, ctx):
        for i in range(int(req)):
            yield f"msg-{i}".encode() * 100

    def slow(req, ctx):
        time.sleep(2)
        return req

    ident = (lambda b: b)
    srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler("t.S", {
        "Echo": grpc.unary_unary_rpc_method_handler(echo, ident, ident),
        "Fail": grpc.unary_unary_rpc_method_handler(fail, ident, ident),
        "Slow": grpc.unary_unary_rpc_method_handler(slow, ident, ident),
        "Stream": grpc.unary_stream_rpc_method_handler(stream, ident, ident)}),))
    srv.add_insecure_port("unix://" + sock)
    srv.start()
    try:
        ch = nat.GrpcChannel(sock)
        code, msg, body = ch.unary("/t.S/Echo", b"x" * 200000)
        assert (code, msg) == (0, "") and body == b"x" * 200000
        code, msg, _ = ch.unary("/t.S/Fail", b"")
        assert code == 9 and msg == "nope: ünïcode"
        code, msg, msgs = ch.server_stream("/t.S/Stream", b"500")
        assert code == 0 and len(msgs) == 500 and msgs[499] == b"msg-499" * 100
        code, msg, _ = ch.unary("/t.S/Missing", b"")
        assert code == 12
        code, msg, _ = ch.unary("/t.S/Slow", b"", timeout_ms=200)
        assert code == 4
        code, msg, body = ch.unary("/t.S/Echo", b"still-usable")
        assert code == 0 and body == b"still-usable"
        ch.close()
    finally:
        srv.stop(None)


def test_node_agent_runs_device_plugin(tmp_path):
    """CONF_DEVICE_PLUGIN=true: the kubelet gets amd.com/gpu through the plugin, so the
    node agent leaves capacity/allocatable to it and keeps labels + condition; a GPU flap
    reaches the kubelet as an Unhealthy device."""
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    try:
        with Cluster(admission=False, controller=False) as c:
            c.start_node_agent(node_name="mi355x-dp", backend="mock", poll_interval_ms=50,
                               extra_env={"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d,
                                          "CONF_HEARTBEAT_SECS": "1"})
            assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists, timeout=15)
            assert len(kubelet.device_lists[-1][1]) == 8
            node = wait_for(lambda: (lambda n: n if n and n.get("status", {}).get("conditions") else None)(
                c.admin.get_or_none("nodes", "mi355x-dp")), timeout=10, desc="node condition published")
            assert "amd.com/gpu" not in node["status"].get("capacity", {})
            assert node["metadata"]["labels"]["amd.com/gpu.count"] == "8"
            fx = json.loads(open(c.fixtures["mi355x-dp"]).read())
            fx["gpus"][5]["telemetry"]["temp_hotspot_c"] = 125
            c.set_gpu_fixture("mi355x-dp", fx)
            assert kubelet.wait(lambda: kubelet.device_lists[-1][1][5][1] == "Unhealthy", timeout=15)
            assert sum(x[1] == "Healthy" for x in kubelet.device_lists[-1][1]) == 7
            # concurrent kubelet calls into the node agent's own server (this path runs
            # under tools/sanitize.sh asan|tsan, unlike the pybind-hosted plugin above)
            ids = [x[0] for x in kubelet.device_lists[-1][1]]
            sock = os.path.join(d, kubelet.registrations[-1].endpoint)
            errors = []

            def worker(k):
                cl = PluginClient(sock)
                try:
                    for i in range(25):
                        req = pb["AllocateRequest"]()
                        req.container_requests.add().devices_ids.append(ids[(k + i) % 8])
                        assert cl.allocate(req, timeout=10).container_responses[0].devices
                        q = pb["PreferredAllocationRequest"]()
                        cq = q.container_requests.add()
                        cq.available_deviceIDs.extend(ids)
                        cq.allocation_size = 1 + (k + i) % 8
                        assert len(cl.preferred(q, timeout=10).container_responses[0].deviceIDs) == 1 + (k + i) % 8
                except Exception as e:  # noqa: BLE001
                    errors.append(repr(e))
                finally:
                    cl.close()

            ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
            for t in ts:
                t.start()
            for t in ts:
                t.join(60)
            assert not errors, errors[:3]
    finally:
        kubelet.stop()


def test_compute_partitions_advertised_as_partition_resource(nat, tmp_path):
    """GPUs in a sub-device compute partition (here CPX, two logical devices per BDF) are
    advertised as amd.com/gpu-partition — the quota key the synchronizer writes for the
    sheet's partition column — with unique device IDs."""
    fx = json.loads(nat.default_mi355x_fixture(8))
    for i, g in enumerate(fx["gpus"]):
        g["compute_partition"] = "CPX"
        g["bdf"] = fx["gpus"][i - i % 2]["bdf"]  # partitions 2k, 2k+1 share a PCI function
    fixture = str(tmp_path / "cpx.json")
    with open(fixture, "w") as f:
        json.dump(fx, f)
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    try:
        with Cluster(admission=False, controller=False) as c:
            c.start_node_agent(node_name="mi355x-cpx", backend="mock", proc_name="na-cpx",
                               extra_env={"CONF_MOCK_FIXTURE_PATH": fixture})
            node = wait_for(lambda: (lambda n: n if n and n.get("status", {}).get("capacity") else None)(
                c.admin.get_or_none("nodes", "mi355x-cpx")), timeout=10, desc="capacity published")
            assert node["status"]["capacity"] == {"amd.com/gpu-partition": "8"}
            c.procs["na-cpx"].stop()
            c.start_node_agent(node_name="mi355x-cpx2", backend="mock", proc_name="na-cpx2",
                               extra_env={"CONF_MOCK_FIXTURE_PATH": fixture, "CONF_DEVICE_PLUGIN": "true",
                                          "CONF_DEVICE_PLUGIN_DIR": d})
            assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists, timeout=15)
            assert kubelet.registrations[-1].resource_name == "amd.com/gpu-partition"
            ids = [x[0] for x in kubelet.device_lists[-1][1]]
            assert len(ids) == 8 and len(set(ids)) == 8
            assert ids[0] == fx["gpus"][0]["bdf"] + "-p0" and ids[1] == fx["gpus"][0]["bdf"] + "-p1"
    finally:
        kubelet.stop()


def test_pod_resources_client_against_grpcio(nat, tmp_path):
    from bacchus_gpu_controller_amd.testing.kubelet import FakePodResources

    pr = FakePodResources(str(tmp_path / "pod-resources" / "kubelet.sock")).start()
    try:
        pr.assign("train-0", "amd.com/gpu", ["0000:05:00.0", "0000:15:00.0"])
        pr.assign("other", "example.com/nic", ["eth0"])
        assert nat.allocated_device_ids(pr.path, "amd.com/gpu") == {"0000:05:00.0", "0000:15:00.0"}
        pr.release("train-0")
        assert nat.allocated_device_ids(pr.path, "amd.com/gpu") == set()
        assert pr.lists == 2
    finally:
        pr.stop()


def test_periodic_diagnostics_skip_gpus_in_use(tmp_path):
    """CONF_RUN_DIAG with CONF_DIAG_INTERVAL_SECS: the agent re-runs the HIP diagnostics on
    GPUs no container holds — GPU 0 is held per the kubelet's pod-resources API, GPU 1 has a
    compute process per amdsmi — and a failed diagnosis drives ListAndWatch and the
    healthy-count label.  (On a host without a GPU every diagnosis fails loudly, which is
    exactly what this test relies on; tests/gpu covers the passing path.)"""
    from bacchus_gpu_controller_amd.testing.kubelet import FakePodResources

    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    pr = FakePodResources(str(tmp_path / "pod-resources" / "kubelet.sock")).start()
    try:
        with Cluster(admission=False, controller=False) as c:
            fx_path = None
            c.start_node_agent(node_name="mi355x-diag", backend="mock", n_mock_gpus=4, poll_interval_ms=50,
                               extra_env={"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d,
                                          "CONF_RUN_DIAG": "true", "CONF_DIAG_INTERVAL_SECS": "1",
                                          "CONF_DIAG_HBM_BYTES": str(64 << 20), "CONF_DIAG_FENCE_SETTLE_MS": "200",
                                          "CONF_POD_RESOURCES_SOCKET": pr.path, "CONF_HEARTBEAT_SECS": "1"})
            fx_path = c.fixtures["mi355x-diag"]
            fx = json.loads(open(fx_path).read())
            fx["gpus"][1]["telemetry"]["busy_processes"] = 2
            c.set_gpu_fixture("mi355x-diag", fx)
            assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists, timeout=15)
            ids = [x[0] for x in kubelet.device_lists[-1][1]]
            pr.assign("train-0", "amd.com/gpu", [ids[0]])
            import requests

            port = c.node_agent_ports["mi355x-diag"]
            desc = wait_for(lambda: (lambda g: g if g["diag_runs"] >= 3 and g["diag_skipped_in_use"] >= 2 else None)(
                requests.get(f"http://127.0.0.1:{port}/gpus", timeout=5).json()), timeout=30, desc="periodic diag runs")
            assert pr.lists >= 1
            assert all(not r["passed"] and r["failures"] for r in desc["diag"])
            assert kubelet.wait(lambda: all(x[1] == "Unhealthy" for x in kubelet.device_lists[-1][1]), timeout=10)
            node = c.admin.get_or_none("nodes", "mi355x-diag")
            assert node["metadata"]["labels"]["amd.com/gpu.diag"] == "failed"
            assert node["metadata"]["labels"]["amd.com/gpu.healthy-count"] == "0"
    finally:
        pr.stop()
        kubelet.stop()


def test_cdi_mode_spec_and_allocate(nat, tmp_path):
    """CDI mode: the plugin writes a CDI spec (cdiVersion 0.6.0, kind amd.com/gpu, one
    device per BDF with its DRM nodes, /dev/kfd spec-wide) and Allocate answers with CDI
    names that a CDI-enabled runtime resolves; decoded by the independent grpcio stack."""
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    gpus = json.loads(nat.default_mi355x_fixture(4))["gpus"]
    drm = tmp_path / "sys" / "bus" / "pci" / "devices" / gpus[1]["bdf"] / "drm"
    os.makedirs(drm / "card9")
    os.makedirs(drm / "renderD140")
    plugin = nat.DevicePlugin(json.dumps(gpus), {"plugin_dir": d, "watch_interval_ms": "50", "cdi": "true",
                                                 "cdi_dir": str(tmp_path / "cdi"), "sysfs_root": str(tmp_path / "sys")})
    plugin.start()
    try:
        spec = json.load(open(tmp_path / "cdi" / "bgc-amd.com-gpu.json"))
        assert spec["cdiVersion"] == "0.6.0" and spec["kind"] == "amd.com/gpu"
        assert spec["containerEdits"]["deviceNodes"] == [{"path": "/dev/kfd"}]
        byname = {x["name"]: [n["path"] for n in x["containerEdits"]["deviceNodes"]] for x in spec["devices"]}
        assert byname[gpus[1]["bdf"]] == ["/dev/dri/card9", "/dev/dri/renderD140"]
        assert byname[gpus[0]["bdf"]] == ["/dev/dri/card1", "/dev/dri/renderD128"]  # amdsmi minors
        assert kubelet.wait(lambda: kubelet.registrations and kubelet.device_lists, timeout=15)
        c = PluginClient(plugin.socket_path)
        try:
            req = pb["AllocateRequest"]()
            req.container_requests.add().devices_ids.extend([gpus[1]["bdf"], gpus[3]["bdf"]])
            r = c.allocate(req, timeout=5).container_responses[0]
        finally:
            c.close()
        assert [x.name for x in r.cdi_devices] == [f"amd.com/gpu={gpus[1]['bdf']}", f"amd.com/gpu={gpus[3]['bdf']}"]
        assert len(r.devices) == 0 and r.envs["BGC_AMD_GPU_SINGLE_XGMI_HIVE"] == "true"
    finally:
        plugin.stop()
        kubelet.stop()


def test_each_health_rule_flips_list_and_watch(tmp_path):
    """every health rule, driven through the node agent's telemetry side
    thread (mock amdsmi fixture edited while it runs), turns that GPU Unhealthy in the
    kubelet's ListAndWatch stream and names the reason in /gpus."""
    import requests

    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    env = {"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d, "CONF_HEARTBEAT_SECS": "30",
           "CONF_SLOW_EVERY": "1", "CONF_RAS_EVERY": "1", "CONF_VIOLATION_SUSTAIN_POLLS": "3",
           "CONF_FAIL_THRESHOLD": "2"}
    try:
        with Cluster(admission=False, controller=False) as c:
            c.start_node_agent(node_name="mi355x-rules", backend="mock", poll_interval_ms=50, extra_env=env)
            assert kubelet.wait(lambda: kubelet.device_lists and
                                all(x[1] == "Healthy" for x in kubelet.device_lists[-1][1]), timeout=15)
            fx = json.loads(open(c.fixtures["mi355x-rules"]).read())
            t = [g["telemetry"] for g in fx["gpus"]]
            t[0]["retired_pages"] = 65                 # over MAX_RETIRED_PAGES (64)
            t[1]["unreservable_pages"] = 1             # a bad page the driver could not retire
            t[2]["violation_thermal_pct"] = 50         # sustained thermal throttling
            t[3]["xgmi_links_up"] = 6                  # one of 7 xGMI links down
            t[4]["ecc_uncorrectable"] = 1              # a new uncorrectable error
            t[5]["temp_mem_c"] = 99                    # HBM over 95 C
            t[6]["pcie_width"] = 8                     # PCIe link trained x8 of x16
            c.set_gpu_fixture("mi355x-rules", fx)
            want = ["Unhealthy"] * 7 + ["Healthy"]
            assert kubelet.wait(lambda: [x[1] for x in kubelet.device_lists[-1][1]] == want, timeout=15), \
                kubelet.device_lists[-1][1]
            desc = requests.get(f"http://127.0.0.1:{c.node_agent_ports['mi355x-rules']}/gpus", timeout=5).json()
            reasons = desc["unhealthy_reason"]
            for needle in ("retired HBM pages 65 > 64", "could not be retired", "sustained thermal throttling",
                           "xGMI links down: 1/7", "uncorrectable ECC errors: 1", "HBM temperature",
                           "PCIe link x8 of x16"):
                assert needle in reasons, (needle, reasons)
            node = c.admin.get("nodes", "mi355x-rules")
            assert node["metadata"]["labels"]["amd.com/gpu.healthy-count"] == "1"
            # a GPU that already has uncorrectable errors when the agent starts is never advertised Healthy
            fx2 = json.loads(open(c.fixtures["mi355x-rules"]).read())
            for g in fx2["gpus"]:
                g["telemetry"] = {k: v for k, v in g["telemetry"].items()
                                  if k not in ("retired_pages", "unreservable_pages", "violation_thermal_pct")}
                g["telemetry"].update({"xgmi_links_up": 7, "temp_mem_c": 40, "ecc_uncorrectable": 0, "pcie_width": 16})
            fx2["gpus"][7]["telemetry"]["ecc_uncorrectable"] = 3
            d2 = str(tmp_path / "dp2")
            kubelet2 = FakeKubelet(d2).start()
            try:
                env2 = dict(env, CONF_DEVICE_PLUGIN_DIR=d2)
                c.start_node_agent(node_name="mi355x-ue", backend="mock", poll_interval_ms=50, extra_env=env2,
                                   proc_name="na-ue", fixture_obj=fx2)
                assert kubelet2.wait(lambda: kubelet2.device_lists and
                                     [x[1] for x in kubelet2.device_lists[-1][1]] == ["Healthy"] * 7 + ["Unhealthy"],
                                     timeout=15), kubelet2.device_lists[-1:]
                desc2 = requests.get(f"http://127.0.0.1:{c.node_agent_ports['mi355x-ue']}/gpus", timeout=5).json()
                assert "already present at agent start" in desc2["unhealthy_reason"]
            finally:
                kubelet2.stop()
    finally:
        kubelet.stop()

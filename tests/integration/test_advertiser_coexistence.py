"""The node agent never fights another advertiser of the node's GPUs.

The reference leaves GPU advertisement to a vendor device plugin and only names quota keys
(/root/reference/src/synchronizer.rs:268,276).  This build replaces that plugin, and an
MI355X node commonly runs AMD's GPU Operator, whose device plugin registers amd.com/gpu
and whose labeller owns amd.com/gpu.* labels.  The agent therefore looks for

* another live device plugin in the kubelet's plugin directory that serves its resource
  (its ListAndWatch ids against the kubelet checkpoint's RegisteredDevices), and
* another field manager on its Node owning amd.com/gpu.* labels or the resource's
  capacity,

and stands down on a finding: no plugin registration, no label or status writes, a
Warning Event and a log line.  CONF_TAKE_OVER=true advertises anyway.  The fake kubelet and
the foreign plugin are python grpcio (testing/kubelet.py), an independent gRPC stack.
"""
import os

import pytest
import requests

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for
from bacchus_gpu_controller_amd.testing.kubelet import FakeDevicePlugin, FakeKubelet

pytestmark = pytest.mark.slow

OPERATOR_IDS = [f"amdgpu_xcp_{i}" for i in range(8)]


def _events(c, reason, node):
    items = c.admin.list("events", namespace="default")["items"]
    return [e for e in items if e["reason"] == reason and e["involvedObject"]["name"] == node]


def _gpus(c, node):
    return requests.get(f"http://127.0.0.1:{c.node_agent_ports[node]}/gpus", timeout=5).json()


def _ours(kubelet):
    return [r for r in kubelet.registrations if r.endpoint == "bgc-amd-gpu.sock"]


def _agent(c, node, d, **extra):
    env = {"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d, "CONF_HEARTBEAT_SECS": "1"}
    env.update(extra)
    return c.start_node_agent(node_name=node, backend="mock", poll_interval_ms=100, proc_name=f"na-{node}",
                              extra_env=env)


@pytest.fixture
def kubelet_with_operator_plugin(tmp_path):
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    other = FakeDevicePlugin(d, "amd.com_gpu", OPERATOR_IDS).start()
    other.register("amd.com/gpu")
    assert kubelet.wait(lambda: kubelet.registered_devices.get("amd.com/gpu") == OPERATOR_IDS)
    assert os.path.exists(os.path.join(d, "kubelet_internal_checkpoint"))
    yield d, kubelet, other
    other.stop()
    kubelet.stop()


def test_stands_down_for_a_registered_device_plugin_then_takes_over_when_it_goes(kubelet_with_operator_plugin):
    d, kubelet, other = kubelet_with_operator_plugin
    with Cluster(admission=False, controller=False) as c:
        _agent(c, "mi355x-co", d)
        ev = wait_for(lambda: _events(c, "GPUAdvertiserConflict", "mi355x-co"), timeout=10, desc="conflict event")[0]
        assert ev["type"] == "Warning" and "amd.com_gpu" in ev["message"]
        g = _gpus(c, "mi355x-co")["advertiser"]
        assert g["standing_down"] and not g["plugin_started"]
        [conf] = g["conflicts"]
        assert conf["kind"] == "device-plugin" and conf["evidence"] == "kubelet checkpoint" and conf["devices"] == 8
        node = c.admin.get("nodes", "mi355x-co")
        assert not any(k.startswith("amd.com/gpu.") for k in node["metadata"].get("labels", {}))
        assert not _ours(kubelet)
        assert "standing down" in c.procs["na-mi355x-co"].output()
        m = requests.get(f"http://127.0.0.1:{c.node_agent_ports['mi355x-co']}/metrics", timeout=5).text
        assert "bgc_node_agent_standing_down 1" in m

        # the operator's plugin is removed: the next heartbeat finds no conflict and advertises
        other.stop()
        assert kubelet.wait(lambda: _ours(kubelet), timeout=10)
        wait_for(lambda: c.admin.get("nodes", "mi355x-co")["metadata"].get("labels", {}).get("amd.com/gpu.count") == "8",
                 timeout=10, desc="labels after the conflict cleared")
        assert wait_for(lambda: _events(c, "GPUAdvertiserConflictResolved", "mi355x-co"), timeout=5, desc="resolved")
        assert not _gpus(c, "mi355x-co")["advertiser"]["standing_down"]


def test_take_over_advertises_anyway(kubelet_with_operator_plugin):
    d, kubelet, _ = kubelet_with_operator_plugin
    with Cluster(admission=False, controller=False) as c:
        _agent(c, "mi355x-to", d, CONF_TAKE_OVER="true")
        assert kubelet.wait(lambda: _ours(kubelet), timeout=10)
        wait_for(lambda: _events(c, "GPUAdvertiserTakeOver", "mi355x-to"), timeout=10, desc="take-over event")
        g = _gpus(c, "mi355x-to")["advertiser"]
        assert not g["standing_down"] and g["plugin_started"] and g["conflicts"]


def test_unrelated_plugins_are_not_a_conflict(tmp_path):
    """A NIC plugin (another resource, other ids) and a stale socket nobody serves."""
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    nic = FakeDevicePlugin(d, "rdma.sock", ["mlx5_0", "mlx5_1"]).start()
    nic.register("rdma/hca")
    stale = FakeDevicePlugin(d, "old.sock", ["x"]).start()
    stale.server.stop(grace=None)  # socket file left behind, nobody listening
    try:
        assert kubelet.wait(lambda: "rdma/hca" in kubelet.registered_devices)
        with Cluster(admission=False, controller=False) as c:
            _agent(c, "mi355x-nic", d)
            assert kubelet.wait(lambda: _ours(kubelet), timeout=10)
            assert _gpus(c, "mi355x-nic")["advertiser"]["conflicts"] == []
    finally:
        nic.stop()
        kubelet.stop()


@pytest.mark.parametrize("owned", ["labels", "labels-update", "capacity"])
def test_stands_down_for_fields_owned_by_another_manager(owned):
    """"labels-update" is a labeller that writes with Update under a
    manager named after its binary and not on CONF_KNOWN_LABELLERS: still a conflict."""
    with Cluster(admission=False, controller=False) as c:
        node = "mi355x-lab"
        c.admin.create("nodes", {"apiVersion": "v1", "kind": "Node", "metadata": {"name": node}})
        if owned == "labels":  # the GPU Operator's node labeller
            c.admin.apply("nodes", node, {"apiVersion": "v1", "kind": "Node",
                                          "metadata": {"name": node, "labels": {"amd.com/gpu.family": "AI",
                                                                                "amd.com/gpu.device-id": "75a3"}}},
                          "amdgpu-node-labeller", force=True)
        elif owned == "labels-update":
            c.admin.merge_patch("nodes", node, {"metadata": {"labels": {"amd.com/gpu.family": "AI"}}},
                                field_manager="k8s-node-labeller")
        else:  # another agent advertising through the Node status
            c.admin.apply("nodes", node, {"apiVersion": "v1", "kind": "Node", "metadata": {"name": node},
                                          "status": {"capacity": {"amd.com/gpu": "8"}}},
                          "other-gpu-agent", force=True, sub="status")
        c.start_node_agent(node_name=node, backend="mock", proc_name="na-lab", extra_env={"CONF_HEARTBEAT_SECS": "1"})
        wait_for(lambda: _events(c, "GPUAdvertiserConflict", node), timeout=10, desc="conflict event")
        [conf] = _gpus(c, node)["advertiser"]["conflicts"]
        assert conf["kind"] == owned.split("-")[0]
        assert conf["manager"] == {"labels": "amdgpu-node-labeller", "labels-update": "k8s-node-labeller",
                                   "capacity": "other-gpu-agent"}[owned]
        assert conf["conflict"] is True
        got = c.admin.get("nodes", node)
        labels = got["metadata"].get("labels", {})
        assert "amd.com/gpu.count" not in labels
        if owned.startswith("labels"):
            assert labels["amd.com/gpu.family"] == "AI"  # not forced over
            assert "amd.com/gpu" not in got.get("status", {}).get("capacity", {})
        assert not any(c["type"] == "AMDGPUHealthy" for c in got.get("status", {}).get("conditions", []))

        # an operator who wants this agent to win sets CONF_TAKE_OVER=true
        c.procs["na-lab"].stop()
        c.start_node_agent(node_name=node, backend="mock", proc_name="na-lab2",
                           extra_env={"CONF_TAKE_OVER": "true", "CONF_HEARTBEAT_SECS": "1"})
        got = wait_for(lambda: (lambda n: n if n["metadata"].get("labels", {}).get("amd.com/gpu.count") == "8" else None)(
            c.admin.get("nodes", node)), timeout=10, desc="take-over publish")
        assert got["metadata"]["labels"]["amd.com/gpu.family"] == "gfx950"
        assert got["status"]["capacity"]["amd.com/gpu"] == "8"


def test_plugin_stopped_for_a_conflict_restarts_once_it_clears(tmp_path):
    """a conflict found while advertising used to stop the device plugin
    until the agent restarted.  Now the plugin serves and registers again once a heartbeat
    finds the other advertiser gone."""
    d = str(tmp_path / "dp")
    kubelet = FakeKubelet(d).start()
    try:
        with Cluster(admission=False, controller=False) as c:
            _agent(c, "mi355x-rs", d, RUST_LOG="info")
            assert kubelet.wait(lambda: len(_ours(kubelet)) == 1, timeout=10)
            other = FakeDevicePlugin(d, "amd.com_gpu", OPERATOR_IDS).start()
            other.register("amd.com/gpu")
            try:
                wait_for(lambda: _gpus(c, "mi355x-rs")["advertiser"]["plugin_stopped"], timeout=10, desc="plugin stopped")
                assert "it starts again once that advertiser is gone" in c.procs["na-mi355x-rs"].output()
            finally:
                other.stop()
            assert kubelet.wait(lambda: len(_ours(kubelet)) == 2, timeout=10), "re-registered after the conflict"
            g = _gpus(c, "mi355x-rs")["advertiser"]
            assert not g["plugin_stopped"] and not g["standing_down"]
            assert "device plugin restarted" in c.procs["na-mi355x-rs"].output()
    finally:
        kubelet.stop()


def test_an_admins_kubectl_label_is_not_a_conflict():
    """a one-off `kubectl label` of an amd.com/gpu.* label (an Update by a
    kubectl manager) is reported, but the agent keeps advertising; a labeller that
    server-side applies the labels still makes it stand down (test above)."""
    with Cluster(admission=False, controller=False) as c:
        node = "mi355x-kl"
        c.admin.create("nodes", {"apiVersion": "v1", "kind": "Node", "metadata": {"name": node}})
        c.admin.merge_patch("nodes", node, {"metadata": {"labels": {"amd.com/gpu.note": "reserved-for-lab"}}},
                            field_manager="kubectl-label")
        c.start_node_agent(node_name=node, backend="mock", proc_name="na-kl", extra_env={"CONF_HEARTBEAT_SECS": "1"})
        got = wait_for(lambda: (lambda n: n if n["metadata"].get("labels", {}).get("amd.com/gpu.count") == "8" else None)(
            c.admin.get("nodes", node)), timeout=10, desc="published despite the admin's label")
        assert got["metadata"]["labels"]["amd.com/gpu.note"] == "reserved-for-lab"
        g = _gpus(c, node)["advertiser"]
        assert not g["standing_down"]
        [conf] = g["conflicts"]
        assert conf["manager"] == "kubectl-label" and conf["conflict"] is False
        assert not _events(c, "GPUAdvertiserConflict", node)

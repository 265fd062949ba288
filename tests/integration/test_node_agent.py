"""Node agent against kube-lite with the file-backed mock amdsmi backend: Node labels,
amd.com/gpu capacity/allocatable, and GPU flap handling (BASELINE config #5)."""
import json
import os
import time

import pytest
import requests

from bacchus_gpu_controller_amd.testing.cluster import NODE_AGENT_TOKEN, Cluster, free_port
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

pytestmark = pytest.mark.slow


def _write_atomic(path, obj):
    # rename, so the agent's mtime-triggered reload never sees a truncated fixture
    tmp = str(path) + ".tmp"
    with open(tmp, "w") as fh:
        json.dump(obj, fh)
    os.replace(tmp, path)


def test_node_agent_advertises_and_flaps(nat):
    with Cluster(admission=False, controller=False) as c:
        fixture = os.path.join(c.workdir, "gpus.json")
        f = json.loads(nat.default_mi355x_fixture(8))
        _write_atomic(fixture, f)
        port = free_port()
        env = c.component_env(NODE_AGENT_TOKEN, port)
        env.update({"CONF_NODE_NAME": "mi355x-0", "CONF_GPU_BACKEND": "mock", "CONF_MOCK_FIXTURE_PATH": fixture,
                    "CONF_POLL_INTERVAL_MS": "50", "CONF_CREATE_NODE": "true", "CONF_HEARTBEAT_SECS": "1"})
        c.start_process("node-agent", "node-agent", env)
        node = wait_for(lambda: (lambda n: n if n and n.get("status", {}).get("capacity") else None)(
            c.admin.get_or_none("nodes", "mi355x-0")), timeout=10, desc="node published")
        labels = node["metadata"]["labels"]
        assert labels["amd.com/gpu.product"] == "MI355X" and labels["amd.com/gpu.count"] == "8"
        assert labels["amd.com/gpu.vram-gb"] == "288"
        assert node["status"]["capacity"]["amd.com/gpu"] == "8"
        assert node["status"]["allocatable"]["amd.com/gpu"] == "8"
        managers = {m["manager"] for m in node["metadata"]["managedFields"]}
        assert "bacchus-gpu-node-agent" in managers
        gp = requests.get(f"http://127.0.0.1:{port}/gpus", timeout=5).json()
        assert len(gp["gpus"]) == 8 and gp["polls"] >= 1
        metrics = requests.get(f"http://127.0.0.1:{port}/metrics", timeout=5).text
        assert 'amd_gpu_power_watts{gpu="0"}' in metrics

        # flap: gpu 3 overheats -> allocatable 7, condition False
        f["gpus"][3]["telemetry"]["temp_hotspot_c"] = 121
        _write_atomic(fixture, f)
        wait_for(lambda: c.admin.get("nodes", "mi355x-0")["status"]["allocatable"]["amd.com/gpu"] == "7",
                 timeout=10, desc="allocatable drops to 7")
        cond = c.admin.get("nodes", "mi355x-0")["status"]["conditions"][0]
        assert cond["status"] == "False" and "gpu3" in cond["message"]
        # recovery
        f["gpus"][3]["telemetry"]["temp_hotspot_c"] = 50
        _write_atomic(fixture, f)
        wait_for(lambda: c.admin.get("nodes", "mi355x-0")["status"]["allocatable"]["amd.com/gpu"] == "8",
                 timeout=10, desc="allocatable back to 8")


def test_node_agent_waits_for_kubelet_registration():
    """Real clusters (CONF_CREATE_NODE=false): the agent never creates the Node; when the
    kubelet registers it, the agent's Node watch publishes immediately (heartbeat is 30 s)."""
    with Cluster(admission=False, controller=False) as c:
        c.start_node_agent(node_name="mi355x-9", backend="mock", proc_name="na",
                           extra_env={"CONF_CREATE_NODE": "false", "CONF_HEARTBEAT_SECS": "30"})
        time.sleep(1.0)
        assert c.admin.get_or_none("nodes", "mi355x-9") is None
        c.admin.create("nodes", {"apiVersion": "v1", "kind": "Node",
                                 "metadata": {"name": "mi355x-9", "labels": {"kubernetes.io/hostname": "mi355x-9"}}})
        node = wait_for(lambda: (lambda n: n if n.get("status", {}).get("allocatable", {}).get("amd.com/gpu") == "8"
                                 else None)(c.admin.get("nodes", "mi355x-9")), timeout=5, desc="published on registration")
        labels = node["metadata"]["labels"]
        assert labels["kubernetes.io/hostname"] == "mi355x-9" and labels["amd.com/gpu.count"] == "8"
        assert c.procs["na"].alive()


def test_diag_worker_protocol():
    """`node-agent --diag-worker` (gpu/diag_runner.h): one JSON request from
    $BGC_DIAG_REQUEST, one JSON result on stdout, exit 0 even on errors (the agent reads
    the error from the result).  On a CPU host HIP sees no devices."""
    import subprocess

    from bacchus_gpu_controller_amd import binary

    from bacchus_gpu_controller_amd import REPO_ROOT

    lib = os.path.join(REPO_ROOT, "bacchus_gpu_controller_amd", "libbgc_gpu_diag.so")

    def worker(req):
        # the in-tree library, wherever the binary under test was built (sanitizer trees)
        env = dict(os.environ, BGC_DIAG_REQUEST=json.dumps(req), BGC_GPU_DIAG_LIB=lib)
        p = subprocess.run([binary("node-agent"), "--diag-worker"], env=env, capture_output=True, text=True, timeout=60)
        assert p.returncode == 0, p.stderr
        return json.loads(p.stdout)

    assert "bdfs" in worker({"op": "devices"})
    assert "unknown diagnostics worker op" in worker({"op": "bogus"})["error"]
    p = subprocess.run([binary("node-agent"), "--diag-worker"], env={k: v for k, v in os.environ.items()
                                                                      if k != "BGC_DIAG_REQUEST"},
                       capture_output=True, text=True, timeout=60)
    assert "BGC_DIAG_REQUEST is not set" in json.loads(p.stdout)["error"]

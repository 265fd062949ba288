"""Round-4 node-agent checks on a real MI355X.

* A diagnostics worker verifies that the one GPU it sees is the GPU the agent meant (PCI
  BDF) and refuses to run on any other: a renumbered or hidden device must never put a
  burn or a verdict on another GPU, possibly a tenant's.
* Device-visibility variables in the agent's own environment (HIP_VISIBLE_DEVICES,
  CUDA_VISIBLE_DEVICES) do not reach its workers: a full pass still diagnoses the GPU.

Results go to gpurun_out/r4_gpu/."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "r4_gpu")


def _dump(name, obj):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)


def _worker(request, **env):
    from bacchus_gpu_controller_amd import binary

    full = dict(os.environ)
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        full.pop(k, None)
    full.update({"BGC_DIAG_REQUEST": json.dumps(request), **env})
    p = subprocess.run([binary("node-agent"), "--diag-worker"], env=full, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_worker_refuses_a_gpu_other_than_requested():
    from bacchus_gpu_controller_amd import native

    bdf = native().diag_device_bdf(0)
    burn = {"op": "burn", "backend": "amdsmi", "fixture": "", "gpu_hip_device": 0, "duration_ms": 300,
            "dtype": "bf16", "seed": 7, "start_at_ns": 0}
    wrong = _worker(dict(burn, expect_bdf="0000:ff:00.0"), ROCR_VISIBLE_DEVICES="0")
    right = _worker(dict(burn, expect_bdf=bdf.upper()), ROCR_VISIBLE_DEVICES="0")  # BDF case does not matter
    _dump("worker_bdf_check.json", {"hip_bdf": bdf, "wrong": wrong, "right_keys": sorted(right)})
    assert "expected 0000:ff:00.0" in wrong.get("error", "") and bdf in wrong["error"], wrong
    assert "error" not in right and right["tflops_mean"] > 500, right


def test_agent_visibility_env_does_not_reach_workers(tmp_path):
    from bacchus_gpu_controller_amd.testing.cluster import Cluster

    import requests

    with Cluster(admission=False, controller=False) as c:
        # device 7 does not exist on a 1-GPU lease: a worker inheriting these would see no GPU
        c.start_node_agent(node_name="mi355x-vis", backend="amdsmi", max_gpus=1, poll_interval_ms=500,
                           extra_env={"CONF_RUN_DIAG": "true", "CONF_DIAG_BURN_MS": "500",
                                      "CONF_DIAG_START_BUSY": "diagnose", "HIP_VISIBLE_DEVICES": "7",
                                      "CUDA_VISIBLE_DEVICES": "7", "CONF_DIAG_HBM_WALK_FRACTION": "0.1",
                                      "CONF_DIAG_MIN_HBM_WALK_COVERAGE": "0.05"})
        desc = requests.get(f"http://127.0.0.1:{c.node_agent_ports['mi355x-vis']}/gpus", timeout=10).json()
        _dump("agent_visibility_env.json", {"diag": desc["diag"], "hip_devices": desc["hip_devices"],
                                            "isolation": desc["diag_isolation"]})
        assert desc["diag_isolation"] == "worker-process"
        assert desc["diag"][0]["passed"], desc["diag"][0]["failures"]

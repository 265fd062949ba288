"""The node-agent image ships only the ROCm libraries `tools/node_image_closure.sh` copies
(Dockerfile, node-agent stage).  Docker is not available on either box, so this runs the
agent the way the image does: every ROCm library from that closure directory
(LD_LIBRARY_PATH, BGC_GPU_DIAG_LIB), through a full diagnostics pass on the real MI355X,
with the dynamic loader's trace on.  Any library the closure missed would have been
found in /opt/rocm through the loader cache instead; the trace shows none was."""
import json
import os
import re
import subprocess

import pytest

from bacchus_gpu_controller_amd import REPO_ROOT

pytestmark = pytest.mark.gpu


def _loaded(ld_dir):
    """Paths the loader initialised, from LD_DEBUG=files output files (one per process)."""
    paths = set()
    for name in os.listdir(ld_dir):
        with open(os.path.join(ld_dir, name), errors="replace") as f:
            for line in f:
                m = re.search(r"calling init: (\S+)", line)
                if m:
                    paths.add(m.group(1))
    return paths


def test_node_agent_runs_on_the_image_closure(tmp_path):
    import requests

    from bacchus_gpu_controller_amd.testing.cluster import Cluster
    from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

    rt = tmp_path / "rt"
    diag_lib = os.path.join(REPO_ROOT, "bacchus_gpu_controller_amd", "libbgc_gpu_diag.so")
    r = subprocess.run(["bash", os.path.join(REPO_ROOT, "tools", "node_image_closure.sh"), str(rt), diag_lib],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    shipped = sorted(os.listdir(rt))
    ld_dir = tmp_path / "ld"
    ld_dir.mkdir()
    with Cluster(admission=False, controller=False) as c:
        c.start_node_agent(node_name="mi355x-img", backend="amdsmi", max_gpus=1, poll_interval_ms=200,
                           extra_env={"LD_LIBRARY_PATH": str(rt), "BGC_GPU_DIAG_LIB": str(rt / "libbgc_gpu_diag.so"),
                                      "LD_DEBUG": "files", "LD_DEBUG_OUTPUT": str(ld_dir / "ld"),
                                      "CONF_RUN_DIAG": "true", "CONF_DIAG_BURN_MS": "1000",
                                      "CONF_DIAG_START_BUSY": "diagnose"})  # this test process may hold the GPU
        port = c.node_agent_ports["mi355x-img"]
        wait_for(lambda: requests.get(f"http://127.0.0.1:{port}/gpus", timeout=5).json().get("diag"), timeout=90,
                 desc="diagnostics pass")
        desc = requests.get(f"http://127.0.0.1:{port}/gpus", timeout=5).json()
    loaded = _loaded(ld_dir)
    rocm = sorted(p for p in loaded if p.startswith("/opt/rocm"))
    from_closure = sorted(os.path.basename(p) for p in loaded if p.startswith(str(rt)))
    out = {"shipped": shipped, "loaded_from_closure": from_closure, "loaded_from_opt_rocm": rocm,
           "closure_mb": round(sum(os.path.getsize(rt / f) for f in shipped) / 2**20, 1),
           "diag_engine": desc.get("diag_engine"), "diag_passed": desc["diag"][0]["passed"],
           "diag_failures": desc["diag"][0].get("failures")}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/node_image_closure.json", "w") as f:
        json.dump(out, f, indent=1)
    assert not rocm, f"loaded from /opt/rocm, missing from the image closure: {rocm}"
    assert "libamdhip64.so.7" in from_closure and "libamd_smi.so" in from_closure, out
    assert desc["diag_engine"] == "hip" and desc["diag"][0]["passed"], out

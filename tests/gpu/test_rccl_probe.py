"""RCCL probe on the real box (world size = visible GPUs on this pool: 1)."""
import json
import subprocess
import sys

import pytest

from bacchus_gpu_controller_amd import REPO_ROOT

pytestmark = pytest.mark.gpu


def test_rccl_probe_single_gpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29571",
           "-m", "bacchus_gpu_controller_amd.parallel.rccl_probe", "--sizes-mb", "1,64", "--iters", "3"]
    r = subprocess.run(cmd, cwd=REPO_ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["all_correct"]
    assert out["hives"][0] not in ("cpu",) and not out["hives"][0].startswith("unavailable")
    # the link counters were read (world 1 sends nothing over xGMI itself; 8-GPU runs
    # compare the written bytes with the ring's expected traffic)
    t = out["xgmi_traffic"][0]
    assert t["xgmi_written_mb"] is not None and t["expected_mb"] == 0 and out["traffic_on_xgmi"] is False

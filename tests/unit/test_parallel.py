"""xGMI placement planning + the RCCL probe's logic (gloo, world_size 2, on CPU)."""
import json
import os
import subprocess
import sys

import pytest

from bacchus_gpu_controller_amd import REPO_ROOT
from bacchus_gpu_controller_amd.parallel import placement


def node(name, hive, count=8, healthy=None, mixed=None):
    topo = [{"index": i, "hive": (mixed[i] if mixed else hive)} for i in range(count)]
    return {"metadata": {"name": name,
                         "labels": {"amd.com/gpu.xgmi-hive-id": hive if not mixed else "mixed",
                                    "amd.com/gpu.count": str(count)},
                         "annotations": {"amd.com/gpu.topology": json.dumps(topo)}},
            "status": {"allocatable": {"amd.com/gpu": str(count if healthy is None else healthy)}}}


def test_plan_tp8_one_group_per_island():
    nodes = [node("a", "h1"), node("b", "h2"), node("c", "h3", healthy=7)]
    plan = placement.plan_tp_groups(nodes, 8, 2)
    assert {p["hive"] for p in plan} == {"h1", "h2"}  # h3 has only 7 healthy GPUs
    with pytest.raises(ValueError):
        placement.plan_tp_groups(nodes, 8, 3)


def test_plan_tp4_packs_islands():
    plan = placement.plan_tp_groups([node("a", "h1")], 4, 2)
    assert [p["hive"] for p in plan] == ["h1", "h1"]


def test_mixed_node_never_splits_tp_group():
    n = node("m", "x", mixed=["h1"] * 4 + ["h2"] * 4)
    with pytest.raises(ValueError):
        placement.plan_tp_groups([n], 8, 1)
    assert len(placement.plan_tp_groups([n], 4, 2)) == 2
    inv = placement.hive_inventory([n])
    assert inv["h1"]["gpus"] == 4 and inv["h2"]["gpus"] == 4


def test_tp_pod_affinity():
    spec = placement.tp_pod_affinity("4ca22c3b0ce7816e", 8)
    assert spec["nodeSelector"]["amd.com/gpu.xgmi-hive-id"] == "4ca22c3b0ce7816e"
    assert spec["resources"]["limits"]["amd.com/gpu"] == "8"


@pytest.mark.slow
def test_rccl_probe_logic_gloo_world2():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29561",
           "-m", "bacchus_gpu_controller_amd.parallel.rccl_probe", "--sizes-mb", "0.25,1", "--iters", "3",
           "--warmup", "1", "--dtype", "fp32"]
    r = subprocess.run(cmd, cwd=REPO_ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["world_size"] == 2 and out["backend"] == "gloo" and out["all_correct"]
    assert out["single_hive"] and len(out["results"]) == 2
    # no GPU: no link counters, and a CPU group never claims xGMI traffic
    assert [t["xgmi_written_mb"] for t in out["xgmi_traffic"]] == [None, None] and out["traffic_on_xgmi"] is False
    assert all(t["expected_mb"] > 0 for t in out["xgmi_traffic"])


def _hive_fixture():
    # two 4-GPU hives; amdsmi hip_id is the host-wide ordinal
    return [{"index": i, "hip_id": i, "bdf": f"0000:{0x05 + 0x10 * i:02x}:00.0",
             "xgmi_hive_id": "aaaa" if i < 4 else "bbbb"} for i in range(8)]


def test_probe_maps_rank_gpu_by_bdf_not_hip_id():
    """Inside a container with HIP_VISIBLE_DEVICES=6,2 HIP calls the GPUs 0 and 1, but
    amdsmi's hip_id 0/1 are other GPUs on the host: the BDF decides."""
    from bacchus_gpu_controller_amd.parallel import rccl_probe

    gpus = _hive_fixture()
    visible = [6, 2]  # HIP ordinal -> host GPU
    for local, host in enumerate(visible):
        bdf = gpus[host]["bdf"]
        g = rccl_probe.match_gpu(gpus, bdf=bdf, local_rank=local)
        assert g["index"] == host and g["xgmi_hive_id"] == gpus[host]["xgmi_hive_id"]
    # torch reports no function number and may use upper-case hex
    assert rccl_probe.match_gpu(gpus, bdf="0000:65:00.0".upper(), local_rank=0)["index"] == 6
    # without a BDF the old hip_id rule is the last resort
    assert rccl_probe.match_gpu(gpus, bdf=None, local_rank=1)["index"] == 1


def test_probe_uses_device_plugin_allocation_for_partitions():
    from bacchus_gpu_controller_amd.parallel import rccl_probe

    # CPX: 4 logical devices share each BDF; the plugin names them <bdf>-p<index>
    gpus = [{"index": i, "hip_id": i, "bdf": "0000:05:00.0" if i < 4 else "0000:15:00.0",
             "xgmi_hive_id": "h" + str(i // 4)} for i in range(8)]
    alloc = ["0000:15:00.0-p6"]
    g = rccl_probe.match_gpu(gpus, bdf="0000:15:00.0", local_rank=0, allocated=alloc)
    assert g["index"] == 6
    # allocation without partitions narrows to the allocated BDFs
    g = rccl_probe.match_gpu(_hive_fixture(), bdf=None, local_rank=0, allocated=["0000:45:00.0"])
    assert g["index"] == 4

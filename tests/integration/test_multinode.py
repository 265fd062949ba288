"""Multi-node churn without a cluster (SURVEY §4.2 "multi-node" row, BASELINE configs #4/#5).

Four synthetic MI355X nodes are published by four native node agents with mock amdsmi
backends, each on its own xGMI hive. While the synchronizer is onboarding tenants from the
sheet, the test drives the following and checks the results:
  * a drain and re-add of one node (cordon, delete the Node, re-register): the agent's Node watch
    re-publishes labels and capacity well before the 30 s heartbeat;
  * a flap of all 8 GPUs on another node (hotspot over the limit, then recovery): allocatable
    0 -> 8 and the AMDGPUHealthy condition follows;
  * a quota edit in the sheet mid-churn: the synchronizer converges every tenant;
  * TP=8 placement over the live Node objects always picks whole, healthy, schedulable islands.
"""
import copy
import json
import time

import pytest

from bacchus_gpu_controller_amd.parallel.placement import hive_inventory, plan_tp_groups
from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

pytestmark = pytest.mark.slow

NODES = [f"mi355x-{i}" for i in range(4)]
USERS = [f"user{i:02d}" for i in range(16)]


def ub(name):
    return {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": name}, "spec": {}}


def alloc(c, node):
    n = c.admin.get_or_none("nodes", node)
    return None if n is None else n.get("status", {}).get("allocatable", {}).get("amd.com/gpu")


def all_synced(c, gpus_of):
    for u in USERS:
        o = c.admin.get("userbootstraps", u)
        if not o.get("status", {}).get("synchronized_with_sheet"):
            return False
        if o["spec"].get("quota", {}).get("hard", {}).get("requests.amd.com/gpu") != str(gpus_of(u)):
            return False
        rq = c.admin.get_or_none("resourcequotas", u, u)
        if rq is None or rq["spec"]["hard"].get("requests.amd.com/gpu") != str(gpus_of(u)):
            return False
    return True


def test_multinode_drain_flap_and_sync_convergence():
    google = FakeGoogle().start()
    try:
        google.set_rows([{"id_username": u, "gpu": 1 + i % 8} for i, u in enumerate(USERS)])
        with Cluster(controller_env={"CONF_REQUEUE_SECS": "5", "CONF_ERROR_REQUEUE_MS": "200"}) as c:
            for i, n in enumerate(NODES):
                c.start_node_agent(node_name=n, backend="mock", hive_id=0x355000 + i, proc_name=f"node-agent-{n}",
                                   poll_interval_ms=50, extra_env={"CONF_HEARTBEAT_SECS": "30"})
            for n in NODES:
                wait_for(lambda: alloc(c, n) == "8", timeout=10, desc=f"{n} advertised")
            inv = hive_inventory(c.admin.list("nodes")["items"])
            assert len(inv) == 4 and all(e["healthy"] == 8 and len(e["nodes"]) == 1 for e in inv.values())

            c.start_synchronizer(google, interval=1)
            for u in USERS:
                c.as_user(f"oidc:{u}", ["gpu"]).create("userbootstraps", ub(u))

            # --- drain + re-add mi355x-1 while tenants are being onboarded
            c.admin.merge_patch("nodes", "mi355x-1", {"spec": {"unschedulable": True}})
            plan = plan_tp_groups(c.admin.list("nodes")["items"], 8, 3)
            assert "mi355x-1" not in {p["node"] for p in plan}
            c.admin.delete("nodes", "mi355x-1")
            t0 = time.time()
            node = wait_for(lambda: (lambda n: n if n and n.get("status", {}).get("capacity", {}).get("amd.com/gpu") == "8"
                                     else None)(c.admin.get_or_none("nodes", "mi355x-1")),
                            timeout=10, desc="mi355x-1 re-published")
            assert time.time() - t0 < 10  # the Node watch, not the 30 s heartbeat
            assert node["metadata"]["labels"]["amd.com/gpu.xgmi-hive-id"] == f"{0x355001:016x}"
            assert not node.get("spec", {}).get("unschedulable")

            # --- all 8 GPUs on mi355x-2 overheat, then recover
            fx = json.load(open(c.fixtures["mi355x-2"]))
            hot = copy.deepcopy(fx)
            for g in hot["gpus"]:
                g["telemetry"]["temp_hotspot_c"] = 121
            c.set_gpu_fixture("mi355x-2", hot)
            wait_for(lambda: alloc(c, "mi355x-2") == "0", timeout=10, desc="mi355x-2 allocatable 0")
            cond = {x["type"]: x for x in c.admin.get("nodes", "mi355x-2")["status"]["conditions"]}
            assert cond["AMDGPUHealthy"]["status"] == "False"
            plan = plan_tp_groups(c.admin.list("nodes")["items"], 8, 3)
            assert {p["node"] for p in plan} == {"mi355x-0", "mi355x-1", "mi355x-3"}
            with pytest.raises(ValueError):
                plan_tp_groups(c.admin.list("nodes")["items"], 8, 4)

            # --- sheet edit mid-churn: everyone's GPU quota changes
            google.set_rows([{"id_username": u, "gpu": 8 - i % 8} for i, u in enumerate(USERS)])
            c.set_gpu_fixture("mi355x-2", fx)
            wait_for(lambda: alloc(c, "mi355x-2") == "8", timeout=10, desc="mi355x-2 recovered")
            wait_for(lambda: all_synced(c, lambda u: 8 - USERS.index(u) % 8), timeout=20,
                     desc="synchronizer converged on the edited sheet")

            plan = plan_tp_groups(c.admin.list("nodes")["items"], 8, 4)
            assert sorted(p["node"] for p in plan) == NODES
            assert len({p["hive"] for p in plan}) == 4
            for n in NODES:
                assert c.procs[f"node-agent-{n}"].alive()
            assert c.procs["synchronizer"].alive() and c.procs["controller"].alive()
            assert not google.errors
    finally:
        google.stop()


def test_flap_bench_mode_reports_convergence(tmp_path):
    """BASELINE config #5 as a bench mode (bacchus_gpu_controller_amd/bench/flap.py): one
    round at fast cadences; every phase converges and is reported."""
    from bacchus_gpu_controller_amd.bench import flap

    out = tmp_path / "flap.json"
    assert flap.main(["--nodes", "2", "--tenants", "8", "--rounds", "2", "--poll-ms", "50", "--sheet-poll-ms", "300",
                      "--churn-hz", "10", "--log-level", "warn", "--json-out", str(out)]) == 0
    res = json.loads(out.read_text())
    for k in ("drain_republish_ms", "flap_unhealthy_ms", "flap_recover_ms", "sheet_converge_ms"):
        assert len(res[k]["samples"]) == 2 and res[k]["p50"] is not None, (k, res[k])
    assert res["flap_unhealthy_ms"]["max"] < 5000 and res["sheet_converge_ms"]["max"] < 10000
    assert all(res["processes_alive"].values()) and res["churn_created"] > 0


def test_tp8_bench_mode_reports_coscheduling(tmp_path):
    """BASELINE config #4 as a bench mode (bacchus_gpu_controller_amd/bench/tp8.py)."""
    from bacchus_gpu_controller_amd.bench import tp8

    out = tmp_path / "tp8.json"
    assert tp8.main(["--nodes", "2", "--iters", "60", "--log-level", "warn", "--json-out", str(out)]) == 0
    res = json.loads(out.read_text())
    assert res["plan_tp8_groups"] == 2 and res["plan_groups_on_distinct_hives"]
    assert res["churn_single_hive_share"] == 1.0 and res["two_quad_direct_xgmi_share"] == 1.0
    assert res["preferred_8_us"]["p50"] > 0 and res["allocate_8_us"]["p50"] > 0
    assert all(res["processes_alive"].values())

"""Node agent: a telemetry poll that never returns (native/gpu/telemetry.cc check_stall).

amdsmi calls block while the driver resets a wedged GPU.  Before the watchdog, the agent
kept advertising the last good readings for as long as the poll hung: the GPUs stayed
allocatable although nothing read them.  Now a poll stuck past CONF_TELEMETRY_STALL_MS
advertises every GPU unhealthy (allocatable 0, AMDGPUHealthy False, a Warning Event), and
the first poll that completes restores what the telemetry says.  The mock backend's
`sample_hang_ms` fixture key makes every reading block.
"""
import copy
import json
import time

import pytest
import requests

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

pytestmark = pytest.mark.slow

NODE = "mi355x-stall"


def alloc(c):
    n = c.admin.get_or_none("nodes", NODE)
    return None if n is None else n.get("status", {}).get("allocatable", {}).get("amd.com/gpu")


def condition(c):
    conds = c.admin.get("nodes", NODE).get("status", {}).get("conditions", [])
    return {x["type"]: x for x in conds}.get("AMDGPUHealthy")


def metric(c, name):
    text = requests.get(f"http://127.0.0.1:{c.node_agent_ports[NODE]}/metrics", timeout=5).text
    for line in text.splitlines():
        if line.startswith(name + " ") or line.startswith(name + "{"):
            return float(line.rsplit(" ", 1)[1])
    return None


def describe(c):
    return requests.get(f"http://127.0.0.1:{c.node_agent_ports[NODE]}/gpus", timeout=5).json()


@pytest.mark.parametrize("stall_ms", [1000])
def test_stuck_poll_marks_gpus_unhealthy_until_a_poll_completes(stall_ms):
    with Cluster(admission=False, controller=False) as c:
        c.start_node_agent(node_name=NODE, backend="mock", poll_interval_ms=50,
                           extra_env={"CONF_TELEMETRY_STALL_MS": str(stall_ms)})
        wait_for(lambda: alloc(c) == "8", timeout=10, desc="advertised")
        assert metric(c, "bgc_telemetry_stalled") == 0.0  # exported before any stall

        fx = json.load(open(c.fixtures[NODE]))
        hung = copy.deepcopy(fx)
        hung["sample_hang_ms"] = 120000
        t0 = time.monotonic()
        c.set_gpu_fixture(NODE, hung)
        wait_for(lambda: alloc(c) == "0", timeout=15, desc="allocatable 0 while the poll hangs")
        took = time.monotonic() - t0
        assert took >= stall_ms / 1e3 * 0.8, took  # not before the stall timeout
        cond = condition(c)
        assert cond["status"] == "False" and "telemetry stalled" in cond["message"], cond
        d = describe(c)
        assert d["telemetry_stalled"] is True and d["healthy"] == 0
        assert metric(c, "bgc_telemetry_stalled") == 1.0
        assert metric(c, "bgc_telemetry_stalls_total") == 1.0
        wait_for(lambda: any(e.get("reason") == "GPUUnhealthy" and "telemetry stalled" in e.get("message", "")
                             for e in c.admin.list("events", namespace="default")["items"]),
                 timeout=10, desc="GPUUnhealthy Event")
        assert c.procs["node-agent"].alive()

        # the hang ends: the next completed poll restores the telemetry's verdict at once
        # (the health state machine was never touched, so no recover_threshold wait)
        c.set_gpu_fixture(NODE, fx)
        wait_for(lambda: alloc(c) == "8", timeout=10, desc="allocatable 8 after the hang")
        wait_for(lambda: condition(c)["status"] == "True", timeout=10, desc="AMDGPUHealthy True")
        assert describe(c)["telemetry_stalled"] is False
        assert metric(c, "bgc_telemetry_stalled") == 0.0


def test_watchdog_off_keeps_last_readings():
    """CONF_TELEMETRY_STALL_MS=0 turns the watchdog off (the previous behaviour): a hung
    poll leaves the last published health in place."""
    with Cluster(admission=False, controller=False) as c:
        c.start_node_agent(node_name=NODE, backend="mock", poll_interval_ms=50,
                           extra_env={"CONF_TELEMETRY_STALL_MS": "0"})
        wait_for(lambda: alloc(c) == "8", timeout=10, desc="advertised")
        fx = json.load(open(c.fixtures[NODE]))
        hung = copy.deepcopy(fx)
        hung["sample_hang_ms"] = 120000
        c.set_gpu_fixture(NODE, hung)
        time.sleep(2.5)
        assert alloc(c) == "8"
        assert describe(c)["telemetry_stalled"] is False
        c.set_gpu_fixture(NODE, fx)  # let the hung sample return before the agent stops
        time.sleep(0.3)


def test_shutdown_is_bounded_while_a_poll_hangs():
    """SIGTERM while a poll is stuck: the agent stops its device plugin and other threads,
    and exits after CONF_SHUTDOWN_TIMEOUT_SECS even though the poll thread never returns."""
    with Cluster(admission=False, controller=False) as c:
        p = c.start_node_agent(node_name=NODE, backend="mock", poll_interval_ms=50,
                               extra_env={"CONF_TELEMETRY_STALL_MS": "500", "CONF_SHUTDOWN_TIMEOUT_SECS": "2"})
        wait_for(lambda: alloc(c) == "8", timeout=10, desc="advertised")
        hung = copy.deepcopy(json.load(open(c.fixtures[NODE])))
        hung["sample_hang_ms"] = 600000
        c.set_gpu_fixture(NODE, hung)
        wait_for(lambda: alloc(c) == "0", timeout=10, desc="stalled")
        t0 = time.monotonic()
        rc = p.stop(timeout=10)
        took = time.monotonic() - t0
        assert 1.5 < took < 6, took
        assert rc == 1
        assert "shutdown did not finish within 2000 ms" in p.output()

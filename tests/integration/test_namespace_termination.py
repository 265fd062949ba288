"""kube-lite: namespace deletion as on a real cluster (native/apiserver/server.cc,
terminate_namespace_locked / finish_namespace).

DELETE marks a Namespace Terminating (deletionTimestamp, status.phase); creates in it are
refused with 403 Forbidden (the NamespaceLifecycle admission plugin, cause
NamespaceTerminating); the namespace controller deletes its contents and then removes the
"kubernetes" spec finalizer, and the Namespace goes once no metadata finalizer holds it.
Before round 5 kube-lite removed a Namespace at once, so a UserBootstrap re-created while its
old Namespace was still terminating was never exercised.
"""
import json
import threading
import time

import pytest
import requests

from bacchus_gpu_controller_amd.testing.cluster import ADMIN_TOKEN, Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

pytestmark = pytest.mark.slow

HOLD = "example.com/hold"


@pytest.fixture(scope="module")
def c():
    with Cluster(admission=False, controller=False) as cl:
        yield cl


def metric(port, name):
    for line in requests.get(f"http://127.0.0.1:{port}/metrics", timeout=5).text.splitlines():
        if line.startswith(name + " "):
            return float(line.rsplit(" ", 1)[1])
    return 0.0


def ns_obj(name, finalizers=()):
    meta = {"name": name}
    if finalizers:
        meta["finalizers"] = list(finalizers)
    return {"apiVersion": "v1", "kind": "Namespace", "metadata": meta}


def cm(name):
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name}, "data": {"k": "v"}}


def raw(c, method, path, body=None):
    return requests.request(method, c.server + path, headers={"Authorization": f"Bearer {ADMIN_TOKEN}"},
                            json=body, timeout=10)


def test_delete_marks_terminating_and_refuses_new_content(c):
    c.admin.create("namespaces", ns_obj("held", [HOLD]))
    c.admin.create("configmaps", cm("a"), namespace="held")
    r = raw(c, "DELETE", "/api/v1/namespaces/held")
    assert r.status_code == 200
    body = r.json()
    assert body["kind"] == "Namespace" and body["status"]["phase"] == "Terminating"
    assert "deletionTimestamp" in body["metadata"]
    # contents go; the namespace stays while its metadata finalizer holds it
    wait_for(lambda: c.admin.get_or_none("configmaps", "a", "held") is None, timeout=5, desc="contents deleted")
    ns = wait_for(lambda: (lambda n: n if n and not n["spec"].get("finalizers") else None)(
        c.admin.get_or_none("namespaces", "held")), timeout=5, desc="kubernetes finalizer removed")
    assert ns["status"]["phase"] == "Terminating"
    r = raw(c, "POST", "/api/v1/namespaces/held/configmaps", cm("b"))
    assert r.status_code == 403, r.text
    st = r.json()
    assert st["reason"] == "Forbidden" and "because it is being terminated" in st["message"]
    assert st["details"]["causes"][0]["reason"] == "NamespaceTerminating"
    # updates of the namespace itself are allowed; a second DELETE is a no-op
    c.admin.merge_patch("namespaces", "held", {"metadata": {"labels": {"x": "y"}}})
    assert raw(c, "DELETE", "/api/v1/namespaces/held").status_code == 200
    # releasing the finalizer removes it
    c.admin.merge_patch("namespaces", "held", {"metadata": {"finalizers": None}})
    wait_for(lambda: c.admin.get_or_none("namespaces", "held") is None, timeout=5, desc="namespace gone")
    c.admin.create("namespaces", ns_obj("held"))
    assert c.admin.create("configmaps", cm("b"), namespace="held")["metadata"]["name"] == "b"


def test_watch_sees_terminating_then_deleted(c):
    c.admin.create("namespaces", ns_obj("watched"))
    c.admin.create("configmaps", cm("a"), namespace="watched")
    rv = c.admin.list("namespaces")["metadata"]["resourceVersion"]
    got = []

    def watch():
        with requests.get(c.server + f"/api/v1/namespaces?watch=1&resourceVersion={rv}&timeoutSeconds=2"
                          "&fieldSelector=metadata.name%3Dwatched",
                          headers={"Authorization": f"Bearer {ADMIN_TOKEN}"}, stream=True, timeout=12) as r:
            for line in r.iter_lines():
                if line:
                    got.append(json.loads(line))

    t = threading.Thread(target=watch)
    t.start()
    time.sleep(0.3)
    raw(c, "DELETE", "/api/v1/namespaces/watched")
    t.join()
    ev = [(e["type"], e["object"].get("status", {}).get("phase")) for e in got if e["type"] != "BOOKMARK"]
    assert ev[0] == ("MODIFIED", "Terminating") and ev[-1][0] == "DELETED", ev
    assert c.admin.get_or_none("configmaps", "a", "watched") is None


def test_instant_mode_removes_at_once():
    with Cluster(admission=False, controller=False, apiserver_args=["--instant-namespace-deletion"]) as c:
        c.admin.create("namespaces", ns_obj("quick"))
        raw(c, "DELETE", "/api/v1/namespaces/quick").raise_for_status()
        assert c.admin.get_or_none("namespaces", "quick") is None


def test_userbootstrap_recreated_while_its_namespace_terminates():
    """The tenant is deleted and created again while its old Namespace is still
    terminating (held here by a finalizer, as a slow namespace controller or a stuck
    finalizer would).  The controller's applies into it are refused (403) and retried
    without being reported as failures; once the old Namespace is gone the new one is
    created with all its children."""
    env = {"CONF_REQUEUE_SECS": "3600", "CONF_ERROR_REQUEUE_MS": "200"}
    with Cluster(admission=False, controller_env=env) as c:
        ub = {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": "again"},
              "spec": {"kube_username": "again", "quota": {"hard": {"requests.amd.com/gpu": "1"}}}}
        c.admin.create("userbootstraps", ub)
        first = wait_for(lambda: c.admin.get_or_none("resourcequotas", "again", "again"), desc="first tenant ready")
        old_ns = c.admin.get("namespaces", "again")
        c.admin.merge_patch("namespaces", "again", {"metadata": {"finalizers": [HOLD]}})
        c.admin.delete("userbootstraps", "again")
        wait_for(lambda: (c.admin.get_or_none("namespaces", "again") or {}).get("status", {}).get("phase")
                 == "Terminating", timeout=5, desc="namespace terminating")
        wait_for(lambda: c.admin.get_or_none("resourcequotas", "again", "again") is None, timeout=5,
                 desc="old quota deleted")
        c.admin.create("userbootstraps", ub)
        time.sleep(1.0)  # the controller retries into the terminating namespace meanwhile
        assert c.admin.get_or_none("resourcequotas", "again", "again") is None
        assert c.procs["controller"].alive()
        # an expected wait, not a failure: no error log, no ReconcileFailed Event
        assert metric(c.controller_port, "bgc_reconcile_namespace_terminating_total") >= 1
        assert "being terminated" not in c.procs["controller"].output()
        assert not [e for e in c.admin.list("events", namespace="default")["items"]
                    if e["reason"] == "ReconcileFailed" and e["involvedObject"]["name"] == "again"]
        c.admin.merge_patch("namespaces", "again", {"metadata": {"finalizers": None}})
        rq = wait_for(lambda: c.admin.get_or_none("resourcequotas", "again", "again"), timeout=10,
                      desc="second tenant ready")
        ns = c.admin.get("namespaces", "again")
        assert ns["metadata"]["uid"] != old_ns["metadata"]["uid"] and ns["status"]["phase"] == "Active"
        assert rq["metadata"]["uid"] != first["metadata"]["uid"]
        new_ub = c.admin.get("userbootstraps", "again")
        assert ns["metadata"]["ownerReferences"][0]["uid"] == new_ub["metadata"]["uid"]


def test_cascade_after_a_tenant_deletion_queues_no_reconciles():
    """Deleting a UserBootstrap turns its Namespace Terminating before the children go.  The
    controller ignores child events that cannot need a reconcile: a child with a
    deletionTimestamp (until its DELETED event) and one whose owner is no longer cached."""
    env = {"CONF_REQUEUE_SECS": "3600"}
    with Cluster(admission=False, controller_env=env) as c:
        for i in range(3):
            c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                              "metadata": {"name": f"gone{i}"}, "spec": {"kube_username": f"gone{i}"}})
        for i in range(3):
            wait_for(lambda: c.admin.get_or_none("namespaces", f"gone{i}"), desc="tenant namespace")
        r0 = metric(c.controller_port, 'bgc_reconcile_total{result="ok"}')
        for i in range(3):
            c.admin.delete("userbootstraps", f"gone{i}")
        for i in range(3):
            wait_for(lambda: c.admin.get_or_none("namespaces", f"gone{i}") is None, timeout=10, desc="namespace gone")
        time.sleep(0.3)
        assert metric(c.controller_port, 'bgc_controller_child_events_ignored_total{reason="terminating"}') >= 3
        assert metric(c.controller_port, 'bgc_reconcile_total{result="ok"}') == r0


def test_namespace_deleted_under_a_live_tenant_is_recreated():
    """An admin deletes a live tenant's Namespace.  It terminates (its quota and bindings go
    first); the controller's repairs into it meanwhile are refused and retried quietly, and
    its DELETED event brings the Namespace and every child back, without waiting for the
    periodic requeue (an hour here)."""
    env = {"CONF_REQUEUE_SECS": "3600", "CONF_RESYNC_SECS": "0"}
    with Cluster(admission=False, controller_env=env) as c:
        c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                          "metadata": {"name": "live"},
                                          "spec": {"kube_username": "live",
                                                   "quota": {"hard": {"requests.amd.com/gpu": "2"}}}})
        first = wait_for(lambda: c.admin.get_or_none("resourcequotas", "live", "live"), desc="tenant ready")
        old_ns = c.admin.get("namespaces", "live")
        raw(c, "DELETE", "/api/v1/namespaces/live").raise_for_status()
        ns = wait_for(lambda: (lambda n: n if n and n["metadata"]["uid"] != old_ns["metadata"]["uid"] else None)(
            c.admin.get_or_none("namespaces", "live")), timeout=10, desc="namespace re-created")
        assert ns["status"]["phase"] == "Active" and ns["metadata"]["ownerReferences"][0]["name"] == "live"
        rq = wait_for(lambda: c.admin.get_or_none("resourcequotas", "live", "live"), timeout=10, desc="quota back")
        assert rq["metadata"]["uid"] != first["metadata"]["uid"]
        assert rq["spec"]["hard"]["requests.amd.com/gpu"] == "2"
        assert c.procs["controller"].alive()
        assert "being terminated" not in c.procs["controller"].output()

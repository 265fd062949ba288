"""Real-apiserver semantics the product depends on, each with the
controller and synchronizer converging through it:

* opaque (non-numeric) resourceVersions;
* paginated LIST (limit/continue) from a consistent snapshot, expired continue -> 410;
* HTTP 410 at watch start (not only an ERROR event in the stream);
* streaming lists: sendInitialEvents + the k8s.io/initial-events-end BOOKMARK;
* 429 Too Many Requests with Retry-After, honoured by the client;
* a non-force server-side apply that conflicts with another field manager -> 409.

Reference call sites: watcher/reflector (src/controller.rs:233-246), SSA with force
(src/controller.rs:67), replace_status + JSON patch (src/synchronizer.rs:217,302-330)."""
import json
import time

import pytest
import requests

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle
from bacchus_gpu_controller_amd.testing.kubeapi import ApiError, wait_for

pytestmark = pytest.mark.slow


def ub(name, **spec):
    return {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": name},
            "spec": spec or {"kube_username": name}}


def metric(port, name):
    text = requests.get(f"http://127.0.0.1:{port}/metrics", timeout=5).text
    total = 0.0
    for line in text.splitlines():
        if line.startswith(name) and not line.startswith("#"):
            total += float(line.rsplit(" ", 1)[1])
    return total


@pytest.fixture()
def google():
    g = FakeGoogle().start()
    yield g
    g.stop()


def test_opaque_resource_versions_onboarding_converges(google):
    google.set_rows([{"id_username": "opaq", "gpu": 2}])
    with Cluster(apiserver_args=["--opaque-rv"], controller_env={"CONF_REQUEUE_SECS": "3600"}) as c:
        c.as_user("oidc:opaq", ["gpu"]).create("userbootstraps", ub("opaq") | {"spec": {}})
        c.start_synchronizer(google, interval=1, extra_env={"CONF_WATCH": "true"})
        rb = wait_for(lambda: c.admin.get_or_none("rolebindings", "opaq", "opaq"), timeout=15, desc="rolebinding")
        assert rb["metadata"]["resourceVersion"].startswith("kl.")
        rq = c.admin.get("resourcequotas", "opaq", "opaq")
        assert rq["spec"]["hard"]["requests.amd.com/gpu"] == "2"
        # resume + relist with opaque versions: compaction forces every watcher to re-list
        c.compact_and_drop_watches()
        time.sleep(0.3)
        c.as_user("oidc:opaq2", ["gpu"]).create("userbootstraps", ub("opaq2") | {"spec": {}})
        wait_for(lambda: c.admin.get_or_none("namespaces", "opaq2"), timeout=15, desc="after relist")
        # a numeric resourceVersion was never issued by this server
        r = requests.get(c.server + "/apis/bacchus.io/v1/userbootstraps?watch=1&resourceVersion=12",
                         headers={"Authorization": "Bearer admin-token"}, timeout=5)
        assert r.status_code == 400
        assert c.procs["controller"].alive() and c.procs["synchronizer"].alive()


def test_paginated_list_snapshot_and_expired_continue():
    with Cluster(admission=False, controller=False, apiserver_args=["--continue-ttl-ms", "1500"]) as c:
        for i in range(25):
            c.admin.create("userbootstraps", ub(f"p{i:02d}"))
        base = c.server + "/apis/bacchus.io/v1/userbootstraps"
        h = {"Authorization": "Bearer admin-token"}
        p1 = requests.get(base + "?limit=10", headers=h, timeout=5).json()
        assert len(p1["items"]) == 10 and p1["metadata"]["remainingItemCount"] == 15
        rv1 = p1["metadata"]["resourceVersion"]
        c.admin.create("userbootstraps", ub("p00a"))  # after the snapshot: not in later pages
        names = [x["metadata"]["name"] for x in p1["items"]]
        tok = p1["metadata"]["continue"]
        while tok:
            pg = requests.get(base + "?limit=10&continue=" + tok, headers=h, timeout=5).json()
            assert pg["metadata"]["resourceVersion"] == rv1
            names += [x["metadata"]["name"] for x in pg["items"]]
            tok = pg["metadata"].get("continue")
        assert names == [f"p{i:02d}" for i in range(25)]
        p1 = requests.get(base + "?limit=5", headers=h, timeout=5).json()
        time.sleep(2.0)
        r = requests.get(base + "?limit=5&continue=" + p1["metadata"]["continue"], headers=h, timeout=5)
        assert r.status_code == 410 and r.json()["reason"] == "Expired"
        # the controller lists in pages of 7 and still provisions everyone
        pages0 = c.stats()["list_pages"]
        c.start_controller(extra_env={"CONF_LIST_PAGE_SIZE": "7", "CONF_REQUEUE_SECS": "3600"})
        wait_for(lambda: all(c.admin.get_or_none("namespaces", f"p{i:02d}") for i in range(25)), timeout=20,
                 desc="all namespaces")
        assert c.stats()["list_pages"] - pages0 >= 4  # 26 UBs / 7 per page


def test_http_410_at_watch_start_relists():
    with Cluster(admission=False, controller_env={"CONF_REQUEUE_SECS": "3600"}) as c:
        c.admin.create("userbootstraps", ub("g1"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "g1"), desc="g1")
        # the next 3 watch requests for userbootstraps fail with HTTP 410 (no stream at all)
        c.fault([{"method": "GET", "path": "userbootstraps.*watch=1", "status": 410, "count": 3}])
        c.compact_and_drop_watches()
        c.admin.create("userbootstraps", ub("g2"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "g2"), timeout=15, desc="g2 after 410s")
        # g2 can arrive with the relist after the second 410; the third follows that list
        wait_for(lambda: c.stats()["faults_hit"] >= 3, timeout=10, desc="all three 410s served")
        assert metric(c.controller_port, 'bgc_watch_errors_total{resource="userbootstraps"}') >= 3


def test_streaming_lists_initial_events_end_bookmark():
    with Cluster(admission=False, controller=False) as c:
        for i in range(5):
            c.admin.create("userbootstraps", ub(f"s{i}"))
        base = c.server + "/apis/bacchus.io/v1/userbootstraps?watch=1&allowWatchBookmarks=true"
        h = {"Authorization": "Bearer admin-token"}
        r = requests.get(base + "&sendInitialEvents=true", headers=h, timeout=5)
        assert r.status_code == 422  # resourceVersionMatch=NotOlderThan is required
        with requests.get(base + "&sendInitialEvents=true&resourceVersionMatch=NotOlderThan&timeoutSeconds=1",
                          headers=h, stream=True, timeout=10) as r:
            events = [json.loads(line) for line in r.iter_lines() if line]
        added = [e["object"]["metadata"]["name"] for e in events if e["type"] == "ADDED"]
        bm = [e for e in events if e["type"] == "BOOKMARK"]
        assert sorted(added) == [f"s{i}" for i in range(5)]
        assert bm[0]["object"]["metadata"]["annotations"] == {"k8s.io/initial-events-end": "true"}
        assert events.index(bm[0]) == 5  # after every initial ADDED
        # the controller gets its initial state from streaming lists: no LIST request at all
        pages0 = c.stats()["list_pages"]
        c.start_controller(extra_env={"CONF_STREAMING_LISTS": "true", "CONF_REQUEUE_SECS": "3600"})
        wait_for(lambda: all(c.admin.get_or_none("namespaces", f"s{i}") for i in range(5)), desc="pre-existing UBs")
        c.admin.create("userbootstraps", ub("s9"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "s9"), desc="new UB")
        assert c.stats()["list_pages"] == pages0


def test_429_retry_after_is_honoured(google):
    google.set_rows([{"id_username": "thr", "gpu": 1}])
    with Cluster(admission=False, controller_env={"CONF_REQUEUE_SECS": "3600", "CONF_ERROR_REQUEUE_MS": "60000"}) as c:
        # two throttled answers for the namespace apply, one for the status PUT
        c.fault([{"method": "PATCH", "path": "/api/v1/namespaces/thr", "status": 429, "retry_after": 1, "count": 2},
                 {"method": "PUT", "path": "userbootstraps/thr/status", "status": 429, "retry_after": 1, "count": 1}])
        t0 = time.time()
        c.admin.create("userbootstraps", ub("thr"))
        # the error requeue is 60 s: converging within ~2 s proves the client retried itself
        wait_for(lambda: c.admin.get_or_none("namespaces", "thr"), timeout=10, desc="namespace after 429s")
        assert time.time() - t0 >= 1.9
        assert metric(c.controller_port, "bgc_kube_client_throttled_total") == 2
        assert metric(c.controller_port, 'bgc_reconcile_total{result="error"}') == 0
        c.start_synchronizer(google, interval=60)
        wait_for(lambda: c.admin.get("userbootstraps", "thr").get("status", {}).get("synchronized_with_sheet"),
                 timeout=10, desc="status after 429")
        assert metric(c.sync_port, "bgc_kube_client_throttled_total") == 1
        assert c.procs["synchronizer"].alive()


def test_non_force_apply_conflict_and_forced_reclaim():
    with Cluster(admission=False, controller_env={"CONF_REQUEUE_SECS": "3600"}) as c:
        c.admin.create("userbootstraps", ub("cf", kube_username="cf", quota={"hard": {"requests.cpu": "8"}}))
        wait_for(lambda: c.admin.get_or_none("resourcequotas", "cf", "cf"), desc="quota")
        url = c.server + "/api/v1/namespaces/cf/resourcequotas/cf?fieldManager=kubectl"
        h = {"Authorization": "Bearer admin-token", "Content-Type": "application/apply-patch+yaml"}
        body = {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "cf", "namespace": "cf"},
                "spec": {"hard": {"requests.cpu": "64"}}}
        r = requests.patch(url, data=json.dumps(body), headers=h, timeout=5)
        assert r.status_code == 409 and "conflict with" in r.json()["message"]
        assert "bacchus-gpu-controller.bacchus.io" in r.json()["message"]
        r = requests.patch(url + "&force=true", data=json.dumps(body), headers=h, timeout=5)
        assert r.status_code == 200 and r.json()["spec"]["hard"]["requests.cpu"] == "64"
        # the foreign change is a child MODIFIED event: the controller re-applies with force
        # and takes the field back (drift repair without waiting for the 30 s requeue)
        rq = wait_for(lambda: (lambda q: q if q["spec"]["hard"]["requests.cpu"] == "8" else None)(
            c.admin.get("resourcequotas", "cf", "cf")), desc="reclaimed")
        managers = {m["manager"] for m in rq["metadata"]["managedFields"]}
        assert "bacchus-gpu-controller.bacchus.io" in managers


def test_streaming_lists_fall_back_to_list_when_rejected():
    """An apiserver without the WatchList feature rejects sendInitialEvents: the watcher
    falls back to a (paginated) LIST for good and the controller still converges."""
    with Cluster(admission=False, controller=False) as c:
        c.admin.create("userbootstraps", ub("fb1"))
        c.fault([{"method": "GET", "path": "sendInitialEvents=true", "status": 400,
                  "message": "sendInitialEvents is forbidden for watch unless the WatchList feature gate is enabled"}])
        pages0 = c.stats()["list_pages"]
        c.start_controller(extra_env={"CONF_STREAMING_LISTS": "true", "CONF_REQUEUE_SECS": "3600"})
        wait_for(lambda: c.admin.get_or_none("namespaces", "fb1"), timeout=15, desc="fb1 via LIST fallback")
        c.admin.create("userbootstraps", ub("fb2"))
        wait_for(lambda: c.admin.get_or_none("namespaces", "fb2"), timeout=15, desc="fb2 via watch")
        assert c.stats()["list_pages"] - pages0 >= 5  # UB + 4 owned kinds listed after the fallback
        assert c.stats()["faults_hit"] >= 5


META = "application/json;as=PartialObjectMetadata;g=meta.k8s.io;v=v1,application/json"
META_LIST = "application/json;as=PartialObjectMetadataList;g=meta.k8s.io;v=v1,application/json"


def test_partial_object_metadata_get_list_watch():
    """metadata-only clients (client-go metadata informers, kube-rs metadata_watcher): the
    apiserver answers GET/LIST/WATCH with PartialObjectMetadata(List) when asked by Accept."""
    with Cluster(admission=False, controller=False) as c:
        c.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace",
                                      "metadata": {"name": "pm1", "labels": {"a": "b"}}})
        c.admin.create("resourcequotas", {"apiVersion": "v1", "kind": "ResourceQuota",
                                          "metadata": {"name": "q", "namespace": "pm1"},
                                          "spec": {"hard": {"requests.amd.com/gpu": "2"}}}, namespace="pm1")
        h = {"Authorization": "Bearer admin-token"}
        url = c.server + "/api/v1/namespaces/pm1/resourcequotas"
        o = requests.get(url + "/q", headers={**h, "Accept": META}, timeout=5).json()
        assert (o["kind"], o["apiVersion"]) == ("PartialObjectMetadata", "meta.k8s.io/v1")
        assert o["metadata"]["name"] == "q" and "spec" not in o
        full = requests.get(url + "/q", headers=h, timeout=5).json()
        assert full["spec"]["hard"] == {"requests.amd.com/gpu": "2"}
        assert o["metadata"]["resourceVersion"] == full["metadata"]["resourceVersion"]
        lst = requests.get(c.server + "/api/v1/namespaces?labelSelector=a%3Db",
                           headers={**h, "Accept": META_LIST}, timeout=5).json()
        assert (lst["kind"], lst["apiVersion"]) == ("PartialObjectMetadataList", "meta.k8s.io/v1")
        assert [i["metadata"]["name"] for i in lst["items"]] == ["pm1"]
        assert all(i["kind"] == "PartialObjectMetadata" and set(i) == {"kind", "apiVersion", "metadata"}
                   for i in lst["items"])
        rv = lst["metadata"]["resourceVersion"]
        # a resumed watch (history) and the live stream both carry metadata only
        c.admin.merge_patch("resourcequotas", "q", {"spec": {"hard": {"requests.amd.com/gpu": "4"}}}, namespace="pm1")
        with requests.get(url + f"?watch=1&resourceVersion={rv}&timeoutSeconds=1",
                          headers={**h, "Accept": META}, stream=True, timeout=10) as r:
            events = [json.loads(line) for line in r.iter_lines() if line]
        mods = [e for e in events if e["type"] == "MODIFIED"]
        assert mods and all(set(e["object"]) == {"kind", "apiVersion", "metadata"} for e in mods)
        assert mods[-1]["object"]["metadata"]["name"] == "q"


@pytest.mark.parametrize("metadata_watches", ["true", "false"])
def test_controller_converges_with_metadata_child_watches(metadata_watches):
    with Cluster(admission=False, controller_env={"CONF_METADATA_WATCHES": metadata_watches,
                                                  "CONF_REQUEUE_SECS": "3600"}) as c:
        c.admin.create("userbootstraps", ub("mw1", quota={"hard": {"requests.amd.com/gpu": "1"}}))
        wait_for(lambda: c.admin.get_or_none("resourcequotas", "mw1", "mw1"), desc="quota")
        # drift on a child is repaired (the MODIFIED event of a metadata watch is enough)
        c.admin.merge_patch("resourcequotas", "mw1", {"spec": {"hard": {"requests.amd.com/gpu": "7"}}}, namespace="mw1")
        wait_for(lambda: c.admin.get("resourcequotas", "mw1", "mw1")["spec"]["hard"] == {"requests.amd.com/gpu": "1"},
                 timeout=15, desc="drift repaired")
        # a deleted child is re-created
        uid = c.admin.get("resourcequotas", "mw1", "mw1")["metadata"]["uid"]
        c.admin.delete("resourcequotas", "mw1", namespace="mw1")
        wait_for(lambda: (c.admin.get_or_none("resourcequotas", "mw1", "mw1") or {"metadata": {"uid": uid}})
                 ["metadata"]["uid"] != uid, timeout=15, desc="re-created")


def test_deleted_event_carries_the_last_object_at_the_deletion_version():
    """A DELETED watch event carries the object as last stored (managedFields and all) at
    the deletion's resourceVersion; kube-lite reuses the last commit's serialization for it."""
    with Cluster(admission=False, controller=False) as c:
        c.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "dw"}})
        rq = {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q", "namespace": "dw",
                                                                        "labels": {"a": "b"}},
              "spec": {"hard": {"requests.amd.com/gpu": "1"}}}
        c.admin.apply("resourcequotas", "q", rq, "mgr-1", namespace="dw")
        rq["spec"]["hard"]["requests.amd.com/gpu"] = "2"
        last = c.admin.apply("resourcequotas", "q", rq, "mgr-1", namespace="dw")
        c.admin.merge_patch("resourcequotas", "q", {"metadata": {"annotations": {"x": "y"}}}, namespace="dw",
                            field_manager="mgr-2")
        last = c.admin.get("resourcequotas", "q", "dw")
        start = last["metadata"]["resourceVersion"]
        with requests.get(f"{c.server}/api/v1/namespaces/dw/resourcequotas",
                          params={"watch": "true", "resourceVersion": start, "timeoutSeconds": "10"},
                          headers={"Authorization": c.admin.s.headers["Authorization"]}, stream=True,
                          timeout=15, verify=c.verify) as r:
            time.sleep(0.2)
            c.admin.delete("resourcequotas", "q", "dw")
            ev = None
            for line in r.iter_lines():
                if line:
                    ev = json.loads(line)
                    if ev["type"] == "DELETED":
                        break
        assert ev and ev["type"] == "DELETED"
        got = ev["object"]
        assert int(got["metadata"].pop("resourceVersion")) > int(last["metadata"].pop("resourceVersion"))
        assert got == last
        assert {m["manager"] for m in got["metadata"]["managedFields"]} == {"mgr-1", "mgr-2"}

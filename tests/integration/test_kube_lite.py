"""kube-lite fidelity: the API semantics the components rely on (SSA ownership and
conflicts, optimistic concurrency, status subresource, generation, finalizers, GC,
namespace scoping, watch resume)."""
import json
import threading

import pytest
import requests

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import ApiError, wait_for

pytestmark = pytest.mark.slow


@pytest.fixture(scope="module")
def c():
    with Cluster(admission=False, controller=False) as cl:
        yield cl


def ns(c, name):
    c.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": name}})


def test_ssa_conflict_and_force(c):
    ns(c, "ssa")
    body = {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q"}, "spec": {"hard": {"cpu": "1"}}}
    c.admin.apply("resourcequotas", "q", body, "mgr-a", namespace="ssa")
    body2 = {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q"}, "spec": {"hard": {"cpu": "2"}}}
    with pytest.raises(ApiError) as e:
        c.admin.apply("resourcequotas", "q", body2, "mgr-b", namespace="ssa")
    assert e.value.code == 409 and 'conflict with "mgr-a"' in e.value.message and ".spec.hard.cpu" in e.value.message
    out = c.admin.apply("resourcequotas", "q", body2, "mgr-b", force=True, namespace="ssa")
    assert out["spec"]["hard"]["cpu"] == "2"
    owners = {m["manager"]: m for m in out["metadata"]["managedFields"]}
    assert "mgr-b" in owners and "mgr-a" not in owners


def test_ssa_prunes_fields_no_longer_applied(c):
    ns(c, "prune")
    c.admin.apply("resourcequotas", "q", {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q"},
                                          "spec": {"hard": {"cpu": "1", "memory": "1Gi"}}}, "m", namespace="prune")
    out = c.admin.apply("resourcequotas", "q", {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q"},
                                                "spec": {"hard": {"cpu": "1"}}}, "m", namespace="prune")
    assert out["spec"]["hard"] == {"cpu": "1"}


def test_ssa_noop_keeps_resource_version(c):
    ns(c, "noop")
    b = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x"}, "data": {"a": "1"}}
    r1 = c.admin.apply("configmaps", "x", b, "m", namespace="noop")
    r2 = c.admin.apply("configmaps", "x", b, "m", namespace="noop")
    assert r1["metadata"]["resourceVersion"] == r2["metadata"]["resourceVersion"]


def test_optimistic_concurrency_and_status_subresource(c):
    obj = c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                            "metadata": {"name": "occ"}, "spec": {"kube_username": "occ"},
                                            "status": {"synchronized_with_sheet": True}})
    assert "status" not in obj                       # status ignored on create
    assert obj["metadata"]["generation"] == 1
    rv = obj["metadata"]["resourceVersion"]
    st = c.admin.replace("userbootstraps", "occ", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                                   "metadata": {"name": "occ", "resourceVersion": rv},
                                                   "status": {"synchronized_with_sheet": True}}, sub="status")
    assert st["status"]["synchronized_with_sheet"] is True and st["metadata"]["generation"] == 1
    with pytest.raises(ApiError) as e:                # stale resourceVersion
        c.admin.replace("userbootstraps", "occ", dict(obj, metadata={"name": "occ", "resourceVersion": rv}), sub="status")
    assert e.value.code == 409
    # main-resource writes can't touch status, and bump generation on spec change
    p = c.admin.merge_patch("userbootstraps", "occ", {"spec": {"kube_username": "occ2"},
                                                      "status": {"synchronized_with_sheet": False}})
    assert p["status"]["synchronized_with_sheet"] is True and p["metadata"]["generation"] == 2


def test_status_writes_own_only_status_fields(c):
    c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                      "metadata": {"name": "stown"}, "spec": {"kube_username": "stown"}},
                   field_manager="creator")
    c.admin.merge_patch("userbootstraps", "stown", {"status": {"synchronized_with_sheet": True, "note": "x"}},
                        sub="status", field_manager="st-mgr")
    o = c.admin.merge_patch("userbootstraps", "stown", {"status": {"note": None}}, sub="status",
                            field_manager="st-mgr2")
    by = {(m["manager"], m.get("subresource", "")): m for m in o["metadata"]["managedFields"]}
    assert by[("creator", "")]["fieldsV1"] == {"f:spec": {"f:kube_username": {}}}
    st = by[("st-mgr", "status")]
    assert st["operation"] == "Update" and st["fieldsV1"] == {"f:status": {"f:synchronized_with_sheet": {}}}
    # removing a status leaf drops it from its owner; a write that changes nothing owns nothing
    assert ("st-mgr2", "status") not in by


def test_namespaced_create_requires_namespace(c):
    with pytest.raises(ApiError) as e:
        c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x"}},
                       namespace="does-not-exist")
    assert e.value.code == 404 and 'namespaces "does-not-exist" not found' in e.value.message


def test_finalizers_and_gc(c):
    ns(c, "fin")
    owner = c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap",
                                          "metadata": {"name": "owner", "finalizers": ["x/y"]}}, namespace="fin")
    c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {
        "name": "dep", "ownerReferences": [{"apiVersion": "v1", "kind": "ConfigMap", "name": "owner",
                                            "uid": owner["metadata"]["uid"]}]}}, namespace="fin")
    c.admin.delete("configmaps", "owner", namespace="fin")
    o = c.admin.get("configmaps", "owner", namespace="fin")
    assert "deletionTimestamp" in o["metadata"]          # held by the finalizer
    assert c.admin.get_or_none("configmaps", "dep", namespace="fin") is not None
    c.admin.json_patch("configmaps", "owner", [{"op": "remove", "path": "/metadata/finalizers"}], namespace="fin")
    wait_for(lambda: c.admin.get_or_none("configmaps", "owner", namespace="fin") is None, desc="owner gone")
    wait_for(lambda: c.admin.get_or_none("configmaps", "dep", namespace="fin") is None, desc="dependent GC")


def test_watch_resume_and_bookmarks(c):
    lst = c.admin.list("namespaces")
    rv = lst["metadata"]["resourceVersion"]
    events = []

    def watch():
        with requests.get(c.server + f"/api/v1/namespaces?watch=1&resourceVersion={rv}&allowWatchBookmarks=true"
                                      "&timeoutSeconds=3", headers={"Authorization": "Bearer admin-token"},
                          stream=True, timeout=10) as r:
            for line in r.iter_lines():
                if line:
                    events.append(json.loads(line))

    t = threading.Thread(target=watch)
    t.start()
    ns(c, "watched")
    t.join(10)
    types = [e["type"] for e in events]
    assert "ADDED" in types and "BOOKMARK" in types
    added = [e for e in events if e["type"] == "ADDED"]
    assert added[0]["object"]["metadata"]["name"] == "watched"


def test_impersonation_requires_masters(c):
    from bacchus_gpu_controller_amd.testing.kubeapi import KubeApi
    api = KubeApi(c.server, "controller-token", as_user="oidc:x")
    with pytest.raises(ApiError) as e:
        api.list("namespaces")
    assert e.value.code == 403
    with pytest.raises(ApiError) as e2:
        KubeApi(c.server, "bogus").list("namespaces")
    assert e2.value.code == 401


def test_label_and_field_selectors(c):
    ns(c, "sel")
    for i, tier in enumerate(["gold", "silver", "gold"]):
        c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap",
                                      "metadata": {"name": f"s{i}", "labels": {"tier": tier}}}, namespace="sel")
    gold = c.admin.list("configmaps", namespace="sel", label_selector="tier=gold")
    assert [i["metadata"]["name"] for i in gold["items"]] == ["s0", "s2"]
    notgold = c.admin.list("configmaps", namespace="sel", label_selector="tier notin (gold)")
    assert [i["metadata"]["name"] for i in notgold["items"]] == ["s1"]


def test_name_prefix_test_extension_filters_list_and_watch(c):
    """kube-lite.test/name-prefix (the bench's per-rank driver filter) on LIST, on a watch's
    history replay and on live events."""
    sel = "kube-lite.test/name-prefix=pfa-"
    rv = c.admin.list("namespaces")["metadata"]["resourceVersion"]
    for n in ("pfa-1", "pfb-1", "pfa-2"):
        ns(c, n)
    names = [i["metadata"]["name"] for i in c.admin.list("namespaces", field_selector=sel)["items"]]
    assert names == ["pfa-1", "pfa-2"]
    events = []

    def watch():  # starts at rv: the three creates are replayed from history, then live
        with requests.get(c.server + f"/api/v1/namespaces?watch=1&resourceVersion={rv}&timeoutSeconds=3"
                                     f"&fieldSelector={sel}", headers={"Authorization": "Bearer admin-token"},
                          stream=True, timeout=10) as r:
            for line in r.iter_lines():
                if line:
                    events.append(json.loads(line))

    t = threading.Thread(target=watch)
    t.start()
    ns(c, "pfb-2")
    ns(c, "pfa-3")
    t.join(10)
    assert [e["object"]["metadata"]["name"] for e in events if e["type"] == "ADDED"] == ["pfa-1", "pfa-2", "pfa-3"]


def _watch_lines(c, path, rv, seconds):
    out = []
    with requests.get(c.server + f"{path}?watch=1&resourceVersion={rv}&timeoutSeconds={seconds}",
                      headers={"Authorization": "Bearer admin-token"}, stream=True, timeout=seconds + 10) as r:
        for line in r.iter_lines():
            if line:
                out.append(json.loads(line))
    return out


def test_namespace_deletion_cascades_across_types(c):
    ns(c, "casc")
    for i in range(5):
        c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": f"cm{i}"}},
                       namespace="casc")
    c.admin.create("resourcequotas", {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q"},
                                      "spec": {"hard": {"requests.amd.com/gpu": "1"}}}, namespace="casc")
    c.admin.delete("namespaces", "casc")
    wait_for(lambda: not c.admin.list("configmaps", namespace="casc")["items"], desc="configmaps collected")
    wait_for(lambda: c.admin.get_or_none("resourcequotas", "q", namespace="casc") is None, desc="quota collected")


def test_gc_cascades_through_owner_chain(c):
    """owner (ConfigMap) -> Secret -> ConfigMap: deleting the root collects both levels (the
    background collector handles each type under its own lock)."""
    ns(c, "chain")
    root = c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "root"}},
                          namespace="chain")
    mid = c.admin.create("secrets", {"apiVersion": "v1", "kind": "Secret", "metadata": {
        "name": "mid", "ownerReferences": [{"apiVersion": "v1", "kind": "ConfigMap", "name": "root",
                                            "uid": root["metadata"]["uid"]}]}}, namespace="chain")
    c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {
        "name": "leaf", "ownerReferences": [{"apiVersion": "v1", "kind": "Secret", "name": "mid",
                                             "uid": mid["metadata"]["uid"]}]}}, namespace="chain")
    c.admin.delete("configmaps", "root", namespace="chain")
    wait_for(lambda: c.admin.get_or_none("secrets", "mid", namespace="chain") is None, desc="mid collected")
    wait_for(lambda: c.admin.get_or_none("configmaps", "leaf", namespace="chain") is None, desc="leaf collected")
    assert c.stats()["gc_collected"] >= 2


def test_concurrent_writers_keep_per_type_watch_order(c):
    """Writers on two types at once (per-type shards, one global resourceVersion): a watch on
    one type sees each of its events exactly once, in increasing resourceVersion order, and a
    resume from a mid-stream resourceVersion yields exactly the suffix."""
    ns(c, "order")
    rv0 = c.admin.list("configmaps", namespace="order")["metadata"]["resourceVersion"]
    n_threads, per = 4, 25

    def cm_writer(t):
        for i in range(per):
            c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap",
                                          "metadata": {"name": f"w{t}-{i}"}}, namespace="order")

    def ns_writer(t):
        for i in range(per):
            ns(c, f"order-ns-{t}-{i}")

    threads = [threading.Thread(target=cm_writer, args=(t,)) for t in range(n_threads)]
    threads += [threading.Thread(target=ns_writer, args=(t,)) for t in range(n_threads)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    events = [e for e in _watch_lines(c, "/api/v1/namespaces/order/configmaps", rv0, 2) if e["type"] == "ADDED"]
    names = [e["object"]["metadata"]["name"] for e in events]
    rvs = [int(e["object"]["metadata"]["resourceVersion"]) for e in events]
    assert sorted(names) == sorted(f"w{t}-{i}" for t in range(n_threads) for i in range(per))
    assert rvs == sorted(rvs) and len(set(rvs)) == len(rvs)
    mid = rvs[len(rvs) // 2]
    suffix = [e for e in _watch_lines(c, "/api/v1/namespaces/order/configmaps", mid, 2) if e["type"] == "ADDED"]
    assert [int(e["object"]["metadata"]["resourceVersion"]) for e in suffix] == [r for r in rvs if r > mid]


def test_watch_coalescing_switches_at_run_time(c):
    """POST /_kl/watch-coalesce-us sets how long a watch writer waits for a burst to grow
    (the bench turns it off for its open-loop windows and restores it): it answers the
    previous value, rejects nonsense, and watches deliver every event either way."""
    url = c.server + "/_kl/watch-coalesce-us"
    kw = {"headers": {"Authorization": "Bearer admin-token"}, "timeout": 5}
    assert requests.post(url, data="x", **kw).status_code == 400
    assert requests.post(url, data="-1", **kw).status_code == 400
    prev = requests.post(url, data="0", **kw)
    assert prev.status_code == 200 and prev.text.strip() == "50"  # kube-lite's default
    try:
        for setting in ("0", "2000"):  # off, and a long hold the burst cannot outlast
            assert requests.post(url, data=setting, **kw).status_code == 200
            rv = c.admin.list("namespaces")["metadata"]["resourceVersion"]
            names = [f"co{setting}-{i}" for i in range(5)]
            got = []
            t = threading.Thread(target=lambda: got.extend(_watch_lines(c, "/api/v1/namespaces", rv, 2)))
            t.start()
            for n in names:
                ns(c, n)
            t.join(15)
            assert [e["object"]["metadata"]["name"] for e in got if e["type"] == "ADDED"] == names
    finally:
        assert requests.post(url, data="50", **kw).text.strip() == "2000"

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

"""kube-lite: label-selector watches across label changes ("next round" #2).

A real apiserver's watch cache delivers an update that moves an object out of a watch's
label selector as DELETED (with the previous object, at the event's resourceVersion) and one
that moves it in as ADDED (k8s.io/apiserver cacheWatcher.convertToWatchEvent).  The
controller's label-selected child watches rely on that to see a child whose label was
stripped.  `--no-selector-transitions` drops those events instead, to model a lost event.
"""
import json
import threading
import time

import pytest
import requests

from bacchus_gpu_controller_amd.testing.cluster import ADMIN_TOKEN, Cluster

pytestmark = pytest.mark.slow

SEL = "team=a"
META_ACCEPT = "application/json;as=PartialObjectMetadata;g=meta.k8s.io;v=v1,application/json"


@pytest.fixture(scope="module")
def c():
    with Cluster(admission=False, controller=False) as cl:
        yield cl


@pytest.fixture(scope="module")
def lossy():
    with Cluster(admission=False, controller=False, apiserver_args=["--no-selector-transitions"]) as cl:
        yield cl


def _watch(c, path, rv, seconds, meta=False):
    headers = {"Authorization": f"Bearer {ADMIN_TOKEN}"}
    if meta:
        headers["Accept"] = META_ACCEPT
    out = []
    with requests.get(c.server + f"{path}?watch=1&resourceVersion={rv}&timeoutSeconds={seconds}"
                      f"&labelSelector={SEL}", headers=headers, stream=True, timeout=seconds + 10) as r:
        for line in r.iter_lines():
            if line:
                out.append(json.loads(line))
    return out


def _churn(c, ns):
    """create labelled; relabel out (and change data); relabel in; change data; delete."""
    base = f"/api/v1/namespaces/{ns}/configmaps"
    c.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    rv0 = c.admin.list("configmaps", namespace=ns)["metadata"]["resourceVersion"]
    cm = c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap",
                                       "metadata": {"name": "x", "labels": {"team": "a"}}, "data": {"v": "1"}},
                        namespace=ns)
    out = c.admin.merge_patch("configmaps", "x", {"metadata": {"labels": {"team": None}}, "data": {"v": "2"}},
                              namespace=ns)
    back = c.admin.merge_patch("configmaps", "x", {"metadata": {"labels": {"team": "a"}}}, namespace=ns)
    data = c.admin.merge_patch("configmaps", "x", {"data": {"v": "3"}}, namespace=ns)
    c.admin.delete("configmaps", "x", namespace=ns)
    return base, rv0, [cm, out, back, data]


def _check_transitions(events, versions, meta=False):
    cm, out, back, data = versions
    types = [e["type"] for e in events if e["type"] != "BOOKMARK"]
    assert types == ["ADDED", "DELETED", "ADDED", "MODIFIED", "DELETED"], types
    ev = [e for e in events if e["type"] != "BOOKMARK"]
    gone = ev[1]["object"]
    # the object as it was before it left the selector, at the leaving event's version
    assert gone["metadata"]["labels"] == {"team": "a"}
    assert gone["metadata"]["resourceVersion"] == out["metadata"]["resourceVersion"]
    if meta:
        assert gone["kind"] == "PartialObjectMetadata" and "data" not in gone
    else:
        assert gone["data"] == {"v": "1"}
    assert ev[2]["object"]["metadata"]["resourceVersion"] == back["metadata"]["resourceVersion"]
    assert ev[3]["object"]["metadata"]["resourceVersion"] == data["metadata"]["resourceVersion"]


@pytest.mark.parametrize("meta", [False, True])
def test_history_replay_emits_transitions(c, meta):
    base, rv0, versions = _churn(c, f"hist-{int(meta)}")
    _check_transitions(_watch(c, base, rv0, 1, meta=meta), versions, meta=meta)


def test_live_watch_emits_transitions(c):
    ns = "live"
    c.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    rv0 = c.admin.list("configmaps", namespace=ns)["metadata"]["resourceVersion"]
    got = {}
    t = threading.Thread(target=lambda: got.setdefault("ev", _watch(c, f"/api/v1/namespaces/{ns}/configmaps", rv0, 3)))
    t.start()
    time.sleep(0.5)  # the watch is registered: everything below arrives live
    cm = c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap",
                                       "metadata": {"name": "x", "labels": {"team": "a"}}, "data": {"v": "1"}},
                        namespace=ns)
    out = c.admin.merge_patch("configmaps", "x", {"metadata": {"labels": {"team": None}}, "data": {"v": "2"}},
                              namespace=ns)
    back = c.admin.merge_patch("configmaps", "x", {"metadata": {"labels": {"team": "a"}}}, namespace=ns)
    data = c.admin.merge_patch("configmaps", "x", {"data": {"v": "3"}}, namespace=ns)
    c.admin.delete("configmaps", "x", namespace=ns)
    t.join()
    _check_transitions(got["ev"], [cm, out, back, data])


def test_unselected_watch_sees_plain_modifications(c):
    base, rv0, _ = _churn(c, "plain")
    headers = {"Authorization": f"Bearer {ADMIN_TOKEN}"}
    with requests.get(c.server + f"{base}?watch=1&resourceVersion={rv0}&timeoutSeconds=1", headers=headers,
                      stream=True, timeout=10) as r:
        types = [json.loads(l)["type"] for l in r.iter_lines() if l]
    assert [t for t in types if t != "BOOKMARK"] == ["ADDED", "MODIFIED", "MODIFIED", "MODIFIED", "DELETED"]


def test_lossy_mode_drops_transition_events(lossy):
    base, rv0, _ = _churn(lossy, "lossy")
    types = [e["type"] for e in _watch(lossy, base, rv0, 1) if e["type"] != "BOOKMARK"]
    # leaving the selector is never delivered; re-entering is a MODIFIED of an unknown object
    assert types == ["ADDED", "MODIFIED", "MODIFIED", "DELETED"], types


def test_events_after_compaction_serialize_the_object_anew(c):
    """the store no longer pins each live object's last event line; once
    the history has dropped it, a DELETED event and a selector transition are serialized
    from the stored object instead, with the same content."""
    ns = "compacted"
    c.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    for n in ("a", "b"):
        c.admin.create("configmaps", {"apiVersion": "v1", "kind": "ConfigMap",
                                      "metadata": {"name": n, "labels": {"team": "a"}}, "data": {"v": n}}, namespace=ns)
    requests.post(c.server + "/_kl/compact", timeout=5).raise_for_status()
    rv0 = c.admin.list("configmaps", namespace=ns)["metadata"]["resourceVersion"]
    out = c.admin.merge_patch("configmaps", "a", {"metadata": {"labels": {"team": None}}}, namespace=ns)
    c.admin.delete("configmaps", "b", namespace=ns)
    ev = [e for e in _watch(c, f"/api/v1/namespaces/{ns}/configmaps", rv0, 1) if e["type"] != "BOOKMARK"]
    assert [e["type"] for e in ev] == ["DELETED", "DELETED"]
    assert ev[0]["object"]["metadata"]["name"] == "a" and ev[0]["object"]["data"] == {"v": "a"}
    assert ev[0]["object"]["metadata"]["labels"] == {"team": "a"}
    assert ev[0]["object"]["metadata"]["resourceVersion"] == out["metadata"]["resourceVersion"]
    assert ev[1]["object"]["metadata"]["name"] == "b" and ev[1]["object"]["data"] == {"v": "b"}

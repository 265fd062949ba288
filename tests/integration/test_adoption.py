"""Adopting a cluster the reference controller managed.

The reference applies children with no labels (/root/reference/src/controller.rs:70-77,
91-99,131-139) and its .owns() watches every object of each kind (controller.rs:234-238).
This build labels its children app.kubernetes.io/managed-by=bacchus-gpu-controller and
its child watches select on that label, so after `helm upgrade` from the reference the
existing children are at first invisible to those watches.  Adoption relies on the first
pass after start-up: every UserBootstrap is listed and reconciled, and the apply (same
field manager, force) adds the label to each existing child in place.

The reference-managed state is produced by this stack running the reference's controller
behaviour (CONF_LABEL_CHILDREN=false, CONF_SKIP_UNCHANGED=false, CONF_PARALLEL_CHILDREN=false:
unlabelled children, sequential unconditional applies, field manager
bacchus-gpu-controller.bacchus.io), then the controller is replaced by one at chart defaults.
"""
import time

import pytest

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

pytestmark = pytest.mark.slow

REFERENCE_CONTROLLER = {"CONF_LABEL_CHILDREN": "false", "CONF_SKIP_UNCHANGED": "false",
                        "CONF_PARALLEL_CHILDREN": "false", "CONF_REQUEUE_SECS": "3600"}
LABEL = "app.kubernetes.io/managed-by"
KINDS = ("namespaces", "resourcequotas", "roles", "rolebindings")


def _ub(name, role=False):
    spec = {"kube_username": name,
            "quota": {"hard": {"requests.amd.com/gpu": "2", "requests.cpu": "16"}},
            "rolebinding": {"role_ref": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "edit"},
                            "subjects": [{"kind": "User", "name": f"oidc:{name}", "apiGroup": "rbac.authorization.k8s.io"}]}}
    if role:
        spec["role"] = {"metadata": {"name": name},
                        "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["get", "list"]}]}
    return {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": name}, "spec": spec}


def _children(c, name):
    out = {}
    for plural in KINDS:
        obj = c.admin.get_or_none(plural, name, None if plural == "namespaces" else name)
        if obj is not None:
            out[plural] = obj
    return out


def _writes(c):
    by_kind = c.stats().get("requests_by_kind", {})
    return sum(v for k, v in by_kind.items() if k.split(" ")[0] in ("POST", "PUT", "PATCH", "DELETE"))


def test_adopts_reference_managed_children():
    names = [f"adopt{i}" for i in range(6)]
    with Cluster(admission=False, controller_env=REFERENCE_CONTROLLER) as c:
        # --- the reference's state: synchronized tenants and their unlabelled children
        for i, n in enumerate(names):
            c.admin.create("userbootstraps", _ub(n, role=(i == 0)))
            ub = c.admin.get("userbootstraps", n)
            ub["status"] = {"synchronized_with_sheet": True}
            c.admin.replace("userbootstraps", n, ub, sub="status")
        for i, n in enumerate(names):
            want = 4 if i == 0 else 3
            wait_for(lambda n=n, want=want: len(_children(c, n)) == want, timeout=15, desc=f"{n} children")
        before = {n: _children(c, n) for n in names}
        for n, kids in before.items():
            for plural, obj in kids.items():
                assert LABEL not in obj["metadata"].get("labels", {}), (plural, n)
                assert obj["metadata"]["ownerReferences"][0]["name"] == n
                managers = {m["manager"] for m in obj["metadata"].get("managedFields", [])}
                assert "bacchus-gpu-controller.bacchus.io" in managers
        n_ns = len(c.admin.list("namespaces")["items"])

        # --- helm upgrade: the controller at chart defaults (fast requeue to show steady state)
        c.procs["controller"].stop()
        c.controller_env = {"CONF_REQUEUE_SECS": "1"}
        c.start_controller()

        def adopted():
            for n in names:
                for plural, obj in _children(c, n).items():
                    if obj["metadata"].get("labels", {}).get(LABEL) != "bacchus-gpu-controller":
                        return False
            return True

        wait_for(adopted, timeout=15, desc="every child labelled on the first pass")
        # adopted in place: same objects (uids), no duplicates
        for n in names:
            after = _children(c, n)
            assert set(after) == set(before[n])
            for plural, obj in after.items():
                assert obj["metadata"]["uid"] == before[n][plural]["metadata"]["uid"], (plural, n)
                assert obj["metadata"]["ownerReferences"] == before[n][plural]["metadata"]["ownerReferences"]
        assert len(c.admin.list("namespaces")["items"]) == n_ns

        # --- drift on an adopted child is repaired (its watch now sees it)
        c.admin.merge_patch("resourcequotas", names[1], {"spec": {"hard": {"requests.amd.com/gpu": "7"}}},
                            namespace=names[1], field_manager="kubectl-edit")
        wait_for(lambda: c.admin.get("resourcequotas", names[1], names[1])["spec"]["hard"]["requests.amd.com/gpu"] == "2",
                 timeout=10, desc="drift repaired")
        c.admin.json_patch("rolebindings", names[2], [{"op": "replace", "path": "/subjects/0/name", "value": "mallory"}],
                           namespace=names[2])
        wait_for(lambda: c.admin.get("rolebindings", names[2], names[2])["subjects"][0]["name"] == f"oidc:{names[2]}",
                 timeout=10, desc="rolebinding drift repaired")

        # --- steady state: no API writes across several 1 s requeue periods
        time.sleep(1.5)
        w0 = _writes(c)
        time.sleep(3.5)
        assert _writes(c) - w0 == 0

        # --- deleting a UserBootstrap still cascades through the adopted children
        c.admin.delete("userbootstraps", names[0])
        wait_for(lambda: not _children(c, names[0]), timeout=15, desc="cascade")
        assert c.procs["controller"].alive()

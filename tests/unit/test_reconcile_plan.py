"""The reconciler's planning step (native/controller/reconcile.cc desired_children):
which children the reference applies for a UserBootstrap, in its order, with which
bodies (reference src/controller.rs:50-155).  The bodies are written as JSON text
directly; these tests pin them to the objects the reference's code builds."""
import json

import pytest

OREF = {"apiVersion": "bacchus.io/v1", "controller": True, "kind": "UserBootstrap", "name": "Alice", "uid": "u-1"}
LABELS = {"app.kubernetes.io/managed-by": "bacchus-gpu-controller"}


def _ub(spec=None, status=None, name="Alice", uid="u-1"):
    ub = {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": name, "uid": uid},
          "spec": spec or {}}
    if status is not None:
        ub["status"] = status
    return json.dumps(ub)


def _plan(nat, ub, label=False):
    return [(p, ns, n, json.loads(b)) for p, ns, n, b in nat.desired_children(ub, label)]


def test_namespace_only(nat):
    [(plural, ns, name, body)] = _plan(nat, _ub())
    assert (plural, ns, name) == ("namespaces", "", "alice")  # lower-cased (controller.rs:55-63)
    assert body == {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "alice", "ownerReferences": [OREF]}}


def test_full_plan_order_and_bodies(nat):
    quota = {"hard": {"requests.amd.com/gpu": "2", "limits.cpu": "8"}}
    role = {"metadata": {"name": "alice", "labels": {"x": "y"}, "ownerReferences": [{"bogus": 1}]},
            "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["get"]}]}
    rb = {"role_ref": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "edit"},
          "subjects": [{"kind": "User", "name": "oidc:alice", "apiGroup": "rbac.authorization.k8s.io"}]}
    plan = _plan(nat, _ub({"quota": quota, "role": role, "rolebinding": rb}, {"synchronized_with_sheet": True}),
                 label=True)
    assert [p[0] for p in plan] == ["namespaces", "resourcequotas", "roles", "rolebindings"]
    meta = {"name": "alice", "ownerReferences": [OREF], "labels": LABELS}
    assert plan[0][3] == {"apiVersion": "v1", "kind": "Namespace", "metadata": meta}
    assert plan[1][1:3] == ("alice", "alice")
    assert plan[1][3] == {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": meta, "spec": quota}
    # the user's Role with ownerReferences overwritten (controller.rs:112-124), labels merged
    assert plan[2][3]["metadata"] == {"name": "alice", "labels": {"x": "y", **LABELS}, "ownerReferences": [OREF]}
    assert plan[2][3]["rules"] == role["rules"]
    assert plan[3][3] == {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding", "metadata": meta,
                          "roleRef": rb["role_ref"], "subjects": rb["subjects"]}
    # JSON text is exact: member order as the reference's serializer would emit them
    body = nat.desired_children(_ub({"quota": quota}), True)[1][3]
    assert body.startswith('{"apiVersion":"v1","kind":"ResourceQuota","metadata":{"name":"alice","ownerReferences":')


@pytest.mark.parametrize("status", [None, {}, {"synchronized_with_sheet": False}, {"synchronized_with_sheet": "true"}])
def test_rolebinding_gated_on_sync(nat, status):
    rb = {"role_ref": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "edit"}}
    plan = _plan(nat, _ub({"rolebinding": rb}, status))
    assert [p[0] for p in plan] == ["namespaces"]  # controller.rs:129-130


def test_rolebinding_without_subjects_and_escaping(nat):
    rb = {"role_ref": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "e\"dit"}}
    plan = _plan(nat, _ub({"rolebinding": rb}, {"synchronized_with_sheet": True}, name='Q"x', uid="u\\2"))
    body = plan[1][3]
    assert "subjects" not in body and body["roleRef"]["name"] == 'e"dit'
    assert body["metadata"]["ownerReferences"][0]["name"] == 'Q"x'
    assert body["metadata"]["ownerReferences"][0]["uid"] == "u\\2"
    assert body["metadata"]["name"] == 'q"x'


def test_missing_keys_raise(nat):
    with pytest.raises(Exception, match="metadata.name"):
        nat.desired_children(json.dumps({"metadata": {"uid": "u"}}), False)
    with pytest.raises(Exception, match="metadata.uid"):
        nat.desired_children(json.dumps({"metadata": {"name": "a"}}), False)

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


@pytest.mark.parametrize("text,value", [
    ("1", 1), ("0", 0), ("1000m", 1), ("1.5", 1.5), ("-2", -2), ("100u", 1e-4), ("5n", 5e-9),
    ("1k", 1e3), ("2M", 2e6), ("3G", 3e9), ("1T", 1e12), ("1P", 1e15), ("1E", 1e18),
    ("1Ki", 1024), ("64Gi", 64 * 2**30), ("0.5Gi", 2**29), ("1Ei", 2**60), ("1e3", 1e3), ("25E-1", 2.5),
])
def test_quantity_values(nat, text, value):
    assert nat.quantity_value(text) == pytest.approx(value, rel=1e-12)


@pytest.mark.parametrize("text", ["", "Gi", "1Xi", "1.2.3", "1e", "edit", "1 Gi", "1gi", "ki"])
def test_not_quantities(nat, text):
    assert nat.quantity_value(text) is None


def test_resync_compares_quota_values_not_spellings(nat):
    """The apiserver stores quantities canonical ("1000m" comes back as "1"): the resync's
    coverage check must not call that drift (it would re-apply every such quota forever)."""
    assert nat.same_quantity("1000m", "1") and nat.same_quantity("1024Mi", "1Gi") and nat.same_quantity("1e3", "1k")
    assert not nat.same_quantity("1", "2") and not nat.same_quantity("1Gi", "1G") and not nat.same_quantity("x", "x")


# apimachinery's canonical forms (resource.Quantity.String): parity unpinned against a real
# apiserver (none on this build's boxes); the cases follow CanonicalizeBytes' rules.
@pytest.mark.parametrize("text,canon", [
    ("1000m", "1"), ("0.5", "500m"), ("2000", "2k"), ("1500", "1500"), ("0.1", "100m"), ("0.0001", "100u"),
    ("12000k", "12M"), ("100m", "100m"), ("1n", "1n"), ("1.1n", "2n"), ("0", "0"), ("0Gi", "0"), ("-1", "-1"),
    ("1024Mi", "1Gi"), ("2048Mi", "2Gi"), ("1536Mi", "1536Mi"), ("1.5Gi", "1536Mi"), ("0.5Gi", "512Mi"),
    ("1023Ki", "1023Ki"), ("0.5Ki", "512"), ("1024", "1024"), ("1E", "1E"), ("1000E", "1e21"),
    ("1e3", "1e3"), ("1.5e3", "1500"), ("12e6", "12e6"), ("1e-10", "1e-9"), ("8", "8"),
])
def test_canonical_quantities(nat, text, canon):
    assert nat.canonical_quantity(text) == canon
    assert nat.same_quantity(text, canon) or text in ("1.1n", "1e-10")  # rounded up to 1n


@pytest.mark.parametrize("text", ["", "abc", "1Xi", ".", "1e", "1 Gi", "1" * 40])
def test_canonical_rejects_non_quantities(nat, text):
    assert nat.canonical_quantity(text) is None

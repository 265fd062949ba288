"""Admission policy (R6g/R6h): the full SURVEY §3.2 decision table (reference
src/admission.rs:206-431), exhaustively for representative inputs plus a hypothesis
property test against an independent Python oracle."""
import base64
import json

import pytest
from hypothesis import given, settings, strategies as st

PREFIX = "oidc:"
GROUPS = ["gpu", "admin"]
ROLE = "edit"


@pytest.fixture(scope="module")
def cfg(nat):
    c = nat.AdmissionConfig()
    c.oidc_username_prefix = PREFIX
    c.default_role_name = ROLE
    c.authorized_group_names = GROUPS
    c.log_full_request = False
    return c


def request(op="CREATE", username="oidc:alice", groups=("gpu",), name="alice", spec=None, obj=True, uid="u-1"):
    r = {"uid": uid, "kind": {"group": "bacchus.io", "version": "v1", "kind": "UserBootstrap"},
         "resource": {"group": "bacchus.io", "version": "v1", "resource": "userbootstraps"},
         "operation": op, "userInfo": {}}
    if username is not None:
        r["userInfo"]["username"] = username
    if groups is not None:
        r["userInfo"]["groups"] = list(groups)
    if obj:
        o = {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {}, "spec": spec if spec is not None else {}}
        if name is not None:
            o["metadata"]["name"] = name
        r["object"] = o
    return r


def run(nat, cfg, req):
    allowed, invalid, msg, patch, rule = nat.admission_mutate(json.dumps(req), cfg)
    return allowed, invalid, msg, (json.loads(patch) if patch else None), rule


def default_rb(subject):
    return {"role_ref": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": ROLE},
            "subjects": [{"apiGroup": "rbac.authorization.k8s.io", "kind": "User", "name": subject}]}


def test_classify(nat):
    assert nat.classify_username("oidc:bob", "oidc:") == ("oidc:bob", "bob", "normal")
    assert nat.classify_username("system:serviceaccount:x:y", "oidc:") == ("system:serviceaccount:x:y", "system:serviceaccount:x:y", "admin")
    assert nat.classify_username("kubernetes-admin", "oidc:") == ("kubernetes-admin", "kubernetes-admin", "admin")


def test_rule1_missing_username(nat, cfg):
    a, inv, msg, _, rule = run(nat, cfg, request(username=None))
    assert (a, inv, msg, rule) == (False, True, "cannot get requester's username from request", 1)


def test_rule4_create_normal_not_in_group(nat, cfg):
    a, inv, msg, _, rule = run(nat, cfg, request(groups=["students"]))
    assert (a, inv, msg, rule) == (False, False, "user is not in authorized group", 4)
    a, *_ = run(nat, cfg, request(groups=None))
    assert a is False


def test_rule5_6_delete(nat, cfg):
    assert run(nat, cfg, request(op="DELETE", obj=False))[:3] == (False, False, "normal user is not allowed to delete resource")
    a, inv, msg, patch, rule = run(nat, cfg, request(op="DELETE", username="admin", obj=False))
    assert (a, patch, rule) == (True, None, 6)


def test_rule7_update_normal(nat, cfg):
    assert run(nat, cfg, request(op="UPDATE"))[:3] == (False, False, "normal user is not allowed to update resource")


def test_rule8_connect(nat, cfg):
    a, inv, msg, _, rule = run(nat, cfg, request(op="CONNECT"))
    assert (a, inv, msg, rule) == (False, True, "invalid operation", 8)


def test_rule9_no_object(nat, cfg):
    a, _, _, patch, rule = run(nat, cfg, request(op="UPDATE", username="admin", obj=False))
    assert (a, patch, rule) == (True, None, 9)


def test_rule10_no_name(nat, cfg):
    a, inv, msg, _, rule = run(nat, cfg, request(name=None))
    assert (a, inv, msg, rule) == (False, True, "cannot get resource name from request", 10)


def test_rule11_name_mismatch(nat, cfg):
    assert run(nat, cfg, request(name="bob"))[2] == "username not match with resource name"


def test_rule12_not_a_userbootstrap(nat, cfg):
    a, inv, msg, _, rule = run(nat, cfg, request(spec={"kube_username": 7}))
    assert (a, inv, rule) == (False, True, 12)
    assert "invalid type" in msg


def test_rule13_16_normal_create_three_ops(nat, cfg):
    a, inv, msg, patch, rule = run(nat, cfg, request(spec={"kube_username": "mallory"}))
    assert a and rule == 19
    assert patch == [
        {"op": "add", "path": "/spec/kube_username", "value": "alice"},
        {"op": "add", "path": "/spec/rolebinding", "value": {}},
        {"op": "add", "path": "/spec/rolebinding", "value": default_rb("oidc:alice")},
    ]


def test_rule14_admin_empty_kube_username(nat, cfg):
    for spec in ({}, {"kube_username": ""}, {"kube_username": None}):
        assert run(nat, cfg, request(username="admin", name="x", spec=spec))[2] == \
            "kube_username field is empty. you are an admin, so fill it"


def test_rule15_normal_quota(nat, cfg):
    assert run(nat, cfg, request(spec={"quota": {"hard": {"cpu": "1"}}}))[2] == \
        "quota field is not empty. you are a normal user, so leave it empty"


def test_rule16_admin_subject_is_kube_username_verbatim(nat, cfg):
    a, _, _, patch, rule = run(nat, cfg, request(username="admin", name="x", spec={"kube_username": "carol"}))
    assert a and patch == [{"op": "add", "path": "/spec/rolebinding", "value": {}},
                           {"op": "add", "path": "/spec/rolebinding", "value": default_rb("carol")}]


def test_rule17_normal_rolebinding(nat, cfg):
    rb = default_rb("x")
    assert run(nat, cfg, request(spec={"rolebinding": rb}))[2] == \
        "rolebinding field is not empty. you are a normal user, so leave it empty"


def test_rule18_admin_full_spec_no_patch(nat, cfg):
    spec = {"kube_username": "carol", "quota": {"hard": {"requests.amd.com/gpu": "1"}}, "rolebinding": default_rb("carol")}
    a, _, _, patch, rule = run(nat, cfg, request(op="UPDATE", username="system:serviceaccount:ns:sync", name="carol", spec=spec))
    assert (a, patch, rule) == (True, None, 18)


def test_normal_role_is_not_validated(nat, cfg):
    # Q11: a normal user's spec.role passes through unchecked.
    a, *_ = run(nat, cfg, request(spec={"role": {"metadata": {"name": "alice"}, "rules": [{"verbs": ["*"], "resources": ["*"], "apiGroups": ["*"]}]}}))
    assert a


def test_http_review_roundtrip(nat, cfg):
    review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": request()}
    status, body, ctype = nat.admission_handle_review(json.dumps(review), "application/json", cfg)
    assert status == 200
    out = json.loads(body)
    assert out["apiVersion"] == "admission.k8s.io/v1" and out["kind"] == "AdmissionReview"
    resp = out["response"]
    assert resp["uid"] == "u-1" and resp["allowed"] is True and resp["patchType"] == "JSONPatch"
    ops = json.loads(base64.b64decode(resp["patch"]))
    assert len(ops) == 3


def test_http_review_invalid_echoes_uid(nat, cfg):
    review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": request(op="CONNECT", uid="zz")}
    status, body, _ = nat.admission_handle_review(json.dumps(review), "application/json", cfg)
    resp = json.loads(body)["response"]
    assert status == 200 and resp["uid"] == "zz" and resp["allowed"] is False
    assert resp["status"]["code"] == 400 and resp["status"]["message"] == "invalid operation"


@pytest.mark.parametrize("body,ctype,code", [
    ("{", "application/json", 400),
    ("{}", "text/plain", 415),
    ('{"request": {"uid": "x"}}', "application/json", 422),
    ('{"request": {"uid":"x","kind":{},"resource":{},"operation":"PATCH","userInfo":{}}}', "application/json", 422),
    ('{"request": ' + "[" * 5000 + "]" * 5000 + "}", "application/json", 400),  # nesting past the parser's depth cap
    ('{"request": {"object": ' + '{"a":' * 600 + "1" + "}" * 600 + "}}", "application/json", 400),
])
def test_http_review_rejections(nat, cfg, body, ctype, code):
    assert nat.admission_handle_review(body, ctype, cfg)[0] == code


def test_missing_request_is_invalid(nat, cfg):
    status, body, _ = nat.admission_handle_review('{"apiVersion":"admission.k8s.io/v1","kind":"AdmissionReview"}',
                                                  "application/json", cfg)
    assert status == 200 and json.loads(body)["response"]["allowed"] is False


# ---------------------------------------------------------------------------
# Property test against an independent oracle of SURVEY §3.2

def oracle(req):
    ui = req.get("userInfo", {})
    uname = ui.get("username")
    if uname is None:
        return ("invalid", "cannot get requester's username from request", None)
    normal = uname.startswith(PREFIX)
    kube = uname[len(PREFIX):] if normal else uname
    in_group = any(g in GROUPS for g in (ui.get("groups") or []))
    op = req["operation"]
    if op == "CREATE":
        if normal and not in_group:
            return ("deny", "user is not in authorized group", None)
    elif op == "DELETE":
        return ("deny", "normal user is not allowed to delete resource", None) if normal else ("allow", "", None)
    elif op == "UPDATE":
        if normal:
            return ("deny", "normal user is not allowed to update resource", None)
    else:
        return ("invalid", "invalid operation", None)
    obj = req.get("object")
    if obj is None:
        return ("allow", "", None)
    name = obj["metadata"].get("name")
    if name is None:
        return ("invalid", "cannot get resource name from request", None)
    if normal and kube != name:
        return ("deny", "username not match with resource name", None)
    spec = obj["spec"]
    patches = []
    if normal:
        patches.append({"op": "add", "path": "/spec/kube_username", "value": kube})
    elif not spec.get("kube_username"):
        return ("deny", "kube_username field is empty. you are an admin, so fill it", None)
    if spec.get("quota") is not None and normal:
        return ("deny", "quota field is not empty. you are a normal user, so leave it empty", None)
    if spec.get("rolebinding") is None:
        patches.append({"op": "add", "path": "/spec/rolebinding", "value": {}})
        patches.append({"op": "add", "path": "/spec/rolebinding",
                        "value": default_rb(uname if normal else spec["kube_username"])})
    elif normal:
        return ("deny", "rolebinding field is not empty. you are a normal user, so leave it empty", None)
    return ("allow", "", patches or None)


names = st.sampled_from(["alice", "bob", "x"])
usernames = st.one_of(st.none(), st.sampled_from(["oidc:alice", "oidc:bob", "admin", "system:serviceaccount:a:b", "oidcalice"]))
groups = st.one_of(st.none(), st.lists(st.sampled_from(["gpu", "admin", "students", ""]), max_size=3))
specs = st.fixed_dictionaries({}, optional={
    "kube_username": st.one_of(st.none(), st.sampled_from(["", "alice", "carol"])),
    "quota": st.one_of(st.none(), st.just({"hard": {"requests.amd.com/gpu": "1"}})),
    "rolebinding": st.one_of(st.none(), st.just(default_rb("z"))),
    "role": st.one_of(st.none(), st.just({"metadata": {"name": "alice"}})),
})


@settings(max_examples=400, deadline=None)
@given(op=st.sampled_from(["CREATE", "UPDATE", "DELETE", "CONNECT"]), username=usernames, grp=groups,
       name=st.one_of(st.none(), names), spec=specs, has_obj=st.booleans())
def test_property_matches_oracle(nat, cfg, op, username, grp, name, spec, has_obj):
    req = request(op=op, username=username, groups=grp, name=name, spec=spec, obj=has_obj)
    allowed, invalid, msg, patch, _ = run(nat, cfg, req)
    kind, omsg, opatch = oracle(req)
    assert allowed == (kind == "allow")
    assert invalid == (kind == "invalid")
    assert msg == omsg
    assert patch == opatch


MANAGED = [{"manager": "kubectl", "operation": "Update", "apiVersion": "bacchus.io/v1", "time": "2024-01-01T00:00:00Z",
            "fieldsType": "FieldsV1", "fieldsV1": {"f:spec": {"f:quota": {".": {}, "f:hard": {"f:requests.cpu": {}}}}}}]


@settings(max_examples=300, deadline=None)
@given(op=st.sampled_from(["CREATE", "UPDATE", "DELETE", "CONNECT"]), username=usernames, grp=groups,
       name=st.one_of(st.none(), names), spec=specs, has_obj=st.booleans(), old=st.booleans(),
       status=st.one_of(st.none(), st.booleans()))
def test_http_review_projection_matches_full_parse(nat, cfg, op, username, grp, name, spec, has_obj, old, status):
    """handle_review parses only what mutate() reads (json::Projection: uid, operation,
    userInfo, object name/spec/status; the shape of the rest).  Its decision equals mutate()
    on the fully parsed request, with managedFields, labels and oldObject present."""
    req = request(op=op, username=username, groups=grp, name=name, spec=spec, obj=has_obj)
    if has_obj:
        req["object"]["metadata"].update({"managedFields": MANAGED, "labels": {"a": "b"}, "resourceVersion": "7",
                                          "uid": "0-1", "annotations": {"x": "y" * 200}})
        if status is not None:
            req["object"]["status"] = {"synchronized_with_sheet": status}
    if old:
        req["oldObject"] = {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                            "metadata": {"name": "alice", "managedFields": MANAGED}, "spec": {"quota": {"hard": {}}}}
    review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": req}
    status_code, body, _ = nat.admission_handle_review(json.dumps(review), "application/json", cfg)
    assert status_code == 200
    resp = json.loads(body)["response"]
    allowed, invalid, msg, patch, _ = run(nat, cfg, req)
    assert resp["uid"] == "u-1" and resp["allowed"] == allowed
    assert resp.get("status", {}).get("message") == (msg or None if not allowed else None)
    got = json.loads(base64.b64decode(resp["patch"])) if "patch" in resp else None
    assert got == patch


@pytest.mark.parametrize("username,uid", [("oidc:alice", "u-1"), ('oidc:q"uo\\te', 'u"\\1'),
                                          ("oidc:ünï\tcode", "ué")])
def test_review_response_wire_format(nat, cfg, username, uid):
    """The response document and its patch are written as text (round 5): byte-compare them
    with compact JSON of the expected documents, in the member order the reference's serde
    types emit, for names that need escaping."""
    name = username[len(PREFIX):]
    req = request(username=username, name=name, uid=uid)
    review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": req}
    status, body, _ = nat.admission_handle_review(json.dumps(review), "application/json", cfg)
    assert status == 200
    compact = lambda o: json.dumps(o, separators=(",", ":"), ensure_ascii=False)  # noqa: E731
    ops = [{"op": "add", "path": "/spec/kube_username", "value": name},
           {"op": "add", "path": "/spec/rolebinding", "value": {}},
           {"op": "add", "path": "/spec/rolebinding",
            "value": {"role_ref": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": cfg.default_role_name},
                      "subjects": [{"apiGroup": "rbac.authorization.k8s.io", "kind": "User", "name": username}]}}]
    patch = json.loads(base64.b64decode(json.loads(body)["response"]["patch"]))
    assert patch == ops
    expected = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                "response": {"uid": uid, "allowed": True,
                             "patch": base64.b64encode(compact(ops).encode()).decode(), "patchType": "JSONPatch"}}
    assert body == compact(expected)


def test_denial_wire_format(nat, cfg):
    req = request(username="oidc:alice", groups=("nope",))
    status, body, _ = nat.admission_handle_review(json.dumps({"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                                                              "request": req}), "application/json", cfg)
    assert body == ('{"apiVersion":"admission.k8s.io/v1","kind":"AdmissionReview","response":{"uid":"u-1",'
                    '"allowed":false,"status":{"message":"user is not in authorized group"}}}')

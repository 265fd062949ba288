"""CRD generation (R1/R3): crdgen output must be byte-identical to the reference chart's
crd.yaml (reference src/crdgen.rs:3-8, charts/.../templates/crd.yaml)."""
import json
import os
import subprocess

import pytest
import yaml

from bacchus_gpu_controller_amd import REPO_ROOT, binary

CHART_CRD = os.path.join(REPO_ROOT, "charts", "bacchus-gpu-controller", "templates", "crd.yaml")


def test_crdgen_binary_matches_reference_bytes(reference_crd_path):
    out = subprocess.run([binary("crdgen")], check=True, capture_output=True).stdout
    if reference_crd_path:
        assert out == open(reference_crd_path, "rb").read()
    assert out == open(CHART_CRD, "rb").read(), "charts/.../crd.yaml is stale: run ./generate-crd.sh"


def test_crd_semantics(nat):
    crd = json.loads(nat.crd_json())
    assert crd["metadata"]["name"] == "userbootstraps.bacchus.io"
    assert crd["spec"]["scope"] == "Cluster"
    assert crd["spec"]["names"]["shortNames"] == ["ub"]
    v = crd["spec"]["versions"][0]
    assert v["subresources"] == {"status": {}}
    s = v["schema"]["openAPIV3Schema"]
    spec = s["properties"]["spec"]["properties"]
    assert set(spec) == {"kube_username", "quota", "role", "rolebinding"}
    assert all(spec[k]["nullable"] for k in spec)
    assert spec["rolebinding"]["required"] == ["role_ref"]
    assert s["properties"]["status"]["required"] == ["synchronized_with_sheet"]


def test_yaml_of_crd_is_valid_yaml(nat):
    assert yaml.safe_load(nat.crd_yaml()) == json.loads(nat.crd_json())


@pytest.mark.parametrize("obj,ok", [
    ({"metadata": {"name": "a"}, "spec": {}}, True),
    ({"metadata": {"name": "a"}, "spec": {"kube_username": 5}}, False),
    ({"metadata": {"name": "a"}, "spec": {"quota": {"hard": {"cpu": "1"}}}}, True),
    ({"metadata": {"name": "a"}, "spec": {"quota": {"hard": {"cpu": 1}}}}, False),
    ({"metadata": {"name": "a"}, "spec": {"rolebinding": {}}}, False),
    ({"metadata": {"name": "a"}, "spec": {"rolebinding": {"role_ref": {"apiGroup": "g", "kind": "k", "name": "n"}}}}, True),
    ({"metadata": {"name": "a"}, "spec": {"role": {"rules": [{"verbs": ["get"]}]}}}, True),
    ({"metadata": {"name": "a"}, "spec": {"role": {"metadata": {"creationTimestamp": "garbage"}}}}, False),
    ({"metadata": {"name": "a"}}, False),
    ({"metadata": {"name": "a"}, "spec": {}, "status": {"synchronized_with_sheet": True}}, True),
    ({"metadata": {"name": "a"}, "spec": {}, "status": {}}, False),
])
def test_parse_userbootstrap_serde_semantics(nat, obj, ok):
    if ok:
        nat.parse_userbootstrap(json.dumps(obj))
    else:
        with pytest.raises(RuntimeError):
            nat.parse_userbootstrap(json.dumps(obj))

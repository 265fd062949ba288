"""C++ JSON / YAML / JSON-Patch core (native/core)."""
import json

import pytest
import yaml as pyyaml


def test_json_roundtrip_preserves_i64_and_order(nat):
    doc = '{"b":1,"a":-9223372036854775808,"c":18446744073709551615,"d":1.5,"e":[true,false,null],"f":"\\u00e9\\n"}'
    out = nat.json_roundtrip(doc)
    assert out == '{"b":1,"a":-9223372036854775808,"c":18446744073709551615,"d":1.5,"e":[true,false,null],"f":"é\\n"}'
    assert json.loads(out) == json.loads(doc)


@pytest.mark.parametrize("bad", ['{"a":}', "[1,]", '{"a" 1}', '"\\x"', "01", "{", '"\\ud800"'])
def test_json_rejects_invalid(nat, bad):
    with pytest.raises(ValueError):
        nat.json_roundtrip(bad)


def test_json_parse_drops_key_at_any_depth(nat):
    """Watchers parse events with managedFields skipped (native/kube/runtime.cc)."""
    mf = [{"manager": "m", "fieldsV1": {"f:spec": {"f:hard": {".": {}, 'f:"x}]': {}}}}, "time": "t"}]
    obj = {"type": "ADDED", "object": {"metadata": {"name": "a", "managedFields": mf, "labels": {"k": "v"}},
                                       "spec": {"managedFields": "s\\\"]}", "n": [1, {"managedFields": 1.5e3}]},
                                       "managedFields": None}}
    out = json.loads(nat.json_roundtrip(json.dumps(obj), drop_key="managedFields"))
    assert out == {"type": "ADDED", "object": {"metadata": {"name": "a", "labels": {"k": "v"}},
                                               "spec": {"n": [1, {}]}}}
    # last member dropped, whitespace around it, and an empty object left behind
    assert json.loads(nat.json_roundtrip('{"a":1, "managedFields" : [ ] }', drop_key="managedFields")) == {"a": 1}
    assert nat.json_roundtrip('{"managedFields":{"x":[1,2]}}', drop_key="managedFields") == "{}"
    for bad in ('{"managedFields":', '{"managedFields":[1,2}', '{"managedFields":"abc}', '{"managedFields":}'):
        with pytest.raises(ValueError):
            nat.json_roundtrip(bad, drop_key="managedFields")


def test_json_surrogate_pairs(nat):
    assert json.loads(nat.json_roundtrip('"\\ud83d\\ude00"')) == "\U0001F600"


def test_json_patch_rfc6902_ops(nat):
    doc = {"spec": {"a": 1, "list": [1, 2, 3]}}
    patch = [
        {"op": "add", "path": "/spec/b", "value": {"x": 1}},
        {"op": "replace", "path": "/spec/a", "value": 2},
        {"op": "remove", "path": "/spec/list/0"},
        {"op": "add", "path": "/spec/list/-", "value": 9},
        {"op": "copy", "from": "/spec/b", "path": "/spec/c"},
        {"op": "move", "from": "/spec/c", "path": "/spec/d"},
        {"op": "test", "path": "/spec/a", "value": 2},
        {"op": "add", "path": "/spec/k~1v", "value": "slash"},
    ]
    out = json.loads(nat.apply_json_patch(json.dumps(doc), json.dumps(patch)))
    assert out == {"spec": {"a": 2, "list": [2, 3, 9], "b": {"x": 1}, "d": {"x": 1}, "k/v": "slash"}}


def test_json_patch_is_atomic(nat):
    doc = {"a": 1}
    with pytest.raises(ValueError):
        nat.apply_json_patch(json.dumps(doc), json.dumps([{"op": "replace", "path": "/a", "value": 5},
                                                          {"op": "replace", "path": "/missing", "value": 1}]))


def test_merge_patch(nat):
    out = nat.apply_merge_patch('{"a":{"b":1,"c":2},"d":3}', '{"a":{"b":null,"e":4},"d":null}')
    assert json.loads(out) == {"a": {"c": 2, "e": 4}}


def test_yaml_emit_styles_match_serde_yaml(nat):
    doc = {
        "plain": "hello world",
        "colon": "a: b",
        "boolish": "true",
        "num": "123",
        "zero_lead": "0123",
        "empty": "",
        "multi": "line1\nline2",
        "multi_nl": "line1\n",
        "multi_keep": "line1\n\n",
        "tab": "a\tb\nc",
        "list": ["x", {"k": "v", "k2": []}],
        "emptymap": {},
        "n": 5,
        "b": True,
    }
    out = nat.json_to_yaml(json.dumps(doc))
    assert out == (
        "plain: hello world\n"
        "colon: 'a: b'\n"
        "boolish: 'true'\n"
        "num: '123'\n"
        "zero_lead: '0123'\n"
        "empty: ''\n"
        "multi: |-\n  line1\n  line2\n"
        "multi_nl: |\n  line1\n"
        "multi_keep: |+\n  line1\n\n"
        'tab: "a\\tb\\nc"\n'
        "list:\n- x\n- k: v\n  k2: []\n"
        "emptymap: {}\n"
        "n: 5\n"
        "b: true\n"
    )
    assert pyyaml.safe_load(out) == doc


def test_yaml_parse_kubeconfig_like(nat):
    text = """
apiVersion: v1
clusters:
- cluster:
    certificate-authority-data: Zm9v
    server: https://127.0.0.1:6443   # comment
  name: kind
contexts:
- context: {cluster: kind, user: admin}
  name: kind
current-context: kind
users:
- name: admin
  user:
    token: "abc:def"
    list: [a, 'b', "c"]
    block: |
      x
      y
"""
    got = json.loads(nat.yaml_to_json(text))
    assert got == pyyaml.safe_load(text)


def test_yaml_parse_reference_crd_roundtrip(nat, reference_crd_path):
    if not reference_crd_path:
        pytest.skip("reference not mounted")
    text = open(reference_crd_path).read()
    assert json.loads(nat.yaml_to_json(text)) == pyyaml.safe_load(text)

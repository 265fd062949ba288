"""Property-based tests of the native core codecs (hypothesis): JSON parse/dump, the
serde_yaml-style YAML emitter against our parser and PyYAML, and RFC 7386 merge patch
against an independent Python implementation."""
import json
import string

import pytest
import yaml
from hypothesis import given, settings
from hypothesis import strategies as st

I64 = st.integers(min_value=-(2 ** 63), max_value=2 ** 63 - 1)
U64_HI = st.integers(min_value=2 ** 63, max_value=2 ** 64 - 1)
FLOATS = st.floats(allow_nan=False, allow_infinity=False, width=64)
TEXT = st.text(max_size=20)
KEYS = st.text(max_size=8)


def json_values(leaf):
    return st.recursive(leaf, lambda kids: st.lists(kids, max_size=4) | st.dictionaries(KEYS, kids, max_size=4),
                        max_leaves=25)


@settings(max_examples=300, deadline=None)
@given(json_values(st.none() | st.booleans() | I64 | U64_HI | FLOATS | TEXT))
def test_json_roundtrip_matches_python(nat, v):
    assert json.loads(nat.json_roundtrip(json.dumps(v))) == v


def _drop(v, key):
    if isinstance(v, dict):
        return {k: _drop(x, key) for k, x in v.items() if k != key}
    if isinstance(v, list):
        return [_drop(x, key) for x in v]
    return v


@settings(max_examples=300, deadline=None)
@given(json_values(st.none() | st.booleans() | I64 | FLOATS | TEXT), st.sampled_from(["", "a", "managedFields"]),
       st.booleans())
def test_json_drop_key_parse_matches_python(nat, v, key, pretty):
    """parse(text, drop_key) == python parse with that key removed at every depth."""
    text = json.dumps({"managedFields": v, "x": [v, {"a": v}]} if key else v, indent=2 if pretty else None)
    if not key:
        key = "managedFields"
    assert json.loads(nat.json_roundtrip(text, drop_key=key)) == _drop(json.loads(text), key)


@settings(max_examples=200, deadline=None)
@given(json_values(st.none() | st.booleans() | I64 | TEXT))
def test_yaml_emit_parses_back_with_our_parser(nat, v):
    assert json.loads(nat.yaml_to_json(nat.json_to_yaml(json.dumps(v)))) == v


def _yaml11_only_nonstring(s):
    """Plain scalars YAML 1.1 (PyYAML) resolves to a non-string although the emitter (like
    serde_yaml, YAML 1.2) leaves them unquoted as strings, e.g. "0_" (1.1 int with a digit
    separator), "1:20" (sexagesimal) or "2001-12-14" (timestamp): not 1.1/1.2-neutral."""
    from bacchus_gpu_controller_amd import native

    try:
        v11 = yaml.safe_load(s)
    except yaml.YAMLError:
        return False
    emitted_plain = native().json_to_yaml(json.dumps(s)).rstrip("\n") == s
    return emitted_plain and not isinstance(v11, str)


SAFE = st.text(alphabet=string.ascii_letters + string.digits + " -_./:", min_size=1, max_size=16).filter(
    lambda s: s.lower() not in {"y", "n", "yes", "no", "on", "off", "true", "false", "null", "~"}
    and not _yaml11_only_nonstring(s))


NEUTRAL_KEYS = KEYS.filter(lambda k: not _yaml11_only_nonstring(k))


@settings(max_examples=200, deadline=None)
@given(st.recursive(st.none() | st.booleans() | st.integers(min_value=-10 ** 9, max_value=10 ** 9) | SAFE,
                    lambda kids: st.lists(kids, max_size=4) | st.dictionaries(NEUTRAL_KEYS, kids, max_size=4),
                    max_leaves=25))
def test_yaml_emit_loads_in_pyyaml(nat, v):
    # YAML 1.1/1.2-neutral scalars: PyYAML (1.1) must read exactly what we emitted
    assert yaml.safe_load(nat.json_to_yaml(json.dumps(v))) == v


def merge_patch_ref(target, patch):
    """RFC 7386 section 2, literally."""
    if not isinstance(patch, dict):
        return patch
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch_ref(out.get(k), v)
    return out


@settings(max_examples=300, deadline=None)
@given(json_values(st.none() | st.booleans() | I64 | TEXT), json_values(st.none() | st.booleans() | I64 | TEXT))
def test_merge_patch_matches_rfc7386(nat, doc, patch):
    got = json.loads(nat.apply_merge_patch(json.dumps(doc), json.dumps(patch)))
    assert got == merge_patch_ref(doc, patch)


@pytest.mark.parametrize("text", ["1e400", "-1e400"])
def test_json_out_of_range_numbers_rejected_or_finite(nat, text):
    try:
        out = json.loads(nat.json_roundtrip(text))
    except ValueError:
        return
    assert out not in (float("inf"), float("-inf"))


MULTILINE = st.text(alphabet=string.ascii_letters + " \n", max_size=16).filter(
    lambda s: not _yaml11_only_nonstring(s))  # "NO", "on", ...: YAML 1.1 booleans


@settings(max_examples=300, deadline=None)
@given(MULTILINE | st.dictionaries(st.sampled_from(["a", "b", "c"]), MULTILINE, max_size=3)
       | st.lists(MULTILINE, max_size=3))
def test_yaml_block_scalars_roundtrip_in_both_parsers(nat, v):
    # literal block scalars (|, |-, |+, |2+) at the top level, in mappings and in sequences
    y = nat.json_to_yaml(json.dumps(v))
    assert json.loads(nat.yaml_to_json(y)) == v
    assert yaml.safe_load(y) == v


@settings(max_examples=200, deadline=None)
@given(st.dictionaries(KEYS, json_values(st.none() | st.booleans() | I64 | TEXT), max_size=6), st.booleans())
def test_raw_member_matches_parse(nat, obj, pretty):
    """json::raw_member (admission logs the received request without re-serializing it):
    the raw slice of every top-level member parses to that member's value."""
    text = json.dumps(obj, indent=1 if pretty else None, ensure_ascii=False)
    for k, v in obj.items():
        raw = nat.json_raw_member(text, json.dumps(k, ensure_ascii=False)[1:-1])
        assert json.loads(raw) == v
    assert nat.json_raw_member(text, "\x00missing") == ""
    assert nat.json_raw_member("[1, 2]", "a") == ""


def _shape(v):
    return {dict: {}, list: [], str: "", bool: False, type(None): None}.get(type(v), 0)


def _project(v, tree):
    """Python model of json::parse_projected: kept paths whole, the rest empty-of-type."""
    if tree is True:
        return v
    if not isinstance(v, dict):
        return v if tree else _shape(v)  # a Descend node that is not an object is kept whole
    return {k: (_project(x, tree[k]) if k in tree else _shape(x)) for k, x in v.items()}


def _tree(paths):
    t = {}
    for p in paths:
        node = t
        parts = p.split(".")
        for k in parts[:-1]:
            node = node.setdefault(k, {})
            if node is True:
                break
        else:
            node[parts[-1]] = True
    return t


@settings(max_examples=300, deadline=None)
@given(json_values(st.none() | st.booleans() | I64 | FLOATS | st.text(alphabet="ab.", max_size=3)),
       st.lists(st.sampled_from(["a", "b", "a.a", "a.b", "b.a.a", "a.b.a"]), max_size=3))
def test_projected_parse_matches_model(nat, v, keep):
    """parse_projected keeps the named paths and only the type of everything else (the
    AdmissionReview fast path of admission/policy.cc)."""
    doc = {"a": v, "b": {"a": v, "b": [v]}} if not isinstance(v, dict) else v
    text = json.dumps(doc)
    assert json.loads(nat.json_parse_projected(text, keep)) == _project(doc, _tree(keep) or {})


def _omit(v, tree):
    if tree is True:
        return v
    if not isinstance(v, dict):
        return v  # a Descend node that is not an object is kept whole
    return {k: _omit(x, tree[k]) for k, x in v.items() if k in tree}


@settings(max_examples=300, deadline=None)
@given(json_values(st.none() | st.booleans() | I64 | FLOATS | st.text(alphabet="ab.\"\\{}[],:", max_size=4)),
       st.lists(st.sampled_from(["a", "b", "a.a", "a.b", "b.a.a", "a.b.a"]), max_size=3))
def test_projected_parse_omit_unnamed_matches_model(nat, v, keep):
    """omit_unnamed (the controller's UserBootstrap watch events): members no projection
    names are stepped over structurally and left out, whatever brackets or quotes their
    strings hold."""
    doc = {"a": v, "b": {"a": v, "b": [v]}, "c": {"x": [v, {"y": v}]}} if not isinstance(v, dict) else v
    text = json.dumps(doc)
    assert json.loads(nat.json_parse_projected(text, keep, True)) == _omit(doc, _tree(keep) or {})


@settings(max_examples=300, deadline=None)
@given(json_values(st.none() | st.booleans() | I64 | TEXT), st.integers(min_value=0, max_value=200),
       st.sampled_from(["", "x", "{", "]", "\\", "\"", ",", "1e", "tru", "\u0001"]))
def test_projected_parse_rejects_what_parse_rejects(nat, v, pos, junk):
    """Skipped subtrees are still validated: a corrupted document fails the projected parse
    with the same error as the full parse."""
    text = json.dumps({"keep": v, "skip": [v, {"deep": v}]})
    pos = min(pos, len(text))
    bad = text[:pos] + junk + text[pos:]
    full = proj = None
    try:
        nat.json_roundtrip(bad)
    except Exception as e:  # noqa: BLE001
        full = str(e)
    try:
        nat.json_parse_projected(bad, ["keep"])
    except Exception as e:  # noqa: BLE001
        proj = str(e)
    assert full == proj

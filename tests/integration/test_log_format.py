"""BGC_LOG_FORMAT=json: every log line a JSON object in tracing-subscriber's `fmt().json()`
layout (native/core/log.cc), for log pipelines that parse structured logs.  The default stays
the reference's text format."""
import json
import re

import pytest

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

pytestmark = pytest.mark.slow


def test_json_log_lines():
    env = {"BGC_LOG_FORMAT": "json", "RUST_LOG": "info"}
    with Cluster(admission=False, controller_env=env) as c:
        c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                          "metadata": {"name": "logged"}, "spec": {"kube_username": "logged"}})
        wait_for(lambda: c.admin.get_or_none("namespaces", "logged"), desc="reconciled")
        lines = [l for l in c.procs["controller"].output().splitlines() if l.strip()]
    assert lines
    for l in lines:
        rec = json.loads(l)
        assert set(rec) == {"timestamp", "level", "fields", "target"}, rec
        assert re.fullmatch(r"\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d\.\d{6}Z", rec["timestamp"])
        assert rec["level"] in ("TRACE", "DEBUG", "INFO", "WARN", "ERROR")
        assert isinstance(rec["fields"]["message"], str)
    assert any(r["target"] == "controller" for r in map(json.loads, lines))


def test_text_log_lines_by_default():
    with Cluster(admission=False, controller_env={"RUST_LOG": "info"}) as c:
        out = c.procs["controller"].output()
    assert out and not out.lstrip().startswith("{")
    assert re.search(r"^\d{4}-\d\d-\d\dT\S+Z\s+INFO \S+: ", out, re.M)

"""The periodic malloc_trim pass (native/core/process.cc) runs only when the process has
grown and is quiet.

A pass walks every free chunk under its arena's lock and stalls the process: 13-15 ms in
the synchronizer on the MI355X box (profiles/r5_trim/), which is on the path to Ready.  Round
5 first limited passes to growth; a pass still fell into a latency window of the bench, so it
now also waits for an interval in which the process used at most BGC_MALLOC_TRIM_IDLE_PCT of
one CPU.
"""
import time

import pytest
import requests

from bacchus_gpu_controller_amd import native
from bacchus_gpu_controller_amd.testing.cluster import Cluster

MB = 1 << 20


@pytest.mark.parametrize("rss,baseline,busy,want", [
    (32 * MB, 8 * MB, 0.0, "skip"),     # under the 64 MB minimum
    (90 * MB, 80 * MB, 0.0, "skip"),    # not 1.5x the last pass
    (100 * MB, 8 * MB, 0.5, "trim"),    # grown and quiet
    (100 * MB, 8 * MB, 40.0, "defer"),  # grown but busy
    (300 * MB, 70 * MB, 40.0, "trim"),  # busy, but past 4x max(previous, minimum)
    (250 * MB, 8 * MB, 40.0, "defer"),  # 4x the minimum is the floor of that valve
])
def test_trim_decision(rss, baseline, busy, want):
    assert native().malloc_trim_decision(rss, baseline, 64 * MB, busy, 5.0) == want


@pytest.mark.parametrize("rss,baseline,limit,want", [
    (100 * MB, 60 * MB, 160 * MB, "trim"),    # past half the container limit: trim while busy
    (100 * MB, 60 * MB, 0, "defer"),          # no limit: wait for a quiet interval
    (100 * MB, 60 * MB, 256 * MB, "defer"),   # under half the limit
    (100 * MB, 80 * MB, 160 * MB, "skip"),    # not grown since the last pass: never every check
])
def test_trim_decision_under_a_memory_limit(rss, baseline, limit, want):
    assert native().malloc_trim_decision(rss, baseline, 64 * MB, 40.0, 5.0, limit) == want


def test_cgroup_memory_limit_reads_as_bytes_or_none():
    v = native().cgroup_memory_limit_bytes()
    assert v == 0 or v >= 4096


def _trim_metrics(c):
    text = requests.get(f"http://127.0.0.1:{c.controller_port}/metrics", timeout=5).text
    return {l.split()[0]: float(l.split()[1]) for l in text.splitlines()
            if l.startswith(("bgc_malloc_trim_deferred_total", "bgc_malloc_trim_seconds_count"))}


def _grow(c):
    for i in range(600):
        c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                          "metadata": {"name": f"u{i}"},
                                          "spec": {"kube_username": f"u{i}",
                                                   "quota": {"hard": {"requests.amd.com/gpu": "1"}}}})


@pytest.mark.slow
@pytest.mark.parametrize("idle_pct,trims", [("50", True), ("0", False)])
def test_controller_trims_only_when_quiet(idle_pct, trims):
    env = {"BGC_MALLOC_TRIM_SECS": "1", "BGC_MALLOC_TRIM_MIN_MB": "1", "BGC_MALLOC_TRIM_IDLE_PCT": idle_pct}
    with Cluster(admission=False, controller_env=env) as c:
        time.sleep(1.2)
        _grow(c)  # the controller's RSS grows past 1.5x its start-up size
        time.sleep(3.5)
        m = _trim_metrics(c)
        if trims:
            assert m["bgc_malloc_trim_seconds_count"] >= 1, m
        else:  # IDLE_PCT=0: the process is never quiet enough
            assert m["bgc_malloc_trim_seconds_count"] == 0 and m["bgc_malloc_trim_deferred_total"] >= 1, m


@pytest.mark.slow
def test_controller_over_half_its_memory_limit_trims_while_busy():
    """The same never-quiet controller (IDLE_PCT=0) under a memory limit it has passed half
    of (BGC_MALLOC_TRIM_LIMIT_MB stands in for the cgroup's memory.max): it trims anyway."""
    env = {"BGC_MALLOC_TRIM_SECS": "1", "BGC_MALLOC_TRIM_MIN_MB": "1", "BGC_MALLOC_TRIM_IDLE_PCT": "0",
           "BGC_MALLOC_TRIM_LIMIT_MB": "2"}
    with Cluster(admission=False, controller_env=env) as c:
        time.sleep(1.2)
        _grow(c)
        time.sleep(3.5)
        assert _trim_metrics(c)["bgc_malloc_trim_seconds_count"] >= 1
        text = requests.get(f"http://127.0.0.1:{c.controller_port}/metrics", timeout=5).text
        assert "bgc_malloc_trim_memory_limit_bytes 2097152" in text

"""The memory-limit valve (native/core/process.cc): the one malloc_trim left.

Round 5 ran a trimmer thread with growth, quiet-interval and 4x heuristics, compensating
for its own 64 MiB heap growth and 512 MiB trim threshold; a pass stalled the process for
13-15 ms (profiles/r5_trim/).  Round 6 bounds the arenas and lets glibc trim heap tops
itself (tune_malloc; profiles/r6_alloc/), so only one valve remains: a process past half its
container's memory limit, and grown 1.5x since the previous pass, trims.
"""
import time

import pytest
import requests

from bacchus_gpu_controller_amd import native
from bacchus_gpu_controller_amd.testing.cluster import Cluster

MB = 1 << 20


@pytest.mark.parametrize("rss,baseline,limit,want", [
    (100 * MB, 0, 0, "skip"),               # no limit known: never
    (100 * MB, 0, 160 * MB, "trim"),        # past half the limit
    (70 * MB, 0, 160 * MB, "skip"),         # under half the limit
    (100 * MB, 80 * MB, 160 * MB, "skip"),  # not grown 1.5x since the last pass: not every check
    (130 * MB, 80 * MB, 160 * MB, "trim"),  # grown again
])
def test_trim_decision(rss, baseline, limit, want):
    assert native().malloc_trim_decision(rss, baseline, limit) == want


def test_cgroup_memory_limit_reads_as_bytes_or_none():
    v = native().cgroup_memory_limit_bytes()
    assert v == 0 or v >= 4096


def _metrics(c):
    text = requests.get(f"http://127.0.0.1:{c.controller_port}/metrics", timeout=5).text
    return text, {l.split()[0]: float(l.split()[1]) for l in text.splitlines()
                  if l.startswith(("bgc_malloc_trim_seconds_count", "bgc_process_resident_memory_bytes",
                                   "bgc_heap_allocated_bytes"))}


def _grow(c, n=600):
    for i in range(n):
        c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                          "metadata": {"name": f"u{i}"},
                                          "spec": {"kube_username": f"u{i}",
                                                   "quota": {"hard": {"requests.amd.com/gpu": "1"}}}})


@pytest.mark.slow
def test_controller_over_half_its_memory_limit_trims():
    """BGC_MALLOC_TRIM_LIMIT_MB stands in for the cgroup's memory.max."""
    env = {"BGC_MALLOC_TRIM_SECS": "1", "BGC_MALLOC_TRIM_LIMIT_MB": "2"}
    with Cluster(admission=False, controller_env=env) as c:
        time.sleep(1.2)
        _grow(c)
        time.sleep(2.5)
        text, m = _metrics(c)
        assert m["bgc_malloc_trim_seconds_count"] >= 1, m
        assert "bgc_malloc_trim_memory_limit_bytes 2097152" in text


@pytest.mark.slow
def test_no_limit_no_trimmer_and_the_heap_stays_near_live():
    """Without a memory limit nothing trims on a timer: the bounded allocator keeps the RSS
    near the live heap by itself."""
    with Cluster(admission=False, controller_env={"BGC_MALLOC_TRIM_SECS": "1", "BGC_MALLOC_TRIM_LIMIT_MB": "0"}) as c:
        _grow(c)
        time.sleep(1.5)
        text, m = _metrics(c)
        assert "bgc_malloc_trim_seconds_count" not in m
        # bounded arenas: a few MB of live heap stays within tens of MB of RSS (a sanitizer
        # build replaces malloc: no glibc heap to measure)
        if m["bgc_heap_allocated_bytes"] > 0:
            assert m["bgc_process_resident_memory_bytes"] < m["bgc_heap_allocated_bytes"] * 2 + 48 * MB, m

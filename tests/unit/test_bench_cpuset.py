"""The bench pins the job to as many CPUs as its cgroup quota grants (harness.quota_cpuset):
unpinned, the threads burst over every visible CPU, spend the quota early in each CFS period
and are frozen for the rest of it."""
from bacchus_gpu_controller_amd.bench import harness


def test_cpulist_round_trip():
    assert harness._cpulist("0-3,8,10-11") == {0, 1, 2, 3, 8, 10, 11}
    assert harness._cpulist_text([1, 2, 3, 5, 7, 8]) == "1-3,5,7-8"
    assert harness._cpulist(harness._cpulist_text(range(16, 32))) == set(range(16, 32))


def test_no_pinning_when_the_quota_covers_the_mask(monkeypatch):
    monkeypatch.setattr(harness.os, "sched_getaffinity", lambda pid: set(range(8)))
    monkeypatch.setattr(harness, "effective_cpus", lambda: 8)
    assert harness.quota_cpuset() is None


def test_quota_sized_set_prefers_the_gpus_numa_cpus_and_skips_cpu0(monkeypatch, tmp_path):
    monkeypatch.setattr(harness.os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(harness, "effective_cpus", lambda: 16)
    # no AMD GPU visible: the first CPUs of the mask, CPU 0 left out
    monkeypatch.setattr(harness.glob, "glob", lambda pattern: [])
    assert harness.quota_cpuset() == list(range(1, 17))
    # an AMD GPU whose NUMA node holds CPUs 64-127
    dev = tmp_path / "renderD128" / "device"
    dev.mkdir(parents=True)
    (dev / "vendor").write_text("0x1002\n")
    (dev / "local_cpulist").write_text("64-127\n")
    monkeypatch.setattr(harness.glob, "glob", lambda pattern: [str(dev)])
    assert harness.quota_cpuset() == list(range(64, 80))

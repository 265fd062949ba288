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


def _box(monkeypatch, local, busy=None):
    # 2 x 64 cores with SMT: CPU c and c + 128 are siblings (the MI355X box's topology)
    monkeypatch.setattr(harness.os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(harness, "effective_cpus", lambda: 16)
    monkeypatch.setattr(harness, "_gpu_local_cpus", lambda: set(local))
    monkeypatch.setattr(harness, "_core_of", lambda c: c % 128)
    monkeypatch.setattr(harness, "_cpu_busy", lambda cpus, interval=0.3: {c: (busy or {}).get(c, 0.0) for c in cpus})


def test_quota_sized_set_prefers_the_gpus_numa_node_and_skips_cpu0(monkeypatch):
    _box(monkeypatch, local=[])  # GPU node unknown: the first CPUs of the mask, not CPU 0
    assert harness.quota_cpuset() == list(range(1, 17))
    _box(monkeypatch, local=list(range(64, 128)) + list(range(192, 256)))
    assert harness.quota_cpuset() == list(range(64, 80))


def test_busy_cpus_and_smt_siblings_come_last(monkeypatch):
    # another tenant holds CPUs 8 and 70 at 100 %: they are skipped for idle ones
    _box(monkeypatch, local=list(range(0, 64)) + list(range(128, 192)), busy={8: 1.0, 12: 0.5})
    cs = harness.quota_cpuset()
    assert len(cs) == 16 and 8 not in cs and 12 not in cs and 0 not in cs
    assert cs == [c for c in range(1, 19) if c not in (8, 12)]
    # one CPU per physical core: never a CPU and its sibling while idle cores remain
    assert len({c % 128 for c in cs}) == 16
    # a node with fewer idle cores than the quota falls back to siblings
    _box(monkeypatch, local=list(range(1, 9)) + list(range(129, 137)))
    cs = harness.quota_cpuset()
    assert sorted(cs) == list(range(1, 9)) + list(range(129, 137))


def test_measured_busy_share_from_proc_stat():
    busy = harness._cpu_busy([0], interval=0.05)
    assert 0.0 <= busy[0] <= 1.0


def test_every_rank_pins_to_rank0s_choice(monkeypatch):
    """The quota covers the whole job: rank 0 chooses the CPU set and every rank applies
    that same set (a rank choosing on its own could pick other CPUs)."""
    chosen = [3, 4, 5]
    pinned = []

    class D:
        def __init__(self, rank):
            self.rank = rank

        def broadcast_obj(self, obj):
            return chosen if self.rank else obj

    monkeypatch.setattr(harness, "quota_cpuset", lambda: chosen)
    monkeypatch.setattr(harness.os, "sched_setaffinity", lambda tid, cs: pinned.append(tuple(cs)))
    assert harness.pin_to_quota(D(0)) == chosen
    monkeypatch.setattr(harness, "quota_cpuset", lambda: (_ for _ in ()).throw(AssertionError("rank 1 chose")))
    assert harness.pin_to_quota(D(1)) == chosen
    assert pinned and set(pinned) == {tuple(chosen)}

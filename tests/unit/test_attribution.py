"""The bench's per-tenant critical path and window tables (bench/attribution.py, the per-thread
readers in bench/harness.py, tools/tail_report.py), on synthetic marks: no cluster."""
import json
import os
import subprocess
import sys

from bacchus_gpu_controller_amd import REPO_ROOT
from bacchus_gpu_controller_amd.bench import attribution, harness

MS = 1_000_000


def _tenant(name, t0, ctl_read_delay_ms=0.0, written_after_read=False):
    """One tenant's marks along the RoleBinding chain, 0.1 ms per stage, with an optional delay
    before the controller reads the status event."""
    stages = ["drv.sched", "drv.sent", "kl.userbootstraps.POST.python.recv", "kl.userbootstraps.POST.python.hook0",
              "adm.review0.CREATE", "adm.review1.CREATE", "kl.userbootstraps.POST.python.hook1",
              "kl.userbootstraps.POST.python.commit", "kl.watch.userbootstraps.synchronizer.sent", "sync.ub_event",
              "sync.dequeue", "sync.quota.send", "kl.userbootstraps.PATCH.x.recv", "adm.review1.UPDATE",
              "kl.userbootstraps.PATCH.x.commit", "sync.status.send", "kl.userbootstraps/status.PUT.s.recv",
              "kl.userbootstraps/status.PUT.s.commit", "kl.watch.userbootstraps.controller.sent"]
    marks, t = [], t0
    for st in stages:
        marks.append([name, st, t])
        t += MS // 10
    sent = t - MS // 10
    t += int(ctl_read_delay_ms * MS)
    read = t
    # kube-lite's clock after its write returned: may come after the reader already read
    marks.append([name, "kl.watch.userbootstraps.controller.written", read + 20_000 if written_after_read else sent + 10_000])
    marks.append([name, "ctl.primary_read", read])
    t = read
    for st in ("ctl.primary_event", "ctl.reconcile0", "ctl.apply.rolebindings.send", "kl.rolebindings.PATCH.x.recv",
               "kl.rolebindings.PATCH.x.commit", "kl.watch.rolebindings.python.sent"):
        t += MS // 10
        marks.append([name, st, t])
    for st in ("drv.ns_seen", "drv.rq_seen", "drv.rb_seen"):
        t += MS // 10
        marks.append([name, st, t])
    return marks


def _fast(n=200):
    """Tenants without a delay: the window's p99 stays below a delayed one's total."""
    return [m for i in range(n) for m in _tenant(f"f{i}", (i + 1) * 100 * MS)]


def test_critical_path_reads_the_watch_leg_to_the_controllers_read():
    marks = _tenant("u1", 0, ctl_read_delay_ms=4.0, written_after_read=True) + _fast()
    out = attribution.analyze([{"marks": marks}], tail_ms=1.0)
    assert out["attributed"] == 201 and not out["unattributed"]
    seg = out["segments"]
    # the read comes before kube-lite's ".written": still on the chain, the write beside it
    assert seg["ctl_watch_sent->ctl_read"]["max_ms"] >= 4.0
    assert "ctl_read->ctl_event" in seg
    assert out["watch_writes"]["userbootstraps.controller"]["n"] == 201
    assert out["tail"]["blame"] == {"ctl_watch_sent->ctl_read": 1}


def test_slow_sections_overlap_the_tail_segment():
    marks = _tenant("u1", 0, ctl_read_delay_ms=6.0)
    t_read = [t for _, st, t in marks if st == "ctl.primary_read"][0]
    stalls = [{"process": "controller", "stalls": [],
               "slow": [[t_read - 1 * MS, 3000.0, "w:userbootstraps queue"],      # inside the segment
                        [t_read + 50 * MS, 2500.0, "w:userbootstraps queue"]]}]   # long after
    out = attribution.analyze([{"marks": marks + _fast()}], stalls, tail_ms=1.0)
    assert out["tail"]["slow_overlap"] == {"controller w:userbootstraps queue": 1}
    assert out["tail"]["examples"][0]["slow_ms"] == {"controller w:userbootstraps queue": 3.0}
    assert out["slow_sections"] == {"controller w:userbootstraps queue": {"n": 2, "max_ms": 3.0}}


def test_waiting_threads_ranks_run_queue_wait_and_keeps_watch_readers():
    t0 = {("controller", "reconcile", str(i)): (1.0, 0.010) for i in range(16)}
    t0.update({("apiserver", "conn:apiserver", "99"): (1.0, 0.0), ("controller", "w:userbootstrap", "7"): (0.5, 0.0)})
    t1 = {k: (v[0] + 0.1, v[1] + 0.002) for k, v in t0.items()}
    t1[("apiserver", "conn:apiserver", "99")] = (1.2, 0.050)
    t1[("controller", "w:userbootstrap", "7")] = (0.6, 0.0001)
    rows = harness.waiting_threads(t0, t1, top=1)
    assert rows[0] == {"process": "apiserver", "thread": "conn:apiserver", "threads": 1, "runq_ms": 50.0,
                       "worst_thread_runq_ms": 50.0}
    # a watch reader is listed even outside the top
    assert rows[1]["thread"] == "w:userbootstrap" and rows[1]["runq_ms"] == 0.1
    busy = harness.busiest_threads(t0, t1, dt=1.0, top=1)
    assert busy == [{"process": "apiserver", "thread": "conn:apiserver", "cpu": 0.2}]


def test_thread_cpu_reads_this_process():
    got = harness.thread_cpu({"me": os.getpid()})
    assert got and all(cpu >= 0 and runq >= 0 for cpu, runq in got.values())
    assert any(tid == str(os.getpid()) for _, _, tid in got)  # the main thread


def test_tail_report_counts_quiet_host_windows(tmp_path):
    def window(p99, foreign=0.0, steal=0.0):
        return {"apply_to_ready_p99_ms": p99, "reconcile_p99_ms": 0.2, "admission_p50_ms": 0.05,
                "job_cpus_used": 2.0, "foreign_cpus": foreign, "steal_cpus": steal, "runqueue_wait_ms_per_s": 50.0}

    def att(idle):
        return {"tail": {"blame": {}, "slow_overlap": {}}, "stalls": {"node-agent": {"n": idle}}}

    run = {"value": 1.0, "latency_at_rate": {
        "this": {"2000": {"windows": [window(7.0), window(6.0, foreign=1.2), window(8.0), window(1.0)]}},
        "reference_controller": {"2000": {"windows": [window(1.0)] * 4}},
        "attribution": {"this": {"2000": [att(0), att(0), att(3), att(0)]},
                        "reference_controller": {"2000": [att(0)] * 4}}}}
    f = tmp_path / "run.json"
    f.write_text(json.dumps(run))
    out = tmp_path / "out.json"
    subprocess.run([sys.executable, os.path.join(REPO_ROOT, "tools", "tail_report.py"), str(f), "--json", str(out)],
                   check=True, capture_output=True)
    s = json.loads(out.read_text())["summary"]["this"]
    # 7.0: quiet host; 6.0: another tenant on the CPUs; 8.0: the idle node agent stalled
    assert s["over_limit"] == 3 and s["over_limit_with_foreign_cpu"] == 1
    assert s["over_limit_on_a_quiet_host"] == 1 and s["quiet_host_windows"] == 2


def test_llc_groups_cover_the_cpus_given():
    cpus = sorted(os.sched_getaffinity(0))
    groups = harness.llc_groups(cpus)
    if groups:  # sysfs cache topology readable
        covered = set()
        for g in groups:
            for part in g.split(","):
                lo, _, hi = part.partition("-")
                covered.update(range(int(lo), int(hi or lo) + 1))
        assert covered == set(cpus)

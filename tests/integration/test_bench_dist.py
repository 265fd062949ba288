"""bench.py under torchrun with 2 ranks (gloo on CPU): the multi-GPU contract the driver
uses for the 2/4/8-GPU scaling runs (one rank per GPU, rank 0 prints one JSON line, the
value aggregates every rank's Ready CRs)."""
import json
import os
import subprocess
import sys

import pytest

from bacchus_gpu_controller_amd import REPO_ROOT
from bacchus_gpu_controller_amd.testing.cluster import free_port

pytestmark = pytest.mark.slow


def test_bench_two_ranks_gloo():
    env = dict(os.environ, BGC_BENCH_CPU="1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO_ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "20", "--rounds", "2",
           "--latency-rates", "200", "--latency-window-s", "1", "--no-reference-arms"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=REPO_ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    # a step is `rounds` rounds of `batch` tenants per rank
    assert d["config"]["global_batch"] == 2 * 20 * 2 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["rounds_per_step"] == 2 and d["config"]["tenants_per_round"] == 20
    assert d["ready_crs"] == 2 * 2 * 20 * 2 and d["failed_crs"] == 0
    assert d["value"] > 0 and d["scaling"] == "weak"
    # config #3's 100 concurrent CRs are split over the ranks
    assert d["config"]["concurrency_per_rank"] == 50 and d["config"]["concurrency_total"] == 100
    assert d["config"]["concurrency_scope"] == "total" and d["config"]["control_plane_cpus"] >= 1
    assert d["config"]["log_level"] == "info" and d["dtype"] == "none"
    # per-rank drivers filter their child watches server-side; the RCCL/xGMI probe runs only
    # on GPU ranks (gloo here)
    assert d["config"]["driver_server_filter"] is True and "rccl_xgmi" not in d
    # per-component CPU cost of the timed region, split product vs test scaffolding
    cpu = d["cpu_ms_per_cr"]
    for k in ("controller", "admission", "synchronizer", "node_agent", "kube_lite", "load_driver", "product_total"):
        assert k in cpu and cpu[k] >= 0
    assert d["apiserver_requests_per_cr"] > 0
    # N>1: the secondary closed-loop phases are N=1 only (they would do N times the work)
    assert "tuned" not in d and "webhook_http1" not in d and "write_latency_2ms" not in d
    # the open-loop phase splits its offered rate over the ranks
    q = d["latency_at_rate"]["this"]["200"]
    # two 1 s windows per rate, each carrying the whole job's offered rate
    assert q["offered_rate"] == 200 and q["ready_crs"] == 400 and q["failed_crs"] == 0
    assert [w["ready_crs"] for w in q["windows"]] == [200, 200]
    # both ranks' tenants are traced through every process and attributed
    for att in d["latency_at_rate"]["attribution"]["this"]["200"]:
        assert att["attributed"] == 200 and att["trace_dropped"] == 0
        # the controller's watch leg splits at its read; kube-lite's writes are timed beside it
        assert {"ctl_watch_sent->ctl_read", "ctl_read->ctl_event"} <= set(att["segments"]), att["segments"]
        assert "userbootstraps.controller" in att["watch_writes"], att["watch_writes"]
        assert "slow_sections" in att
    for w in q["windows"]:  # per-thread CPU and run-queue wait of the window
        assert w["busiest_threads"] and all("runq_ms" in t for t in w["waiting_threads"])
    assert "reference_controller" not in d["latency_at_rate"] and "product_isolated" not in d  # N>1: no isolation


def test_bench_approve_after_create():
    """--approve-after-create: tenants apply, then one sheet edit per step approves them
    (the reference's onboarding order); the JSON times approve -> Ready."""
    cmd = [sys.executable, os.path.join(REPO_ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--batch", "20",
           "--rounds", "1", "--approve-after-create", "--sheet-poll-ms", "300", "--no-tuned-phase", "--write-latency-ms", "1",
           "--latency-rates", "", "--no-isolated-phase"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO_ROOT,
                       env=dict(os.environ, BGC_BENCH_CPU="1"))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert d["ready_crs"] == 40 and d["failed_crs"] == 0
    assert d["config"]["flow"] == "create->approve->Ready" and d["config"]["apiserver_write_latency_ms"] == 1
    assert 0 < d["approve_to_ready_p50_ms"] < 5000
    assert d["create_to_approve_p50_ms"] > 0


def test_default_run_carries_the_reference_arms():
    """The default single-GPU run also times the reference's controller behaviour on the same
    stack and both controllers at an etcd-like write latency; every
    arm's percentiles come from whole windows."""
    cmd = [sys.executable, os.path.join(REPO_ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--batch", "20",
           "--rounds", "1", "--no-tuned-phase", "--no-http1-phase", "--arm-steps", "2", "--arm-warmup", "1",
           "--latency-rates", "100,200", "--latency-window-s", "1", "--time-budget-s", "0"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO_ROOT,
                       env=dict(os.environ, BGC_BENCH_CPU="1"))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert d["vs_baseline"] is None and d["samples_complete"] is True
    assert "skipped_phases" not in d and d["phase_wall_s"]["total"] > 0
    assert d["reconciles"] == d["reconcile_total_delta"] and d["webhook_calls"] == d["webhook_calls_total_delta"]
    rc = d["reference_controller"]
    assert rc["semantics"] == "reference-controller" and rc["failed_crs"] == 0 and rc["value"] > 0
    assert rc["reconciles"] == rc["reconcile_total_delta"] and rc["this_over_reference_cr_per_s"] > 0
    wl = d["write_latency_2ms"]
    for side in ("this", "reference_controller"):
        assert wl[side]["apiserver_write_latency_ms"] == 2 and wl[side]["failed_crs"] == 0
        assert wl[side]["steps"] == 2 and wl[side]["reconciles"] == wl[side]["reconcile_total_delta"]
    assert wl["this_over_reference_cr_per_s"] > 0
    # open loop at equal offered rates, both controllers
    q = d["latency_at_rate"]
    assert q["rates_cr_per_s"] == [100, 200] and q["arrivals"] == "poisson (open loop)"
    assert q["windows_per_arm"] == 2 and q["order"].startswith("A B B A")
    assert q["kube_lite_watch_coalesce_us"] == 0  # the windows time latency without the hold
    for side in ("this", "reference_controller"):
        for rate in ("100", "200"):
            r = q[side][rate]
            assert r["failed_crs"] == 0 and r["ready_crs"] == 2 * int(rate) and len(r["windows"]) == 2
            assert r["reconcile_p99_ms"] > 0 and r["admission_p50_ms"] > 0
            # (the exact 2 % check belongs to the box run; sanitizer builds here are slower)
            assert abs(r["achieved_rate"] - r["offered_rate"]) <= 0.2 * r["offered_rate"]
            # every tenant of every window is attributed along its critical path
            for att in q["attribution"][side][rate]:
                assert att["attributed"] == int(rate), att
                assert att["critical_child"] and att["segments"]
                seg = att["segments"]
                assert "arrival->sent" in seg and any(k.endswith("->seen") for k in seg)
    assert set(q["this_over_reference"]) == {"100", "200"}
    for row in q["this_over_reference"].values():
        assert len(row["reconcile_p99_lower_by_window"]) == 2
    # the compact stage table is the line's last field (the driver keeps the output's tail)
    assert list(d)[-1] == "stage_table" and set(d["stage_table"]["this"]) == {"100", "200"}
    # the headline again with fixtures and product on disjoint CPUs
    pi = d["product_isolated"]
    assert pi["failed_crs"] == 0 and pi["value"] > 0 and pi["reconcile_p99_ms"] > 0
    assert pi["cpus"]["fixtures"] and pi["cpus"]["product"]


def test_auto_concurrency_follows_cpu_share():
    from bacchus_gpu_controller_amd.bench.harness import auto_concurrency, effective_cpus

    # the MI355X box: 16-CPU quota -> 8 per rank alone, 4 per rank from 4 ranks up
    assert [auto_concurrency(n, 16) for n in (1, 2, 4, 8)] == [8, 6, 4, 4]
    # a bigger share keeps more tenants in flight, capped at 32 per rank
    assert [auto_concurrency(n, 128) for n in (1, 2, 4, 8)] == [32, 32, 32, 23]
    assert 1 <= effective_cpus() <= (os.cpu_count() or 1)


def test_single_tenant_bench_config1():
    """BASELINE config #1 as a bench mode: crdgen byte-identical to the chart, and tenants
    onboarded one at a time through the whole stack with per-stage latencies."""
    cmd = [sys.executable, "-m", "bacchus_gpu_controller_amd.bench.single", "--tenants", "4"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO_ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert d["config"] == 1 and d["crdgen"]["byte_identical"] and d["tenants"] == 4
    st = d["apply_to_stage_ms"]
    # each stage is seen on its own watch stream, so their order is not asserted: under load
    # one stream's delivery can lag another's by more than the gap between the writes
    assert all(0 < st[k]["p50"] < 5000 for k in ("namespace", "quota", "rolebinding"))
    assert d["reconcile_ms"]["p50"] > 0


def test_time_budget_skips_the_secondary_phases():
    """--time-budget-s: once the run's wall time (plus the next phase's estimate) passes the
    budget, the secondary phases (write-latency arms, tuned, HTTP/1.1 webhook) are left out
    and listed; the headline, the reference controller and latency_at_rate always run."""
    cmd = [sys.executable, os.path.join(REPO_ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--batch", "20",
           "--rounds", "1", "--latency-rates", "100", "--latency-window-s", "1", "--no-isolated-phase",
           "--time-budget-s", "0.5"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO_ROOT,
                       env=dict(os.environ, BGC_BENCH_CPU="1"))
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert set(d["skipped_phases"]) >= {"rl", "ml", "w"}
    assert "write_latency_2ms" not in d and "webhook_http1" not in d
    assert d["value"] > 0 and d["reference_controller"]["value"] > 0 and d["latency_at_rate"]["this"]["100"]

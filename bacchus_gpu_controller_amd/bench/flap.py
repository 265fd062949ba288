"""BASELINE config #5 as a timed benchmark: node drain/re-add and all-GPU flaps under tenant
churn, with synchronizer convergence after a sheet edit.

    python -m bacchus_gpu_controller_amd.bench.flap [--nodes 4] [--rounds 5] [--json-out f]

Cluster: kube-lite + TLS admission + controller + synchronizer (watch mode, Drive version
poll) + one native node agent per synthetic 8x MI355X node (mock amdsmi backends, one xGMI
hive each; with --real-gpu one more agent on the host's real GPUs via amdsmi).  Services
run at the chart defaults (RUST_LOG=info, 1 s telemetry poll, 3-poll hysteresis, 30 s
heartbeat, 5 s sheet poll) unless overridden.  A background thread keeps onboarding and
deleting tenants for the whole run.

Each round times, from the apiserver's point of view (10 ms polling):
  drain_republish   Node deleted (after a cordon) -> re-published with its amd.com/gpu
                    capacity and xGMI labels (the agent's Node watch; heartbeat is 30 s)
  flap_unhealthy    all 8 GPUs of a node overheat -> allocatable 0 + AMDGPUHealthy=False
  flap_recover      temperatures back to normal   -> allocatable 8
  sheet_converge    the operator edits every tenant's GPU quota in the sheet -> every
                    tenant's ResourceQuota carries the new value
The reference has no node-side component (nothing reacts to a drain or a GPU fault) and
converges a sheet edit on its 60 s tick plus one controller pass
(src/synchronizer.rs:192-212, src/controller.rs:154): its structural sheet_converge is
U(0, 60 s) + processing.
"""
import argparse
import copy
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from bacchus_gpu_controller_amd.testing.cluster import Cluster  # noqa: E402
from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle  # noqa: E402
from bacchus_gpu_controller_amd.testing.kubeapi import ApiError  # noqa: E402


def _pct(v, q):
    if not v:
        return None
    s = sorted(v)
    return round(s[min(len(s) - 1, int(q * len(s)))], 2)


def _until(pred, timeout, step=0.01):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < timeout:
        if pred():
            return (time.perf_counter() - t0) * 1e3
        time.sleep(step)
    raise TimeoutError(f"not converged within {timeout}s")


def _ub(name):
    return {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": name}, "spec": {}}


class Churn(threading.Thread):
    """Background tenant churn: create a tenant, delete the one created `keep` steps ago."""

    def __init__(self, cluster, rate_hz, keep=20):
        super().__init__(daemon=True)
        self.c, self.period, self.keep = cluster, 1.0 / rate_hz, keep
        self.stop_ev = threading.Event()
        self.created = self.deleted = self.errors = 0

    def run(self):
        i = 0
        while not self.stop_ev.is_set():
            try:
                self.c.as_user(f"oidc:churn{i}", ["gpu"]).create("userbootstraps", _ub(f"churn{i}"))
                self.created += 1
                if i >= self.keep:
                    self.c.admin.delete("userbootstraps", f"churn{i - self.keep}")
                    self.deleted += 1
            except (ApiError, OSError):
                self.errors += 1
            i += 1
            self.stop_ev.wait(self.period)

    def stop(self):
        self.stop_ev.set()
        self.join(10)


def run(args):
    google = FakeGoogle().start()
    tenants = [f"tenant{i:03d}" for i in range(args.tenants)]
    churn_rows = [{"id_username": f"churn{i}", "gpu": 1} for i in range(3000)]

    def rows(round_no):
        return [{"id_username": u, "gpu": 1 + (i + round_no) % 8} for i, u in enumerate(tenants)] + churn_rows

    google.set_rows(rows(0))
    nodes = [f"mi355x-{i}" for i in range(args.nodes)]
    out = {"drain_republish_ms": [], "flap_unhealthy_ms": [], "flap_recover_ms": [], "sheet_converge_ms": []}
    agent_env = {"CONF_HEARTBEAT_SECS": str(args.heartbeat_secs)}
    t_start = time.time()
    with Cluster(log_level=args.log_level, controller_env={"CONF_WORKERS": "16"}) as c:
        for i, n in enumerate(nodes):
            c.start_node_agent(node_name=n, backend="mock", hive_id=0x355000 + i, proc_name=f"na-{n}",
                               poll_interval_ms=args.poll_ms, extra_env=agent_env)
        if args.real_gpu:
            c.start_node_agent(node_name="mi355x-real", backend="amdsmi", proc_name="na-real",
                               poll_interval_ms=args.poll_ms, extra_env=agent_env)
            nodes.append("mi355x-real")
        c.start_synchronizer(google, interval=60, extra_env={"CONF_WATCH": "true",
                                                            "CONF_SHEET_POLL_MS": str(args.sheet_poll_ms)})
        a = c.admin

        def capacity(n):
            node = a.get_or_none("nodes", n)
            return None if node is None else node.get("status", {}).get("capacity", {}).get("amd.com/gpu")

        def alloc(n):
            node = a.get_or_none("nodes", n)
            return None if node is None else node.get("status", {}).get("allocatable", {}).get("amd.com/gpu")

        for n in nodes:
            _until(lambda: capacity(n) is not None, 30)
        for u in tenants:
            c.as_user(f"oidc:{u}", ["gpu"]).create("userbootstraps", _ub(u))

        def converged(round_no):
            want = {u: str(1 + (i + round_no) % 8) for i, u in enumerate(tenants)}
            for q in a.list("resourcequotas")["items"]:
                u = q["metadata"]["name"]
                if u in want and q["spec"]["hard"].get("requests.amd.com/gpu") == want[u]:
                    want.pop(u)
            return not want

        _until(lambda: converged(0), 60)
        churn = Churn(c, args.churn_hz)
        churn.start()
        try:
            for r in range(1, args.rounds + 1):
                # drain + re-add
                n = nodes[r % len(nodes)]
                a.merge_patch("nodes", n, {"spec": {"unschedulable": True}})
                a.delete("nodes", n)
                out["drain_republish_ms"].append(_until(lambda: capacity(n) is not None, 60))
                # all-GPU flap (mock nodes only: the fixture is the GPU)
                m = nodes[(r + 1) % args.nodes]
                fx = json.load(open(c.fixtures[m]))
                hot = copy.deepcopy(fx)
                for g in hot["gpus"]:
                    g["telemetry"]["temp_hotspot_c"] = 121
                c.set_gpu_fixture(m, hot)
                out["flap_unhealthy_ms"].append(_until(lambda: alloc(m) == "0", 60))
                c.set_gpu_fixture(m, fx)
                out["flap_recover_ms"].append(_until(lambda: alloc(m) == "8", 60))
                # sheet edit -> every tenant's quota
                google.set_rows(rows(r))
                out["sheet_converge_ms"].append(_until(lambda: converged(r), 120, step=0.02))
                print(json.dumps({"round": r, **{k: round(v[-1], 1) for k, v in out.items()}}), flush=True)
        finally:
            churn.stop()
        alive = {name: p.alive() for name, p in c.procs.items()}
    google.stop()
    res = {
        "metric": "config #5: node drain/re-add + all-GPU flap under tenant churn; synchronizer convergence (ms)",
        "nodes": args.nodes + (1 if args.real_gpu else 0), "gpus_per_node": 8, "tenants": args.tenants,
        "rounds": args.rounds, "churn_hz": args.churn_hz, "churn_created": churn.created,
        "churn_deleted": churn.deleted, "churn_errors": churn.errors,
        "poll_interval_ms": args.poll_ms, "heartbeat_secs": args.heartbeat_secs, "sheet_poll_ms": args.sheet_poll_ms,
        "log_level": args.log_level, "wall_s": round(time.time() - t_start, 1), "processes_alive": alive,
    }
    for k, v in out.items():
        res[k] = {"p50": _pct(v, 0.5), "p99": _pct(v, 0.99), "max": round(max(v), 2) if v else None,
                  "mean": round(statistics.mean(v), 2) if v else None, "samples": [round(x, 1) for x in v]}
    res["reference_structural"] = {
        "drain_republish": "none (no node-side component)", "flap": "none (no GPU health)",
        "sheet_converge_s": "U(0, 60) + one reconcile (src/synchronizer.rs:192, src/controller.rs:154)"}
    return res


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nodes", type=int, default=4)
    ap.add_argument("--tenants", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--churn-hz", type=float, default=20.0)
    ap.add_argument("--poll-ms", type=int, default=1000, help="telemetry poll (chart default 1000)")
    ap.add_argument("--heartbeat-secs", type=int, default=30)
    ap.add_argument("--sheet-poll-ms", type=int, default=5000)
    ap.add_argument("--log-level", default="info")
    ap.add_argument("--real-gpu", action="store_true", help="add an amdsmi node agent for this host's GPUs")
    ap.add_argument("--json-out", default="")
    args = ap.parse_args(argv)
    res = run(args)
    line = json.dumps(res)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")
    print(line, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

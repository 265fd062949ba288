#!/usr/bin/env python3
"""Open-loop window table from bench.py JSON lines (latency_at_rate, round 6).

For every run and every window of each arm: apply->Ready p99, reconcile p99, the job's own
CPU use and other tenants' CPU use on the job's CPU set, and (when traced) the segment the
window's tail tenants spent the longest in, the slow section (stall::note_slow) most of
them overlapped, and for a window over the limit the thread that waited longest for a CPU.
"idle" counts the node agent's stalls (an idle process: the host took its CPU); a window
with none, no steal and foreign_cpus < 0.5 counts as on a quiet host.  Ends with the count of windows over --limit-ms
per arm.

  python3 tools/tail_report.py gpurun_out/r6_tg*.json [--limit-ms 5] [--json out.json]
"""
import argparse
import json


def rows(path):
    d = json.load(open(path))
    q = d.get("latency_at_rate") or {}
    att = q.get("attribution", {})
    for arm in ("this", "reference_controller"):
        for rate, v in (q.get(arm) or {}).items():
            for k, w in enumerate(v.get("windows", [])):
                a = (att.get(arm, {}).get(rate) or [None] * 8)[k] if att else None
                blame = slow = None
                if a and a["tail"]["blame"]:
                    blame = max(a["tail"]["blame"].items(), key=lambda kv: kv[1])[0]
                if a and a["tail"].get("slow_overlap"):
                    slow = max(a["tail"]["slow_overlap"].items(), key=lambda kv: kv[1])[0]
                wt = (w.get("waiting_threads") or [None])[0]
                # the node agent is idle during these windows: its stall sampler firing means
                # the host took CPUs from every process, not that the stack was busy
                idle = (a or {}).get("stalls", {}).get("node-agent", {}).get("n")
                yield {"run": path, "value": d.get("value"), "arm": arm, "rate": rate, "window": k,
                       "a2r_p99_ms": w.get("apply_to_ready_p99_ms"), "reconcile_p99_ms": w.get("reconcile_p99_ms"),
                       "admission_p50_ms": w.get("admission_p50_ms"), "job_cpus": w.get("job_cpus_used"),
                       "foreign_cpus": w.get("foreign_cpus"), "runq_ms_per_s": w.get("runqueue_wait_ms_per_s"),
                       "steal_cpus": w.get("steal_cpus"), "idle_process_stalls": idle,
                       "tail_blame": blame, "tail_slow_section": slow,
                       "most_runq": f"{wt['process']}/{wt['thread']} {wt['runq_ms']}ms" if wt else None}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("files", nargs="+")
    ap.add_argument("--limit-ms", type=float, default=5.0)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    all_rows = [r for f in a.files for r in rows(f)]
    print(f"{'run':34s} {'arm':5s} {'rate':>5s} w  {'a2r99':>6s} {'rec99':>6s} {'job':>5s} {'foreign':>7s} {'idle':>4s}  tail blame [slow section] (thread with most run-queue wait)")
    for r in all_rows:
        print(f"{r['run'][-34:]:34s} {r['arm'][:5]:5s} {r['rate']:>5s} {r['window']}  {r['a2r_p99_ms'] or 0:6.2f} "
              f"{r['reconcile_p99_ms'] or 0:6.3f} {r['job_cpus'] if r['job_cpus'] is not None else '':>5} "
              f"{r['foreign_cpus'] if r['foreign_cpus'] is not None else '':>7} "
              f"{r['idle_process_stalls'] if r['idle_process_stalls'] is not None else '':>4}  {r['tail_blame'] or ''}"
              + (f" [{r['tail_slow_section']}]" if r["tail_slow_section"] else "")
              + (f" ({r['most_runq']})" if r["most_runq"] and (r["a2r_p99_ms"] or 0) > a.limit_ms else ""))
    def quiet(r):
        """No sign of the host in the window: no other tenant on the job's CPUs, no steal,
        and the idle node agent's stall sampler silent (None: not traced, not known)."""
        return ((r["foreign_cpus"] or 0) < 0.5 and (r["steal_cpus"] or 0) < 0.05
                and r["idle_process_stalls"] == 0)

    summary = {}
    for arm in ("this", "reference_controller"):
        ws = [r for r in all_rows if r["arm"] == arm]
        over = [r for r in ws if (r["a2r_p99_ms"] or 0) > a.limit_ms]
        summary[arm] = {"windows": len(ws), "over_limit": len(over),
                        "over_limit_with_foreign_cpu": sum(1 for r in over if (r["foreign_cpus"] or 0) >= 0.5),
                        "over_limit_on_a_quiet_host": sum(1 for r in over if quiet(r)),
                        "quiet_host_windows": sum(1 for r in ws if quiet(r)),
                        "max_a2r_p99_ms": max((r["a2r_p99_ms"] or 0 for r in ws), default=None)}
    pairs = [(t, r) for t in all_rows if t["arm"] == "this" for r in all_rows
             if r["arm"] == "reference_controller" and r["run"] == t["run"] and r["rate"] == t["rate"]
             and r["window"] == t["window"]]
    summary["reconcile_p99_this_lower"] = f"{sum(1 for t, r in pairs if t['reconcile_p99_ms'] < r['reconcile_p99_ms'])}" \
                                          f" of {len(pairs)} window pairs"
    summary["limit_ms"] = a.limit_ms
    print(json.dumps(summary, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"summary": summary, "windows": all_rows}, f, indent=1)


if __name__ == "__main__":
    main()

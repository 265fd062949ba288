#!/usr/bin/env python3
"""One-screen summary of bench.py JSON lines (headline, arms, latency_at_rate, isolation).

    python3 tools/bench_summary.py gpurun_out/<dir>/bench_*.json
    python3 tools/bench_summary.py --aggregate profiles/r5_*/bench_*.json   # medians, ranges, window counts

`--aggregate` prints the figures the README's results tables quote: median (min-max) over
the runs given, and in how many latency_at_rate windows this build's reconcile p99 and
admission p50 are below the reference controller's.
"""
import json
import statistics
import sys


def main(paths):
    for p in paths:
        d = json.load(open(p))
        print(f"{p}: {d['value']:.0f} CR/s, reconcile p99 {d['reconcile_p99_ms']} ms, admission p50 "
              f"{d['admission_p50_ms']} ms, apply->Ready p99 {d['apply_to_ready_p99_ms']} ms, "
              f"cpu/CR {d['cpu_ms_per_cr']}")
        rc = d.get("reference_controller")
        if rc:
            print(f"  reference controller: {rc['value']:.0f} CR/s, reconcile p99 {rc['reconcile_p99_ms']}, "
                  f"admission p50 {rc['admission_p50_ms']}, ratio {rc.get('this_over_reference_cr_per_s')}")
        q = d.get("latency_at_rate")
        if q:
            for side in ("this", "reference_controller"):
                for rate, v in q.get(side, {}).items():
                    print(f"  {side:20s} {rate:>6s}: achieved {v['achieved_rate']}, reconcile p99 {v['reconcile_p99_ms']}"
                          f" p50 {v['reconcile_p50_ms']}, admission p50 {v['admission_p50_ms']} p99 "
                          f"{v.get('admission_p99_ms')}, a2r p50 {v['apply_to_ready_p50_ms']} p99 {v['apply_to_ready_p99_ms']},"
                          f" reconciles {v.get('reconciles')}, failed {v['failed_crs']}")
            print(f"  this/reference: {q.get('this_over_reference')}")
        pi = d.get("product_isolated")
        if pi:
            print(f"  isolated: {pi['value']:.0f} CR/s, cpus {pi['cpus']}, reconcile p99 {pi['reconcile_p99_ms']}, "
                  f"admission p50 {pi['admission_p50_ms']}, handler p50 {pi['admission_handler_p50_ms']}, "
                  f"a2r p50 {pi['apply_to_ready_p50_ms']}, throttled {pi.get('cgroup_throttled')}")


def _rng(xs, fmt="{:.4g}"):
    xs = [x for x in xs if x is not None]
    if not xs:
        return "-"
    return f"{fmt.format(statistics.median(xs))} ({fmt.format(min(xs))}-{fmt.format(max(xs))})"


def aggregate(paths):
    rows = [json.load(open(p)) for p in paths]
    print(f"{len(rows)} runs")
    print("headline CR/s       ", _rng([r["value"] for r in rows], "{:.0f}"))
    print("reconcile p99 ms    ", _rng([r["reconcile_p99_ms"] for r in rows]))
    print("admission p50 ms    ", _rng([r["admission_p50_ms"] for r in rows]))
    ref = [r["reference_controller"] for r in rows if r.get("reference_controller")]
    if ref:
        print("reference CR/s      ", _rng([x["value"] for x in ref], "{:.0f}"))
        print("this/reference      ", _rng([x["this_over_reference_cr_per_s"] for x in ref], "{:.3f}"))
    iso = [r["product_isolated"] for r in rows if r.get("product_isolated")]
    if iso:
        print("isolated CR/s       ", _rng([x["value"] for x in iso], "{:.0f}"))
        print("isolated rec p99    ", _rng([x["reconcile_p99_ms"] for x in iso]))
        print("isolated adm p50    ", _rng([x["admission_p50_ms"] for x in iso]))
    lar = [r["latency_at_rate"] for r in rows if r.get("latency_at_rate", {}).get("reference_controller")]
    if not lar:
        return
    for rate in lar[0]["this"]:
        t = [x["this"][rate] for x in lar if rate in x["this"] and rate in x["reference_controller"]]
        f = [x["reference_controller"][rate] for x in lar if rate in x["this"] and rate in x["reference_controller"]]
        for key, label in (("reconcile_p99_ms", "reconcile p99"), ("admission_p50_ms", "admission p50"),
                           ("apply_to_ready_p99_ms", "apply->Ready p99")):
            lower = sum(a[key] < b[key] for a, b in zip(t, f))
            print(f"{rate:>6s} CR/s {label:17s} this {_rng([a[key] for a in t])} / reference "
                  f"{_rng([b[key] for b in f])}; this lower in {lower} of {len(t)}")
        dev = max(abs(v["achieved_rate"] - float(rate)) / float(rate) * 100 for v in t + f)
        print(f"{rate:>6s} CR/s achieved rate within {dev:.2f} % of the offered rate in every window")


if __name__ == "__main__":
    if sys.argv[1:2] == ["--aggregate"]:
        aggregate(sys.argv[2:])
    else:
        main(sys.argv[1:])

#!/usr/bin/env python3
"""One-screen summary of bench.py JSON lines (headline, arms, latency_at_rate, isolation).

    python3 tools/bench_summary.py gpurun_out/<dir>/bench_*.json
"""
import json
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
                          f"{v['admission_p99_ms']}, a2r p50 {v['apply_to_ready_p50_ms']} p99 {v['apply_to_ready_p99_ms']},"
                          f" reconciles {v['reconciles']}, failed {v['failed_crs']}")
            print(f"  this/reference: {q.get('this_over_reference')}")
        pi = d.get("product_isolated")
        if pi:
            print(f"  isolated: {pi['value']:.0f} CR/s, cpus {pi['cpus']}, reconcile p99 {pi['reconcile_p99_ms']}, "
                  f"admission p50 {pi['admission_p50_ms']}, handler p50 {pi['admission_handler_p50_ms']}, "
                  f"a2r p50 {pi['apply_to_ready_p50_ms']}, throttled {pi.get('cgroup_throttled')}")


if __name__ == "__main__":
    main(sys.argv[1:])

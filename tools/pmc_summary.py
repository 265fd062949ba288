#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc CSV runs of the diagnostic kernels into derived metrics.

    python3 tools/pmc_summary.py gpurun_out/pmc > profiles/archive/pmc_diag_r1.json

Expects sub-runs sq/ (SQ_* + GRBM_*), fetch/ (FETCH_SIZE) and write/ (WRITE_SIZE), each with
<name>_counter_collection.csv and <name>_kernel_trace.csv.
gfx950 notes applied: FETCH_SIZE counts half the bytes of wide coalesced reads (x2), GRBM_GUI_ACTIVE
is summed over the 8 XCDs, and SQ_VALU_MFMA_BUSY_CYCLES is summed over the 1024 SIMDs.
"""
import collections
import csv
import json
import os
import sys

SIMDS = 256 * 4
XCDS = 8


def load(d, name):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(os.path.join(d, name, f"{name}_counter_collection.csv"))):
        agg[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    t = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(os.path.join(d, name, f"{name}_kernel_trace.csv"))):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        n[k] += 1
    return agg, t, n


def main(d):
    sq, t_sq, n_sq = load(d, "sq")
    fe, t_fe, _ = load(d, "fetch")
    wr, t_wr, _ = load(d, "write")
    out = {}
    for k in sq:
        if k.startswith("__amd"):
            continue
        e = {"dispatches": n_sq[k], "kernel_time_s": round(t_sq[k], 6)}
        gui = sq[k]["GRBM_GUI_ACTIVE"] / XCDS
        e["effective_clock_ghz"] = round(gui / t_sq[k] * 1e-9, 3) if t_sq[k] else None
        if sq[k]["SQ_VALU_MFMA_BUSY_CYCLES"]:
            e["mfma_busy_fraction"] = round(sq[k]["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * SIMDS), 4)
        rd = fe.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 * 2  # x2: gfx950 FETCH_SIZE under-counts wide reads
        wb = wr.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        if rd > 1e6:
            e["hbm_read_tbps"] = round(rd / t_fe[k] * 1e-12, 3)
        if wb > 1e6:
            e["hbm_write_tbps"] = round(wb / t_wr[k] * 1e-12, 3)
        if rd > 1e6 and wb > 1e6:
            e["hbm_read_plus_write_tbps"] = round((rd / t_fe[k] + wb / t_wr[k]) * 1e-12, 3)  # concurrent in one kernel
        e["waves"] = int(sq[k]["SQ_WAVES"])
        out[k] = e
    print(json.dumps({"source": "rocprofv3 --pmc (counters only) on 1x MI355X, workload tools/probes/gpu_probe.py",
                      "kernels": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])

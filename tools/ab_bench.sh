#!/usr/bin/env bash
# Interleaved A/B of the headline bench on one box: base binaries (BGC_BIN_DIR=$1, a
# directory holding the binaries under test, e.g. an older build of admission and
# controller next to symlinks to the current bin/) against the current build, $2 rounds
# of (base, current), further args passed to bench.py.  Writes gpurun_out/ab/<arm>_<i>.json.
set -o pipefail
base=${1:?base bin dir}; rounds=${2:-3}; shift 2
out=gpurun_out/ab
mkdir -p "$out"
for i in $(seq 1 "$rounds"); do
  BGC_BIN_DIR="$PWD/$base" timeout -k 10 300 python -u bench.py "$@" > "$out/base_$i.json" 2> "$out/base_$i.err" || exit $?
  timeout -k 10 300 python -u bench.py "$@" > "$out/cur_$i.json" 2> "$out/cur_$i.err" || exit $?
done
python3 - "$out" "$rounds" <<'PY'
import json, statistics, sys
out, rounds = sys.argv[1], int(sys.argv[2])
rows = {}
for arm in ("base", "cur"):
    for i in range(1, rounds + 1):
        d = json.loads(open(f"{out}/{arm}_{i}.json").read().strip().splitlines()[-1])
        r = rows.setdefault(arm, {"value": [], "admission": [], "controller": [], "product_total": [],
                                  "admission_p50_ms": [], "reconcile_p99_ms": []})
        r["value"].append(d["value"])
        for k in ("admission", "controller", "product_total"):
            r[k].append(d["cpu_ms_per_cr"][k])
        r["admission_p50_ms"].append(d["admission_p50_ms"])
        r["reconcile_p99_ms"].append(d["reconcile_p99_ms"])
summary = {arm: {k: {"median": statistics.median(v), "all": v} for k, v in r.items()} for arm, r in rows.items()}
json.dump(summary, open(f"{out}/summary.json", "w"), indent=1)
for k in rows["base"]:
    print(f"{k:18s} base {statistics.median(rows['base'][k]):9.4f}  cur {statistics.median(rows['cur'][k]):9.4f}")
PY

#!/usr/bin/env bash
# Consecutive default bench runs on the GPU box, each with its tail tenants' timelines dumped
# (--trace-dump), for tools/tail_report.py and offline study.  Output: gpurun_out/$OUT_NAME/.
set -o pipefail
OUT=gpurun_out/${OUT_NAME:-tail_runs}
mkdir -p "$OUT"
for i in $(seq 1 "${RUNS:-6}"); do
  timeout -k 10 300 python -u bench.py --trace-dump "$OUT/td_$i" > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || exit $?
  echo "run $i done"
done

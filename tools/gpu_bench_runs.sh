#!/usr/bin/env bash
# N default bench.py runs with --report-cpu on a 1-GPU box (run through gpurun from the repo
# root): per-process CPU, RSS and malloc_trim passes in every JSON.  Each run has its own
# time limit; the first failure ends the call.  Output: gpurun_out/${OUT_NAME}/bench_<i>.json.
#   OUT_NAME=r5_runs RUNS=5 bash tools/gpu_bench_runs.sh
set -o pipefail
OUT=gpurun_out/${OUT_NAME:-bench_runs}
RUNS=${RUNS:-3}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in $(seq 1 "$RUNS"); do
  s=$(date +%s)
  timeout -k 10 420 python -u bench.py --report-cpu > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || exit $?
  echo "bench_$i run_s=$(( $(date +%s) - s ))" | tee -a "$OUT/timing.txt"
done

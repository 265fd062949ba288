#!/usr/bin/env bash
# Long-window headline bench on the MI355X box (through gpurun, from the repo root):
# one default bench.py run with STEPS timed steps (default 100: about 12 s of timed churn,
# against the driver's 20 steps), then the node agent's RSS and kube-lite's from the JSON.
# Output lands in gpurun_out/long_bench/.
set -o pipefail
OUT=gpurun_out/long_bench
STEPS=${STEPS:-100}
mkdir -p "$OUT"
export TMPDIR=/tmp
# the headline phase only: the secondary phases and reference arms would run as long
timeout -k 10 600 python -u bench.py --steps "$STEPS" --warmup 5 --no-tuned-phase --no-http1-phase --no-reference-arms \
    > "$OUT/bench_long.json" 2> "$OUT/bench_long.err" &&
timeout -k 10 300 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
rc=$?
cut -c1-400 "$OUT/bench_long.json" "$OUT/bench_default.json"
exit $rc

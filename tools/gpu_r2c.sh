#!/usr/bin/env bash
# Round-2 GPU pass c: headline bench (twice), config #4 TP=8 co-scheduling bench with the
# real MI355X as a fifth node, rocprofv3 kernel stats of the HIP diagnostics.
set -o pipefail
OUT=gpurun_out/r2c
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step bench-1 &&
timeout -k 10 300 python -u bench.py --json-out "$OUT/bench_1.json" > "$OUT/bench_1.log" 2>&1 &&
step bench-2 &&
timeout -k 10 300 python -u bench.py --json-out "$OUT/bench_2.json" > "$OUT/bench_2.log" 2>&1 &&
step tp8 &&
timeout -k 10 300 python -u -m bacchus_gpu_controller_amd.bench.tp8 --real-gpu --json-out "$OUT/tp8.json" > "$OUT/tp8.log" 2>&1 &&
step rocprof-diag &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_diag" -o diag -- python3 tools/diag_floor_sweep.py "$OUT/diag_floors_rocprof.json" > "$OUT/rocprof_diag.log" 2>&1
rc=$?
step "done rc=$rc"
for f in "$OUT"/bench_*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['reconcile_p99_ms'], d['admission_p50_ms'], d['apply_to_ready_p99_ms'], d['cpu_ms_per_cr'], d['tuned']['value'])"; done
exit $rc

#!/usr/bin/env bash
# Round-2 GPU pass (run through gpurun from the repo root): GPU tests, the config #5 flap
# bench with the real MI355X as one node, the headline bench, create->approve->Ready, and a
# rocprofv3 kernel trace of the diagnostics.  Each step has its own time limit and the
# steps are chained with && so the first failure ends the call.
set -o pipefail
OUT=gpurun_out/r2b
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest-gpu &&
timeout -k 10 400 python -u -m pytest tests/gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
step flap &&
timeout -k 10 300 python -u -m bacchus_gpu_controller_amd.bench.flap --real-gpu --rounds 5 --json-out "$OUT/flap.json" > "$OUT/flap.log" 2>&1 &&
step bench-default &&
timeout -k 10 300 python -u bench.py --json-out "$OUT/bench_default.json" > "$OUT/bench_default.log" 2>&1 &&
step bench-approve &&
timeout -k 10 400 python -u bench.py --no-tuned-phase --approve-after-create --steps 10 --warmup 1 --json-out "$OUT/bench_approve.json" > "$OUT/bench_approve.log" 2>&1 &&
step rocprof-diag &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_diag" -o diag -- python3 tools/diag_floor_sweep.py "$OUT/diag_floors_rocprof.json" > "$OUT/rocprof_diag.log" 2>&1
rc=$?
step "done rc=$rc"
tail -3 "$OUT/pytest_gpu.log"
exit $rc

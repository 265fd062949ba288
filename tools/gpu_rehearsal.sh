#!/usr/bin/env bash
# Round-end rehearsal on a 1-GPU MI355X box (run through gpurun from the repo root):
#   pytest -m gpu, smoke(), BENCH_RUNS default bench.py runs (default 1; extra flags in
#   BENCH_ARGS, e.g. --report-cpu; BENCH_ONLY=1: just those), rocprofv3 kernel
#   stats of smoke().  Every GPU step has its own time limit and the steps are chained with
#   &&, so the first failure ends the call.  Output lands in gpurun_out/${OUT_NAME:-rehearsal}/.
set -o pipefail
OUT=gpurun_out/${OUT_NAME:-rehearsal}
RUNS=${BENCH_RUNS:-1}
mkdir -p "$OUT"
export TMPDIR=/tmp
bench_runs() {
  for i in $(seq 1 "$RUNS"); do
    s=$(date +%s)
    # shellcheck disable=SC2086
    timeout -k 10 420 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || return $?
    echo "bench_$i run_s=$(( $(date +%s) - s ))" >> "$OUT/timing.txt"
  done
}
if [ -n "${BENCH_ONLY:-}" ]; then  # only the bench runs (a tail study): no tests, no profile
  bench_runs
  rc=$?
  cat "$OUT/timing.txt" 2>/dev/null
  exit $rc
fi
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 240 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 &&
bench_runs &&
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/$OUT/prof" -- python3 -c \
    "import sys; sys.path.insert(0, '$GRAFT_REPO_ROOT'); import __graft_entry__ as g; g.smoke()" \
    > "$GRAFT_REPO_ROOT/$OUT/rocprof.log" 2>&1)
rc=$?
tail -3 "$OUT/pytest_gpu.log"; tail -2 "$OUT/smoke.log"; cat "$OUT/timing.txt" 2>/dev/null
exit $rc

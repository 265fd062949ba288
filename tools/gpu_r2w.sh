#!/usr/bin/env bash
# Round-2 GPU pass w: re-verify a tree rebuilt from source in a fresh container —
# GPU tests, smoke() under rocprofv3 kernel stats, headline bench at defaults.
set -o pipefail
OUT=${OUT:-gpurun_out/r2w}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
step smoke && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/smoke_prof" -o smoke \
  -- python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
step bench && timeout -k 10 300 python -u bench.py --report-cpu --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 \
  || { tail -30 "$OUT/bench.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
find "$OUT/smoke_prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/smoke_kernel_stats.csv" \;
tail -1 "$OUT/bench.log"
step done

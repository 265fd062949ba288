#!/usr/bin/env bash
# Round-2 GPU pass d: telemetry poll cost per cadence on the real MI355X, under rocprofv3
# --marker-trace (roctx ranges bgc.telemetry.poll.{fast,slow,ras}), then GPU tests.
set -o pipefail
OUT=gpurun_out/r2d
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[$(date +%T)] telemetry probe" &&
timeout -k 10 120 python3 tools/telemetry_probe.py 240 > "$OUT/telemetry_probe.json" 2> "$OUT/telemetry_probe.err" &&
echo "[$(date +%T)] rocprof marker trace" &&
(cd /tmp && timeout -k 10 180 rocprofv3 --marker-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/roctx" \
   -o telemetry -- python3 "$GRAFT_REPO_ROOT/tools/telemetry_probe.py" 240 > "$GRAFT_REPO_ROOT/$OUT/rocprof.log" 2>&1) &&
echo "[$(date +%T)] pytest gpu" &&
timeout -k 10 400 python -u -m pytest tests/gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "[$(date +%T)] done rc=$rc"
cat "$OUT/telemetry_probe.json" | head -c 600; echo
find "$OUT/roctx" -name "*marker*stats*" -exec cat {} \;
tail -2 "$OUT/pytest_gpu.log"
exit $rc

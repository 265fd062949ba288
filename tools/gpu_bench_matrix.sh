#!/usr/bin/env bash
# Headline bench matrix on a 1-GPU MI355X box (run through gpurun from the repo root).
#   1. default bench.py (BASELINE config #3: 100 in flight, RUST_LOG=info, tuned phase)
#   2. this build vs the reference's controller behaviour, at 0 and 2 ms API write latency
#   3. full reference semantics (60 s sheet tick) at 0 ms, few steps
#   4. create -> approve -> Ready at the product's 5 s sheet poll
# Each run has its own time limit; runs are chained with && so the first failure ends
# the call.  JSON lines land in gpurun_out/matrix/.
set -o pipefail
OUT=${OUT:-gpurun_out/matrix}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, timeout, bench args...
  local name=$1 t=$2
  shift 2
  echo "[$(date +%T)] $name: bench.py $*"
  timeout -k 10 "$t" python -u bench.py "$@" --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1
}
run default 300 &&
run this_wl0 300 --no-tuned-phase &&
run refctl_wl0 300 --no-tuned-phase --semantics reference-controller &&
run this_wl2 300 --no-tuned-phase --write-latency-ms 2 &&
run refctl_wl2 300 --no-tuned-phase --semantics reference-controller --write-latency-ms 2 &&
run ref_wl0 400 --no-tuned-phase --semantics reference --steps 3 --warmup 1 &&
run approve 400 --no-tuned-phase --approve-after-create --steps 10 --warmup 1
rc=$?
for f in "$OUT"/*.json; do echo "$f"; python3 -c "
import json,sys
d=json.load(open('$f'))
keys=['value','ms_per_step','reconcile_p99_ms','admission_p50_ms','apply_to_ready_p50_ms','apply_to_ready_p99_ms',
      'approve_to_ready_p50_ms','apiserver_requests_per_cr','failed_crs']
print({k:d.get(k) for k in keys}, d.get('cpu_ms_per_cr'), (d.get('tuned') or {}).get('value'))"; done
exit $rc

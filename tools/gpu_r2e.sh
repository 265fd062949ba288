#!/usr/bin/env bash
# Round-2 GPU pass e: webhook callouts over HTTP/2 (default) vs HTTP/1.1 (--webhook-http1),
# interleaved A/B of the headline bench on the MI355X box.
set -o pipefail
OUT=gpurun_out/r2e
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
run() {  # name, extra args
  step "$1" && timeout -k 10 300 python -u bench.py --json-out "$OUT/$1.json" "${@:2}" > "$OUT/$1.log" 2>&1
}
run h2_a && run h1_a --apiserver-arg=--webhook-http1 && run h2_b && run h1_b --apiserver-arg=--webhook-http1
rc=$?
step "done rc=$rc"
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['reconcile_p99_ms'], d['admission_p50_ms'], d['apply_to_ready_p99_ms'], d['cpu_ms_per_cr'], d['tuned']['value'])"; done
exit $rc

#!/usr/bin/env bash
# Round-2 GPU pass e: API server -> webhook over HTTP/2 (--webhook-http2, multiplexed
# streams like the real apiserver) vs HTTP/1.1 (kube-lite's default), interleaved A/B of
# the headline bench on the MI355X box, 3 runs each.
set -o pipefail
OUT=${OUT:-gpurun_out/r2e}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
run() {  # name, extra args
  step "$1" && timeout -k 10 300 python -u bench.py --json-out "$OUT/$1.json" "${@:2}" > "$OUT/$1.log" 2>&1
}
H2=--apiserver-arg=--webhook-http2
run h2_1 $H2 && run h1_1 && run h2_2 $H2 && run h1_2 && run h2_3 $H2 && run h1_3
rc=$?
step "done rc=$rc"
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['config']['webhook_protocol'], d['value'], 'adm_rt_p50', d['admission_p50_ms'], 'adm_handler_p50', d['admission_handler_p50_ms'], 'ready_p99', d['apply_to_ready_p99_ms'], d['cpu_ms_per_cr'], 'tuned', d['tuned']['value'], d['tuned']['admission_p50_ms'])"; done
exit $rc

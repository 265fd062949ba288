#!/usr/bin/env bash
# Round-2 GPU pass i: webhook protocol at N=4/8 gloo ranks (800 creates in flight at N=8):
# one multiplexed h2 connection (default) vs 4 h2 connections vs the HTTP/1.1 pool.
set -o pipefail
OUT=gpurun_out/r2i
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
nn() {  # n, name, extra args
  step "$2" && BGC_BENCH_CPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $1 \
    --master-addr 127.0.0.1 --master-port $((29600+$1)) bench.py --gpus $1 --steps 20 --warmup 3 --report-cpu \
    --no-tuned-phase --json-out "$OUT/$2.json" "${@:3}" > "$OUT/$2.log" 2>&1
}
nn 8 n8_wh1 --apiserver-arg=--webhook-http1 && nn 8 n8_wc4 --apiserver-arg=--webhook-h2-connections --apiserver-arg=4 &&
nn 8 n8_wc1 && nn 4 n4_wh1 --apiserver-arg=--webhook-http1 && nn 4 n4_wc4 --apiserver-arg=--webhook-h2-connections --apiserver-arg=4
rc=$?
step "done rc=$rc"
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['cpu_ms_per_cr']; print('$f', d['config']['webhook_protocol'], d['value'], 'adm', d['admission_p50_ms'], d['admission_p99_ms'], 'srv99', d.get('admission_h2_server_p99_ms'), 'ready99', d['apply_to_ready_p99_ms'], 'kl', c['kube_lite'], 'prod', c['product_total'])"; done
exit $rc

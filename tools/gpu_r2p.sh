#!/usr/bin/env bash
# Round-2 GPU pass p: webhook protocol at N=4/8 gloo ranks after the kube-lite store-lock change.
set -o pipefail
OUT=${OUT:-gpurun_out/r2p}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
nn() {  # n, name, extra args
  step "$2" && BGC_BENCH_CPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $1 \
    --master-addr 127.0.0.1 --master-port $((29600+$1)) bench.py --gpus $1 --steps 20 --warmup 3 --report-cpu \
    --no-tuned-phase --json-out "$OUT/$2.json" "${@:3}" > "$OUT/$2.log" 2>&1
}
H1=--apiserver-arg=--webhook-http1
nn 8 n8_h2 && nn 8 n8_h1 $H1 && nn 8 n8_h2b && nn 8 n8_h1b $H1 && nn 4 n4_h2 && nn 4 n4_h1 $H1 && nn 2 n2_h2 && nn 2 n2_h1 $H1
rc=$?
step "done rc=$rc"
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['cpu_ms_per_cr']; print('$f', d['config']['webhook_protocol'], d['value'], 'kl', c['kube_lite'], 'adm_cpu', c['admission'], 'prod', c['product_total'], 'adm', d['admission_p50_ms'], d['admission_p99_ms'], 'ready99', d['apply_to_ready_p99_ms'])"; done
exit $rc

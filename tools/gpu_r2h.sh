#!/usr/bin/env bash
# Round-2 GPU pass h: the load driver (tenants = kubectl/client-go users) over HTTP/2
# (default) vs HTTP/1.1 keep-alive pools, at N=1 on the MI355X and N=4/8 gloo ranks
# (BGC_BENCH_CPU=1, ranks do not touch the card) on the box's 16-CPU share.
set -o pipefail
OUT=${OUT:-gpurun_out/r2h}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
n1() {  # name, extra args
  step "$1" && timeout -k 10 300 python -u bench.py --report-cpu --json-out "$OUT/$1.json" "${@:2}" > "$OUT/$1.log" 2>&1
}
nn() {  # n, name, extra args
  step "$2" && BGC_BENCH_CPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $1 \
    --master-addr 127.0.0.1 --master-port $((29600+$1)) bench.py --gpus $1 --steps 20 --warmup 3 --report-cpu \
    --no-tuned-phase --json-out "$OUT/$2.json" "${@:3}" > "$OUT/$2.log" 2>&1
}
n1 n1_h2 --driver-http2 && n1 n1_h1 && n1 n1_h2b --driver-http2 && n1 n1_h1b &&
nn 4 n4_h2 --driver-http2 && nn 4 n4_h1 && nn 8 n8_h2 --driver-http2 && nn 8 n8_h1
rc=$?
step "done rc=$rc"
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['cpu_ms_per_cr']; print('$f', d['config']['driver_protocol'], d['value'], 'adm', d['admission_p50_ms'], 'rec99', d['reconcile_p99_ms'], 'ready99', d['apply_to_ready_p99_ms'], 'kl', c['kube_lite'], 'prod', c['product_total'], 'drv', c['load_driver'], 'tuned', (d.get('tuned') or {}).get('value'))"; done
exit $rc

#!/usr/bin/env bash
# Round-2 GPU pass o: kube-lite store lock, writer-preferring rwlock (default) vs one
# mutex (BGC_KL_RWLOCK=mutex), at N=8 and N=4 gloo ranks and N=1 on the MI355X.
set -o pipefail
OUT=${OUT:-gpurun_out/r2o}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
nn() {  # n, name, lock
  step "$2" && BGC_KL_RWLOCK=$3 BGC_BENCH_CPU=$([ $1 -gt 1 ] && echo 1 || echo 0) timeout -k 10 300 python -u -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $((29600+$1)) bench.py --gpus $1 --steps 20 \
    --warmup 3 --report-cpu --no-tuned-phase --json-out "$OUT/$2.json" > "$OUT/$2.log" 2>&1
}
nn 8 n8_rw writer && nn 8 n8_mx mutex && nn 8 n8_rw2 writer && nn 8 n8_mx2 mutex && nn 4 n4_rw writer && nn 4 n4_mx mutex &&
nn 1 n1_rw writer && nn 1 n1_mx mutex
rc=$?
step "done rc=$rc"
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['cpu_ms_per_cr']; l=d.get('apiserver_store_lock', {}); print('$f', d['value'], 'kl', c['kube_lite'], 'prod', c['product_total'], 'adm', d['admission_p50_ms'], 'ready99', d['apply_to_ready_p99_ms'], 'lockwait_ms', round(l.get('wait_ms', 0)))"; done
exit $rc

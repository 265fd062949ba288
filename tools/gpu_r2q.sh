#!/usr/bin/env bash
# Round-2 GPU pass q: headline bench at defaults (3 runs), then the scale rehearsal
# (N=1 on the MI355X, N=2/4/8 gloo ranks on the box's CPU share).
set -o pipefail
OUT=${OUT:-gpurun_out/r2q}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
for i in 1 2 3; do
  step "bench $i" && timeout -k 10 300 python -u bench.py --report-cpu --json-out "$OUT/bench_$i.json" > "$OUT/bench_$i.log" 2>&1 || exit 1
done
step scale && bash tools/bench_scale_rehearsal.sh > "$OUT/scale.log" 2>&1 && cp -r gpurun_out/scale "$OUT/scale"
rc=$?
step "done rc=$rc"
for f in "$OUT"/bench_*.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['cpu_ms_per_cr']; print('$f', d['value'], 'rec99', d['reconcile_p99_ms'], 'adm', d['admission_p50_ms'], 'ready', d['apply_to_ready_p50_ms'], d['apply_to_ready_p99_ms'], 'prod', c['product_total'], 'kl', c['kube_lite'], 'tuned', d['tuned']['value'], 'req/CR', d.get('apiserver_requests_per_cr'))"; done
cat "$OUT/scale.log" | tail -5
exit $rc

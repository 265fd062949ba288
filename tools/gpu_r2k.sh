#!/usr/bin/env bash
# Round-2 GPU pass k: controller child watches metadata-only (default) vs full objects,
# interleaved A/B of the headline bench with per-process CPU.
set -o pipefail
OUT=${OUT:-gpurun_out/r2k}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
run() {  # name, extra args
  step "$1" && timeout -k 10 300 python -u bench.py --report-cpu --json-out "$OUT/$1.json" "${@:2}" > "$OUT/$1.log" 2>&1
}
F=--controller-env=CONF_METADATA_WATCHES=false
run meta_1 && run full_1 $F && run meta_2 && run full_2 $F && run meta_3 && run full_3 $F
rc=$?
step "done rc=$rc"
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['cpu_ms_per_cr']; print('$f', d['value'], 'rec99', d['reconcile_p99_ms'], 'ready99', d['apply_to_ready_p99_ms'], 'ctrl', c['controller'], 'kl', c['kube_lite'], 'prod', c['product_total'], 'tuned', (d.get('tuned') or {}).get('value'))"; done
exit $rc

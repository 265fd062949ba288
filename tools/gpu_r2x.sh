#!/usr/bin/env bash
# Round-2 GPU pass x: scale rehearsal A/B of the load drivers' server-side child-watch
# filter (kube-lite.test/name-prefix) against the old client-side line filter, interleaved.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2x/filter_1 bash tools/bench_scale_rehearsal.sh > /dev/null 2>&1 || exit 1
echo "[$(date +%T)] filter 1 done"
OUT=gpurun_out/r2x/nofilter_1 EXTRA=--no-driver-server-filter bash tools/bench_scale_rehearsal.sh > /dev/null 2>&1 || exit 1
echo "[$(date +%T)] nofilter 1 done"
OUT=gpurun_out/r2x/filter_2 bash tools/bench_scale_rehearsal.sh > /dev/null 2>&1 || exit 1
echo "[$(date +%T)] filter 2 done"
for d in filter_1 nofilter_1 filter_2; do
  python3 -c "
import json; rows=json.load(open('gpurun_out/r2x/$d/summary.json'))
print('$d', [(r['n'], r['cr_s'], r['cpu_ms_per_cr']['kube_lite'], r['cpu_ms_per_cr']['load_driver'], r['cpu_ms_per_cr']['product_total']) for r in rows])"
done

#!/usr/bin/env bash
# Worker-count sweep of the headline bench (one process tree at a time):
#   tools/bench_sweep.sh OUT_DIR
set -uo pipefail
cd "$(dirname "$0")/.."
out=${1:?out dir}
mkdir -p "$out"
for cfg in "16 32" "32 32" "64 32" "32 64" "64 64"; do
  set -- $cfg
  tag="sync$1-ctrl$2"
  timeout -k 10 300 python3 bench.py --steps 30 --warmup 2 --sync-workers "$1" --controller-workers "$2" \
    --report-cpu --json-out "$out/$tag.json" > "$out/$tag.log" 2>&1 || { echo "$tag failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$tag.json')); print('$tag', d['value'], d['reconcile_p99_ms'], d['admission_p50_ms'], d['stage_p50_ms'], d['apply_to_ready_p50_ms'])"
done

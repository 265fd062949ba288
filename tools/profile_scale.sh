#!/usr/bin/env bash
# Sampling profiles of every service under an N-rank gloo bench (ranks do not touch the
# GPU): what grows with N.   tools/profile_scale.sh OUT_DIR N
set -euo pipefail
cd "$(dirname "$0")/.."
out=${1:?out dir}; n=${2:-8}
mkdir -p "$out/raw"
out=$(cd "$out" && pwd)
rm -f "$out"/raw/*.prof
BGC_CPU_PROFILE="$out/raw/%p.prof" BGC_BENCH_CPU=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus "$n" --steps 20 --warmup 3 \
  --report-cpu --no-tuned-phase --json-out "$out/bench.json" > "$out/bench.log" 2>&1
for f in "$out"/raw/*.prof; do
  bin=$(grep -m1 -o "/bin/[a-z-]*$" "$f" | head -1 | sed 's#/bin/##')
  [ -n "$bin" ] || bin=unknown
  python3 tools/cpuprof_report.py "$f" --top 40 --collapsed "$out/$bin.collapsed" > "$out/$bin.txt"
done
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['cpu_ms_per_cr'])"

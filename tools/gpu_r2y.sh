#!/usr/bin/env bash
# Round-2 GPU pass y: GEMM soak A/B, the shipped 2-stage BK=64 kernel vs the 4-stage BK=32
# pipeline (BGC_SOAK_KERNEL=deep), interleaved; checksums at every size first.
set -o pipefail
OUT=${OUT:-gpurun_out/r2y}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp SOAK_VS_TORCH=0
for i in 1 2; do
  echo "[$(date +%T)] deep $i" && BGC_SOAK_KERNEL=deep timeout -k 10 180 python -u tools/soak_probe.py "$OUT/deep_$i.json" > "$OUT/deep_$i.log" 2>&1 || { tail -20 "$OUT/deep_$i.log"; exit 1; }
  echo "[$(date +%T)] base $i" && timeout -k 10 180 python -u tools/soak_probe.py "$OUT/base_$i.json" > "$OUT/base_$i.log" 2>&1 || { tail -20 "$OUT/base_$i.log"; exit 1; }
done
for f in "$OUT"/*.json; do python3 -c "
import json; rs=json.load(open('$f')); print('$f', [(r['m'], r['passed'], round(r['tflops_mean']), round(r['tflops_best'])) for r in rs if 'm' in r and r['m']>=1024])"; done

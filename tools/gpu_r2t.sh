#!/usr/bin/env bash
# Round-2 GPU pass t: GEMM soak, 256x256 kernel with float4 C stores vs one 4-byte store per element
# kernel, interleaved A/B/A/B, then torch.matmul as the yardstick.
set -o pipefail
OUT=${OUT:-gpurun_out/r2t}
rm -rf "$OUT" && mkdir -p "$OUT"
export SOAK_VS_TORCH=0
for i in 1 2; do
  echo "vec-c $i" && timeout -k 10 180 python -u tools/soak_probe.py "$OUT/vecc_$i.json" > "$OUT/vecc_$i.log" 2>&1 || { cat "$OUT/vecc_$i.log"; exit 1; }
  echo "scalar-c $i" && BGC_SOAK_KERNEL=scalar-c timeout -k 10 180 python -u tools/soak_probe.py "$OUT/scalarc_$i.json" > "$OUT/scalarc_$i.log" 2>&1 || exit 1
done
SOAK_VS_TORCH=1 timeout -k 10 240 python -u tools/soak_probe.py "$OUT/with_torch.json" > "$OUT/with_torch.log" 2>&1 || exit 1
for f in "$OUT"/*.json; do python3 - "$f" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1].split("/")[-1], [(r["m"], r["tile"], round(r["tflops_mean"]), round(r["tflops_best"]), r["row_mismatches"] + r["col_mismatches"]) for r in d if "m" in r], [r["torch_matmul"] for r in d if "torch_matmul" in r])
PY
done

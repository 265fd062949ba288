#!/usr/bin/env bash
# Round-2 GPU pass u: PMC counters (counters only, no trace domains) of the two 256x256 soak
# kernels at 8192^3, one run per kernel.
set -o pipefail
OUT=${OUT:-gpurun_out/r2u}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for kern in phased 2phase; do
  if [ "$kern" = 2phase ]; then export BGC_SOAK_KERNEL=2phase; else unset BGC_SOAK_KERNEL; fi
  echo "pmc $kern"
  timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/$kern" -o sq -- python3 tools/soak_one.py 8192 8192 8192 5 > "$OUT/$kern.log" 2>&1 || { tail -20 "$OUT/$kern.log"; exit 1; }
done
find "$OUT" -name "*counter_collection.csv" | while read -r f; do
  python3 - "$f" <<'PY'
import collections, csv, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if not k.startswith("gemm_soak"):
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    w = c["SQ_WAVE_CYCLES"] or 1
    print(sys.argv[1], k, {x: round(c[x] / w, 3) for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")},
          "bank_conflict_per_lds_inst", round(c["SQ_LDS_BANK_CONFLICT"] / max(1, c["SQ_INSTS_LDS"]), 3),
          "mfma_busy_fraction", round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1, c["GRBM_GUI_ACTIVE"] / 8 * 1024), 3),
          "gui_active", c["GRBM_GUI_ACTIVE"])
PY
done

#!/usr/bin/env bash
# PMC counters (counters only, no trace domains) of the 256x256 soak kernels at 8192^3:
# BGC_SOAK_KERNEL values in $KERNELS (default "2buf pingpong"), one rocprofv3 pass each.
#   OUT=gpurun_out/pmc_soak [KERNELS="pingpong0 pingpong"] bash tools/pmc_soak.sh
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_soak}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for kern in ${KERNELS:-2buf pingpong}; do
  export BGC_SOAK_KERNEL=$kern
  echo "pmc $kern"
  timeout -s KILL 90 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d "$OUT/$kern" -o sq -- python3 tools/probes/soak_one.py 8192 8192 8192 5 > "$OUT/$kern.log" 2>&1 || { tail -20 "$OUT/$kern.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, json, os, re, sys
out = {}
name = lambda s: re.sub(r"^void ", "", s.replace("(anonymous namespace)::", "")).split("(")[0]
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*", "*counter_collection.csv"))):
    arm = os.path.relpath(f, sys.argv[1]).split(os.sep)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = name(r["Kernel_Name"])
        if k.startswith("gemm_"):
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    t, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(f.replace("counter_collection", "kernel_trace"))):
        k = name(r["Kernel_Name"])
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        n[k] += 1
    for k, c in agg.items():
        w = c["SQ_WAVE_CYCLES"] or 1
        out[f"{arm}:{k}"] = {**{x: round(c[x] / w, 3) for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")},
                             "lds_bank_conflicts_per_lds_instr": round(c["SQ_LDS_BANK_CONFLICT"] / max(1, c["SQ_INSTS_LDS"]), 3),
                             # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs
                             "mfma_busy": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1, c["GRBM_GUI_ACTIVE"] / 8 * 1024), 3),
                             "clock_ghz": round(c["GRBM_GUI_ACTIVE"] / 8 / t[k] / 1e9, 3) if t[k] else None,
                             "ms_per_launch_profiled": round(t[k] / n[k] * 1e3, 3) if n[k] else None}
json.dump(out, open(os.path.join(sys.argv[1], "summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
PY

#!/usr/bin/env bash
# PMC counters (counters only, no trace domains) of the register-operand matrix-core
# kernels: bf16 mfma_throughput and the MX fp8/fp4 mfma_lowp_throughput, as the node
# agent's check runs them (ops.mfma_lowp, ops.mfma).  One rocprofv3 pass.
#   OUT=gpurun_out/pmc_mx bash tools/pmc_mx.sh
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_mx}
rm -rf "$OUT" && mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
    --output-format csv -d "$OUT/run" -o mx -- python3 -c \
    "import sys; sys.path.insert(0, '.'); from bacchus_gpu_controller_amd import ops; ops.mfma(0); ops.mfma_lowp(0); ops.mfma_lowp(0)" \
    > "$OUT/run.log" 2>&1 || { tail -20 "$OUT/run.log"; exit 1; }
python3 - "$OUT" <<'PY'
import collections, csv, glob, json, os, re, sys
name = lambda s: re.sub(r"^void ", "", s.replace("(anonymous namespace)::", "")).split("(")[0]
out = {}
for f in glob.glob(os.path.join(sys.argv[1], "run", "**", "*counter_collection.csv"), recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = name(r["Kernel_Name"])
        if "throughput" in k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    t, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(f.replace("counter_collection", "kernel_trace"))):
        k = name(r["Kernel_Name"])
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        n[k] += 1
    for k, c in agg.items():
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs
        out[k] = {"mfma_busy": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1, c["GRBM_GUI_ACTIVE"] / 8 * 1024), 3),
                  "clock_ghz": round(c["GRBM_GUI_ACTIVE"] / 8 / t[k] / 1e9, 3) if t[k] else None,
                  "launches": n[k], "ms_per_launch_profiled": round(t[k] / n[k] * 1e3, 3) if n[k] else None}
json.dump(out, open(os.path.join(sys.argv[1], "summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
PY

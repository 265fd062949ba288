"""GEMM soak kernels A/B in one process (cdna guide §5.4 rule 24: interleaved rounds):
the kernels named in $KERNELS (BGC_SOAK_KERNEL values: 2buf = double-buffered, round 2;
pingpong = the 8-phase kernel; a variant under test gets its own value), on the soak's
{-1,0,1} operands, plus an ABFT race screen over several shapes.  Writes
gpurun_out/soak_ab.json."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from bacchus_gpu_controller_amd import native  # noqa: E402

n = native()
rounds = int(os.environ.get("ROUNDS", "4"))
kernels = os.environ.get("KERNELS", "2buf,pingpong").split(",")
out = {"screen": [], "ab": {}}
# race screen: every shape, both kernels, checksums exact
for m, nn, k in ((256, 256, 128), (512, 768, 1024), (768, 512, 384), (1024, 1024, 4096), (4096, 8192, 2048),
                 (2048, 2048, 8192)):
    for kern in kernels:
        os.environ["BGC_SOAK_KERNEL"] = kern
        r = json.loads(n.diag_gemm_soak(0, m, nn, k, 3, 0x51 + m))
        out["screen"].append({"m": m, "n": nn, "k": k, "req": kern, "kernel": r["kernel"], "passed": r["passed"],
                              "row_mismatches": r["row_mismatches"], "col_mismatches": r["col_mismatches"]})
        print(out["screen"][-1], flush=True)
for size in (4096, 8192):
    res = {k: [] for k in kernels}
    for rd in range(rounds):
        for kern in kernels:
            os.environ["BGC_SOAK_KERNEL"] = kern
            r = json.loads(n.diag_gemm_soak(0, size, size, size, 20 if size == 8192 else 40, 7 + rd))
            assert r["passed"], r
            res[kern].append({"mean": r["tflops_mean"], "best": r["tflops_best"], "kernel": r["kernel"]})
            print(size, kern, rd, round(r["tflops_mean"], 1), round(r["tflops_best"], 1), flush=True)
    out["ab"][str(size)] = {k: {"median_mean_tflops": statistics.median(x["mean"] for x in v),
                                "median_best_tflops": statistics.median(x["best"] for x in v), "runs": v}
                            for k, v in res.items()}
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/soak_ab.json", "w"), indent=1)
print(json.dumps({s: {k: round(v["median_mean_tflops"], 1) for k, v in d.items()} for s, d in out["ab"].items()}))
print("screen all passed:", all(x["passed"] for x in out["screen"]))

"""Measure the HIP diagnostics at the node agent's sizes to set DiagFloors defaults.

Runs (on cuda:0) the HBM test at several buffer sizes and the MFMA test at the agent's
setting (16 waves/CU, 2048 iters) a few times each, plus the GEMM host cross-check, and
prints/writes a JSON summary (min / median per metric)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bacchus_gpu_controller_amd import native, ops


def main(out_path):
    n = native()
    res = {"hbm": {}, "mfma": [], "gemm": None}
    for mb in (256, 512, 1024, 2048):
        runs = [ops.hbm(0, nbytes=mb << 20, iters=2) for _ in range(3)]
        res["hbm"][str(mb)] = {k: {"min": min(r[k] for r in runs), "median": statistics.median(r[k] for r in runs)}
                               for k in ("read_gbps", "copy_gbps", "write_gbps", "elapsed_ms")}
        print(mb, res["hbm"][str(mb)], flush=True)
    for _ in range(3):
        r = ops.mfma(0, waves_per_cu=16, iters=2048)
        res["mfma"].append({k: r[k] for k in ("tflops", "xcc_balance", "xcc_wave_us", "xccs_seen", "cus_seen",
                                              "elapsed_ms", "mismatches")})
        print(res["mfma"][-1], flush=True)
    t0 = time.time()
    res["gemm"] = json.loads(n.diag_gemm_check(0, 64, 64, 512, 0x5eed))
    res["gemm"]["wall_ms"] = (time.time() - t0) * 1e3
    print(res["gemm"], flush=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag_floors.json")

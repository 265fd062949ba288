"""MX fp8 / fp4 matrix-core check on the MI355X: tiles, scaled tiles and dense rates at a
few occupancies.  Writes gpurun_out/lowp_probe.json.

    python3 tools/probes/lowp_probe.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from bacchus_gpu_controller_amd import ops  # noqa: E402


def main():
    out = []
    for waves, iters in [(16, 1024), (32, 4096), (32, 16384), (64, 8192), (32, 4096)]:
        t0 = time.time()
        r = ops.mfma_lowp(0, waves, iters)
        r["waves_per_cu"], r["iters"], r["wall_s"] = waves, iters, round(time.time() - t0, 3)
        out.append(r)
        print(json.dumps({k: r[k] for k in ("waves_per_cu", "iters", "fp8_tflops", "fp4_tflops", "fp8_mismatches",
                                            "fp8_scaled_mismatches", "fp4_mismatches", "fp4_scaled_mismatches",
                                            "cus_seen", "throughput_ok", "elapsed_ms")}), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/lowp_probe.json", "w") as f:
        json.dump(out, f, indent=1)
    return 0 if all(r["passed"] for r in out) else 1


if __name__ == "__main__":
    sys.exit(main())

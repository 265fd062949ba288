"""Power, clocks and rate of the burn-in on each matrix-core path of one MI355X (bf16, MX
fp8, MX fp4): which one is the harder power/thermal stress?

    python3 tools/probes/burn_dtype_probe.py [seconds=4]

Writes gpurun_out/burn_dtype_probe.json; one line per dtype on stdout."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from bacchus_gpu_controller_amd import native  # noqa: E402

KEYS = ("dtype", "tflops_mean", "tflops_max", "sustain", "power_mean_w", "power_max_w", "gfxclk_mean_mhz",
        "max_hotspot_c", "ppt_violation_pct", "thermal_violation_pct", "mismatches")


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    n = native()
    backend = n.gpu_backend("amdsmi")
    out = {}
    for dtype in ("bf16", "fp8", "fp4", "bf16"):
        r = json.loads(n.diag_burn(backend, 0, 0, int(seconds * 1000), 0x5EED, dtype))
        row = {k: r.get(k) for k in KEYS}
        row["passed"] = json.loads(n.judge_diag(json.dumps({"burn": r})))["passed"]
        out.setdefault(dtype, []).append(row)
        print(json.dumps(row), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/burn_dtype_probe.json", "w") as f:
        json.dump(out, f, indent=1)
    return 0 if all(r["passed"] and r["mismatches"] == 0 for rows in out.values() for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())

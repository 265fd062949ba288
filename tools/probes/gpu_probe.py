#!/usr/bin/env python3
"""Print a JSON report of the MI355X diagnostics + amdsmi telemetry cost (GPU box)."""
import json
import statistics
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

from bacchus_gpu_controller_amd import native, ops  # noqa: E402


def main():
    n = native()
    out = {"arch": ops.device_arch(0), "devices": ops.device_count(), "library": ops.library_path()}
    out["hbm"] = ops.hbm(0, nbytes=4 << 30, iters=5)
    out["mfma"] = ops.mfma(0, waves_per_cu=32, iters=16384)
    b = n.gpu_backend("amdsmi", "")
    out["discover"] = json.loads(b.discover())
    lat = []
    for _ in range(200):
        t0 = time.perf_counter()
        b.sample(0)
        lat.append((time.perf_counter() - t0) * 1e6)
    out["amdsmi_sample_us"] = {"p50": statistics.median(lat), "p99": sorted(lat)[int(0.99 * len(lat)) - 1],
                               "mean": statistics.mean(lat)}
    out["telemetry_sample"] = json.loads(b.sample(0))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Telemetry hot-path probe: N polls of the native TelemetryPoller over all local GPUs
(amdsmi), reporting per-poll latency. Run under `rocprofv3 --marker-trace` to see the
`bgc.telemetry.poll` roctx ranges."""
import json
import statistics
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from bacchus_gpu_controller_amd import native  # noqa: E402


def main(polls=240, slow_every=10, ras_every=60):
    """Polls at the node agent's cadences (every 10th poll reads VRAM/ECC totals, every
    60th the RAS counters) and reports the wall time of each kind of poll separately."""
    n = native()
    b = n.gpu_backend("amdsmi", "")
    gpus = json.loads(b.discover())
    p = n.TelemetryPoller(b, [g["index"] for g in gpus], 1000, "{}", slow_every, ras_every)
    lat = {"fast": [], "slow": [], "ras": []}
    for i in range(polls):
        kind = "ras" if i % ras_every == 0 else "slow" if i % slow_every == 0 else "fast"
        t0 = time.perf_counter()
        p.poll_once()
        lat[kind].append((time.perf_counter() - t0) * 1e6)
    out = {"gpus": len(gpus), "polls": polls, "slow_every": slow_every, "ras_every": ras_every,
           "roctx": n.roctx_available()}
    for k, v in lat.items():
        v.sort()
        out[k] = {"n": len(v), "p50_us": round(statistics.median(v), 1), "max_us": round(v[-1], 1)}
    # time-averaged cost of the side thread per poll interval
    out["mean_poll_us"] = round(sum(sum(v) for v in lat.values()) / polls, 1)
    out["snapshot"] = json.loads(p.snapshot())["devices"][0]
    print(json.dumps(out))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 240)

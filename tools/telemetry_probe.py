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


def main(polls=200):
    n = native()
    b = n.gpu_backend("amdsmi", "")
    gpus = json.loads(b.discover())
    p = n.TelemetryPoller(b, [g["index"] for g in gpus], 1000)
    lat = []
    for _ in range(polls):
        t0 = time.perf_counter()
        p.poll_once()
        lat.append((time.perf_counter() - t0) * 1e6)
    lat.sort()
    print(json.dumps({"gpus": len(gpus), "polls": polls, "roctx": n.roctx_available(),
                      "poll_us_p50": statistics.median(lat), "poll_us_p99": lat[int(0.99 * len(lat)) - 1],
                      "poll_us_min": lat[0], "snapshot": json.loads(p.snapshot())["devices"][0]}))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)

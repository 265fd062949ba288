"""Telemetry poll cost vs device count: a TelemetryPoller over N mock
MI355X whose backend sleeps the per-call latency measured for amdsmi on MI355X
(profiles/archive/amdsmi_cost_r2.json: Fast 141 us, Slow 960 us, Ras 1836 us p50 per device).
Devices are sampled concurrently (one task per GPU), so a poll should cost about one
device's latency at every N, not N of them.  Writes a JSON summary.

UNVERIFIED ON HARDWARE: this model assumes amdsmi calls on different devices run
concurrently (one call at a time per handle, none across handles).  Every lease so far had
one GPU, so no multi-GPU poll has been timed.  On MI355X the metrics call is also mostly the
kernel's synchronous SMU exchange, on-CPU in the polling thread
(profiles/r6_telemetry/: ~0.65 ms in round 6), so eight devices may also need eight CPUs'
worth of short busy-waits at once, or contend inside the driver."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bacchus_gpu_controller_amd import native  # noqa: E402

COST_US = {"fast": 141, "slow": 960, "ras": 1836}


def measure(nat, n, level, polls=40):
    f = json.loads(nat.default_mi355x_fixture(n))
    for g in f["gpus"]:
        g["telemetry"]["sample_delay_us"] = COST_US[level]
    b = nat.gpu_backend("mock", json.dumps(f))
    slow_every, ras_every = {"fast": (10**6, 10**6), "slow": (1, 10**6), "ras": (1, 1)}[level]
    p = nat.TelemetryPoller(b, list(range(n)), 1000, "{}", slow_every, ras_every)
    p.poll_once()  # poll 0 is always a Ras poll; measure the cadence of interest after it
    us = []
    for _ in range(polls):
        p.poll_once()
        us.append(json.loads(p.snapshot())["poll_us"])
    us.sort()
    return {"p50_us": round(statistics.median(us), 1), "p99_us": round(us[int(0.99 * (len(us) - 1))], 1),
            "per_device_us": COST_US[level]}


def main(out):
    nat = native()
    res = {lvl: {str(n): measure(nat, n, lvl) for n in (1, 2, 4, 8)} for lvl in COST_US}
    res["note"] = ("mock backend sleeping amdsmi's measured per-call latency; poll_us = wall time of one poll "
                   "over all N devices (concurrent per-device sampling)")
    print(json.dumps(res, indent=1))
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/archive/telemetry_scaling_r2.json")

#!/usr/bin/env python3
"""Per-call cost of the amdsmi queries the telemetry poller issues (GPU box)."""
import json
import time

import amdsmi


def timed(fn, *a, n=50):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        try:
            fn(*a)
        except Exception as e:  # noqa: BLE001
            return {"error": str(e)}
        ts.append((time.perf_counter() - t0) * 1e6)
    ts.sort()
    return {"p50_us": ts[len(ts) // 2], "min_us": ts[0]}


amdsmi.amdsmi_init()
h = amdsmi.amdsmi_get_processor_handles()[0]
out = {
    "gpu_metrics_info": timed(amdsmi.amdsmi_get_gpu_metrics_info, h),
    "vram_usage": timed(amdsmi.amdsmi_get_gpu_vram_usage, h),
    "total_ecc_count": timed(amdsmi.amdsmi_get_gpu_total_ecc_count, h),
    "gpu_activity": timed(amdsmi.amdsmi_get_gpu_activity, h),
    "power_info": timed(amdsmi.amdsmi_get_power_info, h),
    "temp_hotspot": timed(amdsmi.amdsmi_get_temp_metric, h, amdsmi.AmdSmiTemperatureType.HOTSPOT,
                          amdsmi.AmdSmiTemperatureMetric.CURRENT),
    "n_devices": len(amdsmi.amdsmi_get_processor_handles()),
}
amdsmi.amdsmi_shut_down()
print(json.dumps(out, indent=1))

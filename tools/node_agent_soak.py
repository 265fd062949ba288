"""Node-agent soak on a real MI355X: periodic diagnostics passes back to back with the
telemetry poller and the kubelet device plugin running, to show that repeated passes do
not leak (agent RSS, VRAM in use after each pass) and that their verdicts and rates are
stable.

    python3 tools/node_agent_soak.py OUT.json [minutes=8] [interval_s=20] [tenant_from_min tenant_to_min]

With a tenant window, a "tenant" process (torch: 16 GiB resident and a matmul loop)
holds the GPU in that window: passes then must skip the GPU as in use, and resume once
the tenant exits.  Prints one progress line per sample (every 10 s).
"""
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import requests  # noqa: E402

from bacchus_gpu_controller_amd.testing.cluster import Cluster  # noqa: E402
from bacchus_gpu_controller_amd.testing.kubelet import FakeKubelet  # noqa: E402


def rss_mb(pid):
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024.0
    return None


TENANT = """
import time, torch
x = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
print("tenant up", flush=True)
while True:
    for _ in range(50):
        a = (a @ a).clamp_(-1, 1)
    torch.cuda.synchronize()
    time.sleep(0.05)
"""


def main():
    out_path = sys.argv[1]
    minutes = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
    interval = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    window = (float(sys.argv[4]) * 60, float(sys.argv[5]) * 60) if len(sys.argv) > 5 else None
    tenant = None
    d = "/tmp/bgc-soak-dp"
    os.makedirs(d, exist_ok=True)
    kubelet = FakeKubelet(d).start()
    samples, passes = [], []
    try:
        with Cluster(admission=False, controller=False) as c:
            c.start_node_agent(node_name="mi355x-soak", backend="amdsmi", max_gpus=1, poll_interval_ms=1000,
                               extra_env={"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d,
                                          "CONF_RUN_DIAG": "true", "CONF_DIAG_BURN_MS": "2000",
                                          "CONF_DIAG_INTERVAL_SECS": str(interval),
                                          "CONF_DIAG_FENCE_SETTLE_MS": "500"})
            url = f"http://127.0.0.1:{c.node_agent_ports['mi355x-soak']}/gpus"
            pid = c.procs["node-agent"].p.pid
            t0 = time.time()
            seen_runs = 0
            while time.time() - t0 < minutes * 60:
                time.sleep(10)
                now = time.time() - t0
                if window and tenant is None and window[0] <= now < window[1]:
                    tenant = subprocess.Popen([sys.executable, "-c", TENANT], stdout=subprocess.DEVNULL)
                if window and tenant is not None and now >= window[1] and tenant.poll() is None:
                    tenant.kill()
                    tenant.wait(30)
                g = requests.get(url, timeout=10).json()
                tele = (g.get("telemetry") or [{}])[0] if isinstance(g.get("telemetry"), list) else {}
                runs = g.get("diag_runs", 0)
                s = {"t_s": round(time.time() - t0, 1), "rss_mb": rss_mb(pid), "diag_runs": runs,
                     "tenant": tenant is not None and tenant.poll() is None,
                     "skipped_in_use": g.get("diag_skipped_in_use"),
                     "vram_used_mb": tele.get("vram_used_mb"), "healthy": g.get("healthy"),
                     "last_pass_ms": g.get("diag_last_pass_ms")}
                samples.append(s)
                if runs != seen_runs:
                    seen_runs = runs
                    r = (g.get("diag") or [{}])[0]
                    passes.append({"run": runs, "t_s": s["t_s"], "tenant": s["tenant"],
                                   "skipped_in_use": g.get("diag_skipped_in_use"),
                                   "passed": r.get("passed"), "failures": r.get("failures"),
                                   "pass_ms": g.get("diag_last_pass_ms"),
                                   "soak_tflops": (r.get("soak") or {}).get("tflops_mean"),
                                   "burn_tflops": (r.get("burn") or {}).get("tflops_mean"),
                                   "walk_gb": (r.get("hbm_walk") or {}).get("bytes_covered", 0) / 1e9,
                                   "hbm_read_gbps": (r.get("hbm") or {}).get("read_gbps")})
                print(json.dumps(s), flush=True)
            out = {"minutes": minutes, "interval_s": interval, "samples": samples, "passes": passes,
                   "fence_races": g.get("diag_fence_races"), "agent_alive": c.procs["node-agent"].alive()}
    finally:
        if tenant is not None and tenant.poll() is None:
            tenant.kill()
        kubelet.stop()
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    ok = out["agent_alive"] and passes and all(p["passed"] for p in passes)
    print(json.dumps({"passes": len(passes), "all_passed": bool(ok),
                      "rss_first_last_mb": [samples[0]["rss_mb"], samples[-1]["rss_mb"]]}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())

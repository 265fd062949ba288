#!/usr/bin/env python3
"""rocprofv3 --marker-trace of the node agent's telemetry poll on the final tree
(VERDICT r5 #4), quiet or during a default bench run.

The node agent runs under rocprofv3 with the agent right after "--" (testing/cluster.py
BGC_WRAP_NODE_AGENT); its roctx ranges are the poll by cadence
(bgc.telemetry.poll.{fast,slow,ras}) and each amdsmi call inside it (bgc.amdsmi.*, the
per-handle lock wait included; native/gpu/device.cc).  The agent's own sample logs add the
poll's split into on-CPU time, run-queue wait and blocked time (core/schedstat.h).

  quiet:  kube-lite + the node agent alone, 1 GPU, polling every 250 ms (the bench's
          cadence) for --seconds
  bench:  bench.py with its node agent wrapped the same way (arguments after "--" go to
          bench.py)

Writes <out>/<mode>/summary.json: per roctx range n, mean, p50, p99, max (us), and the
poll split percentiles.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def _pct(v, q):
    if not v:
        return None
    v = sorted(v)
    return v[max(0, min(len(v) - 1, int(round(q * len(v) + 0.5)) - 1))]


def summarize_markers(trace_dir):
    """Per range name: n, mean/p50/p99/max in us, from rocprofv3's marker_api_trace.csv."""
    files = glob.glob(os.path.join(trace_dir, "**", "*marker_api_trace.csv"), recursive=True)
    durs = {}
    for path in files:
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Function") or row.get("Name") or row.get("Message") or ""
                try:
                    d = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
                except (KeyError, ValueError):
                    continue
                if name.startswith("bgc."):
                    durs.setdefault(name, []).append(d)
    stats = {}
    for path in glob.glob(os.path.join(trace_dir, "**", "*marker_api_stats.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Name", "").startswith("bgc."):
                    stats[row["Name"]] = {"calls": int(row["Calls"]), "mean_us": round(float(row["AverageNs"]) / 1e3, 1),
                                          "min_us": round(float(row["MinNs"]) / 1e3, 1),
                                          "max_us": round(float(row["MaxNs"]) / 1e3, 1)}
    return {"files": [os.path.relpath(p, trace_dir) for p in files], "stats": stats,
            "ranges": {k: {"n": len(v), "mean_us": round(sum(v) / len(v), 1), "p50_us": round(_pct(v, 0.5), 1),
                           "p99_us": round(_pct(v, 0.99), 1), "max_us": round(max(v), 1)}
                       for k, v in sorted(durs.items())}}


def _split(url):
    import requests

    out = {}
    for name in ("telemetry_poll", "telemetry_poll_cpu", "telemetry_poll_runq"):
        r = requests.get(f"{url}/debug/samples/{name}", timeout=10)
        if r.status_code != 200:
            continue
        v = [x * 1e3 for x in r.json()["samples"]]
        out[name] = {"n": len(v), "p50_ms": round(_pct(v, 0.5), 4), "p99_ms": round(_pct(v, 0.99), 4),
                     "mean_ms": round(sum(v) / len(v), 4) if v else None}
    return out


def _thread_times(pid, name):
    """(utime, stime) seconds of the thread called `name` in process `pid` (user vs kernel
    CPU: the amdsmi metrics call's kernel part is the driver's synchronous SMU exchange)."""
    tck = os.sysconf("SC_CLK_TCK")
    for tid in os.listdir(f"/proc/{pid}/task"):
        try:
            raw = open(f"/proc/{pid}/task/{tid}/stat").read()
        except OSError:
            continue
        if raw[raw.index("(") + 1:raw.rindex(")")] == name:
            f = raw.rsplit(")", 1)[1].split()
            return int(f[11]) / tck, int(f[12]) / tck
    return None


def quiet(out_dir, seconds, poll_ms):
    from bacchus_gpu_controller_amd.testing.cluster import Cluster

    with Cluster(admission=False, controller=False) as c:
        p = c.start_node_agent(max_gpus=1, poll_interval_ms=poll_ms, extra_env={"CONF_RUN_DIAG": "false"})
        url = f"http://127.0.0.1:{c.node_agent_port}"
        t0 = _thread_times(p.p.pid, "telemetry")
        time.sleep(seconds)
        t1 = _thread_times(p.p.pid, "telemetry")
        split = _split(url)
        if t0 and t1:
            split["telemetry_thread_cpu_s"] = {"user": round(t1[0] - t0[0], 3), "kernel": round(t1[1] - t0[1], 3)}
        gpus = __import__("requests").get(url + "/gpus", timeout=10).json()
        c.procs["node-agent"].stop(timeout=30)  # SIGTERM: rocprofv3 writes its trace at exit
    return {"mode": "quiet", "seconds": seconds, "poll_ms": poll_ms, "backend": gpus.get("backend"),
            "split": split}


def bench(out_dir, bench_args):
    path = os.path.join(out_dir, "bench.json")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--json-out", path] + bench_args
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
    d = json.load(open(path))
    return {"mode": "bench", "value": d["value"], "telemetry_poll_p50_ms": d.get("telemetry_poll_p50_ms"),
            "telemetry_poll_split_p50_ms": d.get("telemetry_poll_split_p50_ms"),
            "gpu_telemetry": d.get("gpu_telemetry")}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("mode", choices=("quiet", "bench"))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "telemetry_marker"))
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--poll-ms", type=int, default=250)
    a, rest = ap.parse_known_args()  # bench mode: everything after "--" goes to bench.py
    a.rest = [x for x in rest if x != "--"]
    out_dir = os.path.abspath(os.path.join(a.out, a.mode))
    os.makedirs(out_dir, exist_ok=True)
    os.environ["BGC_WRAP_NODE_AGENT"] = (f"rocprofv3 --marker-trace --stats --output-format csv -d {out_dir}/trace "
                                         "-o agent --")
    res = quiet(out_dir, a.seconds, a.poll_ms) if a.mode == "quiet" else bench(out_dir, a.rest)
    res["markers"] = summarize_markers(os.path.join(out_dir, "trace"))
    with open(os.path.join(out_dir, "summary.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

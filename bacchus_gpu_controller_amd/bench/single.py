"""BASELINE configs #1 and #2 as timed runs: one tenant at a time, no concurrency, so the
numbers are the latency of the plumbing itself.

    python -m bacchus_gpu_controller_amd.bench.single [--tenants 50] [--real-gpu] [--json-out f]

config #1 (default, 0 GPUs, CPU only):
  * `crdgen` run 20 times: wall time per run, and its output byte-compared with the
    chart's templates/crd.yaml (generate-crd.sh's check);
  * kube-lite + TLS admission + controller + synchronizer (watch mode), no node agent;
    `--tenants` UserBootstraps onboarded one after another as OIDC users
    (create -> webhook -> Namespace -> sheet sync -> ResourceQuota -> RoleBinding), each
    deleted before the next, with the time to every stage from the API server's view.
config #2 (`--real-gpu`, one MI355X): the node agent discovers the GPU through amdsmi
  (with its start-up diagnostics off, so this times discovery and advertisement), the
  Node must carry amd.com/gpu=1, and every tenant's ResourceQuota requests.amd.com/gpu=1.

The reference does the same steps with its 60 s sheet tick in the middle
(src/synchronizer.rs:192): its create -> RoleBinding is U(0, 60 s) + processing.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

import requests

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from bacchus_gpu_controller_amd import binary  # noqa: E402
from bacchus_gpu_controller_amd.testing.cluster import Cluster  # noqa: E402
from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle  # noqa: E402
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for  # noqa: E402


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def crdgen_check(runs=20):
    ref = open(os.path.join(ROOT, "charts", "bacchus-gpu-controller", "templates", "crd.yaml"), "rb").read()
    times, same = [], True
    for _ in range(runs):
        t0 = time.perf_counter()
        out = subprocess.run([binary("crdgen")], capture_output=True, check=True).stdout
        times.append((time.perf_counter() - t0) * 1e3)
        same = same and out == ref
    return {"runs": runs, "wall_ms_p50": round(statistics.median(times), 3), "byte_identical": same}


def run(tenants=50, real_gpu=False):
    out = {"config": 2 if real_gpu else 1, "crdgen": crdgen_check()}
    names = [f"s-{i:03d}" for i in range(tenants)]
    google = FakeGoogle().start()
    google.set_rows([{"id_username": n, "gpu": 1} for n in names])
    stages = {"namespace": [], "quota": [], "rolebinding": []}
    try:
        with Cluster(tls_apiserver=True) as c:  # components reach the API server over HTTPS
            c.start_synchronizer(google, interval=60, extra_env={"CONF_WATCH": "true"})
            if real_gpu:  # config #1 has no GPU, so no node agent (it refuses to run without one)
                t0 = time.perf_counter()
                c.start_node_agent(max_gpus=1, backend="amdsmi", poll_interval_ms=1000)
                node = wait_for(lambda: (lambda n: n if n and n["status"].get("capacity", {}).get("amd.com/gpu") == "1"
                                         else None)(c.admin.get_or_none("nodes", "mi355x-0")),
                                timeout=60, interval=0.01, desc="amd.com/gpu advertised")
                out["node_agent_start_to_advertised_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
                out["node"] = {"capacity": node["status"].get("capacity", {}),
                               "labels": {k: v for k, v in node["metadata"]["labels"].items()
                                          if k.startswith("amd.com/")}}
            # the native churn driver (native/bench/churn.cc) at concurrency 1: it creates each
            # tenant as an OIDC user and timestamps every child from its own watches
            from bacchus_gpu_controller_amd import native
            from bacchus_gpu_controller_amd.testing.cluster import ADMIN_TOKEN

            driver = native().ChurnDriver(c.server, ADMIN_TOKEN, "s-", 1, ca_pem=open(c.apiserver_ca).read())
            driver.start()
            time.sleep(0.2)
            try:
                prev = []
                for n in names:
                    res = json.loads(driver.step_with_delete([n], prev, 30.0))
                    if res["ready"] != 1:
                        raise RuntimeError(f"{n} not Ready: {res}")
                    for k, key in (("namespace", "ns"), ("quota", "rq"), ("rolebinding", "rb")):
                        stages[k] += [x * 1e3 for x in res[f"{key}_latency_s"]]
                    prev = [n]
                rq = c.admin.get("resourcequotas", names[-1], names[-1])
                if rq["spec"]["hard"].get("requests.amd.com/gpu") != "1":
                    raise RuntimeError(f"quota {rq['spec']}")
                driver.remove(prev)
            finally:
                driver.stop()
            rec = c.samples("controller", "reconcile")["samples"]
            adm = requests.get(f"https://127.0.0.1:{c.admission_port}/debug/samples/admission", timeout=5,
                               verify=os.path.join(c.cert_dir, "ca.crt")).json()["samples"]
    finally:
        google.stop()
    out["tenants"] = tenants
    out["apply_to_stage_ms"] = {k: {"p50": round(_pct(v, 0.5), 3), "p99": round(_pct(v, 0.99), 3)}
                                for k, v in stages.items()}
    out["reconcile_ms"] = {"p50": round(_pct(rec, 0.5) * 1e3, 4), "p99": round(_pct(rec, 0.99) * 1e3, 4)} if rec else None
    out["admission_handler_ms"] = {"p50": round(_pct(adm, 0.5) * 1e3, 4)} if adm else None
    out["reference_structural"] = {"create_to_rolebinding": "U(0, 60 s) + processing (synchronizer.rs:192)"}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--tenants", type=int, default=50)
    ap.add_argument("--real-gpu", action="store_true", help="config #2: the node agent on the host's MI355X")
    ap.add_argument("--json-out")
    args = ap.parse_args(argv)
    out = run(args.tenants, args.real_gpu)
    line = json.dumps(out)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")
    return 0 if out["crdgen"]["byte_identical"] else 1


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Steady-state cost of the periodic resync (reference: every UserBootstrap re-applies its
children every 30 s, controller.rs:154).

A population of onboarded tenants is left alone, and the API-server request rate and the
controller CPU are measured over a window, first with the reference behaviour (every requeue
re-applies; CONF_SKIP_UNCHANGED=false) and then with this build's default (children already
as last written are skipped). The requeue period is compressed to make the window short.

    python3 tools/steady_state.py --tenants 2000 --requeue-secs 2 --window 10 > profiles/archive/steady_state_r1.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bacchus_gpu_controller_amd.bench.harness import _cpu_seconds  # noqa: E402
from bacchus_gpu_controller_amd.testing.cluster import Cluster  # noqa: E402
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for  # noqa: E402


def measure(tenants, requeue_secs, window, skip):
    env = {"CONF_REQUEUE_SECS": str(requeue_secs), "CONF_SKIP_UNCHANGED": "true" if skip else "false",
           "CONF_WORKERS": "32"}
    with Cluster(admission=False, controller_env=env, tls_apiserver=True) as c:
        for i in range(tenants):
            n = f"t{i:05d}"
            c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                              "metadata": {"name": n},
                                              "spec": {"kube_username": n,
                                                       "quota": {"hard": {"requests.amd.com/gpu": "1"}},
                                                       "rolebinding": {"role_ref": {"apiGroup": "rbac.authorization.k8s.io",
                                                                                    "kind": "ClusterRole", "name": "edit"},
                                                                       "subjects": [{"kind": "User", "name": n,
                                                                                     "apiGroup": "rbac.authorization.k8s.io"}]}}})
            c.admin.replace("userbootstraps", n, {**c.admin.get("userbootstraps", n),
                                                  "status": {"synchronized_with_sheet": True}}, sub="status")
        last = f"t{tenants - 1:05d}"
        wait_for(lambda: c.admin.get_or_none("rolebindings", last, last), timeout=120, desc="population ready")
        time.sleep(requeue_secs + 1)  # let the onboarding burst drain
        s0, cpu0 = c.stats(), _cpu_seconds(c.procs["controller"].p.pid)
        time.sleep(window)
        s1, cpu1 = c.stats(), _cpu_seconds(c.procs["controller"].p.pid)
        req = {k: v - s0["requests_by_kind"].get(k, 0) for k, v in s1["requests_by_kind"].items()
               if v - s0["requests_by_kind"].get(k, 0) > 0}
        return {"skip_unchanged": skip, "tenants": tenants, "requeue_secs": requeue_secs, "window_s": window,
                "api_requests_per_s": round((s1["requests"] - s0["requests"]) / window, 1),
                "controller_cpu_cores": round((cpu1 - cpu0) / window, 3),
                "requests_by_kind_per_s": {k: round(v / window, 1) for k, v in sorted(req.items())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tenants", type=int, default=2000)
    ap.add_argument("--requeue-secs", type=int, default=2)
    ap.add_argument("--window", type=float, default=10.0)
    a = ap.parse_args()
    ref = measure(a.tenants, a.requeue_secs, a.window, skip=False)
    ours = measure(a.tenants, a.requeue_secs, a.window, skip=True)
    print(json.dumps({"reference_behaviour": ref, "this_build": ours,
                      "note": "requeue period compressed from 30 s; scale rates by requeue_secs/30 for production"},
                     indent=1))


if __name__ == "__main__":
    main()

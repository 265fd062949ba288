#!/usr/bin/env python3
"""Controller cost of cluster churn that is not its own (a real cluster's other tenants,
CI namespaces, operators' RoleBindings...).  The reference's .owns() watches every
Namespace/ResourceQuota/Role/RoleBinding in the cluster (controller.rs:235-238), so each
unrelated write reaches the controller: event parse, cache update, owner mapping.  This
build labels its children and selects on the label (CONF_LABEL_CHILDREN).

A few tenants are onboarded, then unrelated Namespaces and RoleBindings are created and
deleted at a steady rate for a window; controller CPU and watch-cache sizes are measured
with the label selector on and off.

    python3 tools/unrelated_churn.py --rate 400 --window 10 > profiles/archive/unrelated_churn_r2.json
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import requests  # noqa: E402

from bacchus_gpu_controller_amd.bench.harness import _cpu_seconds  # noqa: E402
from bacchus_gpu_controller_amd.testing.cluster import Cluster  # noqa: E402
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for  # noqa: E402


def gauges(c):
    txt = requests.get(f"http://127.0.0.1:{c.controller_port}/metrics", timeout=5).text
    return {l.split("{")[1].split("}")[0].split('"')[1]: float(l.split()[-1]) for l in txt.splitlines()
            if l.startswith("bgc_controller_store_objects{")}


def measure(labelled, rate, window, tenants):
    env = {"CONF_REQUEUE_SECS": "3600", "CONF_LABEL_CHILDREN": "true" if labelled else "false"}
    with Cluster(admission=False, controller_env=env, tls_apiserver=True, log_level="info") as c:
        for i in range(tenants):
            c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                              "metadata": {"name": f"t{i}"}, "spec": {"kube_username": f"t{i}"}})
        wait_for(lambda: c.admin.get_or_none("namespaces", f"t{tenants - 1}"), timeout=60, desc="tenants")
        stop = threading.Event()
        done = [0]

        def churn(k):
            i = 0
            while not stop.is_set():
                ns = f"other-{k}-{i}"
                c.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
                c.admin.create("rolebindings", {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                                                "metadata": {"name": "ci", "namespace": ns},
                                                "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                                                            "name": "view"},
                                                "subjects": [{"kind": "User", "name": "ci-bot",
                                                              "apiGroup": "rbac.authorization.k8s.io"}]}, namespace=ns)
                if i >= 50:
                    c.admin.delete("namespaces", f"other-{k}-{i - 50}")
                done[0] += 1
                i += 1
                time.sleep(4.0 / rate)

        threads = [threading.Thread(target=churn, args=(k,), daemon=True) for k in range(4)]
        for t in threads:
            t.start()
        time.sleep(2.0)
        cpu0, n0 = _cpu_seconds(c.procs["controller"].p.pid), done[0]
        time.sleep(window)
        cpu1, n1 = _cpu_seconds(c.procs["controller"].p.pid), done[0]
        g = gauges(c)
        stop.set()
        for t in threads:
            t.join(10)
        return {"label_children": labelled, "unrelated_writes_per_s": round(3 * (n1 - n0) / window, 1),
                "controller_cpu_cores": round((cpu1 - cpu0) / window, 4), "watch_cache_objects": g}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", type=float, default=400, help="unrelated namespace+rolebinding creations per second")
    ap.add_argument("--window", type=float, default=10.0)
    ap.add_argument("--tenants", type=int, default=20)
    a = ap.parse_args()
    ref = measure(False, a.rate, a.window, a.tenants)
    ours = measure(True, a.rate, a.window, a.tenants)
    print(json.dumps({"watch_everything (reference .owns())": ref, "label_selected (this build)": ours}, indent=1))


if __name__ == "__main__":
    main()

"""BASELINE config #4 as a timed benchmark: xGMI-hive node labels + RCCL-aware TP=8 pod
co-scheduling.

    python -m bacchus_gpu_controller_amd.bench.tp8 [--nodes 4] [--iters 300] [--real-gpu]

Cluster: kube-lite + one native node agent per synthetic 8x MI355X node (mock amdsmi, one
xGMI hive each; node 1 is wired as two 4-GPU xGMI quads joined only by PCIe, to exercise
the link map) with the kubelet device plugin on, each registered with its own fake kubelet
(grpcio, an independent gRPC stack); with --real-gpu one more agent on this host's GPUs via
amdsmi.  Measured from the kubelet's and the scheduler's side:

  publish_ms          agent start -> Node carries amd.com/gpu.xgmi-hive-id + topology
  plan_ms             plan_tp_groups() over the live Node objects (TP=8 per hive)
  preferred_8_us      kubelet GetPreferredAllocation(size 8 of 8) round trip
  allocate_8_us       kubelet Allocate(8 devices) round trip
  churn               random pod sizes (1/2/4/8) allocated and released through
                      GetPreferredAllocation + Allocate on every node: share of
                      allocations that stay inside one xGMI hive, and (two-quad node)
                      share of 2..4-GPU allocations whose GPUs are all directly xGMI-linked
                      whenever the free set held such a group

The reference has no scheduling side at all (GPUs are only quota keys,
src/synchronizer.rs:268); these are the north star's node-side numbers for config #4.
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from bacchus_gpu_controller_amd import native  # noqa: E402
from bacchus_gpu_controller_amd.parallel.placement import hive_inventory, plan_tp_groups  # noqa: E402
from bacchus_gpu_controller_amd.testing.cluster import Cluster  # noqa: E402
from bacchus_gpu_controller_amd.testing.kubelet import FakeKubelet, PluginClient, pb  # noqa: E402


def _pct(v, q):
    if not v:
        return None
    s = sorted(v)
    return round(s[min(len(s) - 1, int(q * len(s)))], 2)


def _until(pred, timeout, step=0.005):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < timeout:
        r = pred()
        if r:
            return (time.perf_counter() - t0) * 1e3, r
        time.sleep(step)
    raise TimeoutError(f"not converged within {timeout}s")


def two_quad_fixture(nat, hive_id):
    """8 GPUs, one hive, but xGMI only inside {0,2,4,6} and {1,3,5,7} (PCIe between)."""
    f = json.loads(nat.default_mi355x_fixture(8, hive_id))
    quad = lambda i: i % 2  # noqa: E731
    for g in f["gpus"]:
        for link in g["links"]:
            if quad(g["index"]) != quad(link["peer"]):
                link.update({"type": "pcie", "hops": 2, "weight": 40, "min_bw_mbps": 0, "max_bw_mbps": 0})
    return f


def run(args):
    nat = native()
    rng = random.Random(7)
    res = {"metric": "config #4: xGMI-hive labels + TP=8 co-scheduling (kubelet device-plugin RPCs, placement)",
           "nodes": args.nodes + (1 if args.real_gpu else 0), "iters": args.iters}
    kubelets = {}
    publish = []
    with Cluster(admission=False, controller=False, log_level=args.log_level) as c:
        for i in range(args.nodes):
            name = f"mi355x-{i}"
            d = os.path.join(c.workdir, f"dp-{name}")
            kubelets[name] = FakeKubelet(d).start()
            extra = {"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d}
            t0 = time.perf_counter()
            # node 1: two xGMI quads (exercises the link-aware preferred allocation)
            c.start_node_agent(node_name=name, backend="mock", hive_id=0x355000 + i, proc_name=f"na-{name}",
                               extra_env=extra, fixture_obj=two_quad_fixture(nat, 0x355001) if i == 1 else None)
            _until(lambda: (lambda n: n and n["metadata"].get("annotations", {}).get("amd.com/gpu.topology")
                                    and n["metadata"]["labels"].get("amd.com/gpu.xgmi-hive-id"))(
                c.admin.get_or_none("nodes", name)), 30)
            publish.append((time.perf_counter() - t0) * 1e3)
        if args.real_gpu:
            d = os.path.join(c.workdir, "dp-real")
            kubelets["mi355x-real"] = FakeKubelet(d).start()
            t0 = time.perf_counter()
            c.start_node_agent(node_name="mi355x-real", backend="amdsmi", proc_name="na-real",
                               extra_env={"CONF_DEVICE_PLUGIN": "true", "CONF_DEVICE_PLUGIN_DIR": d})
            _until(lambda: (lambda n: n and n["metadata"]["labels"].get("amd.com/gpu.xgmi-hive-id"))(
                c.admin.get_or_none("nodes", "mi355x-real")), 60)
            publish.append((time.perf_counter() - t0) * 1e3)
        res["publish_ms"] = {"p50": _pct(publish, 0.5), "max": round(max(publish), 1)}

        # -- placement over the live Node objects
        nodes = c.admin.list("nodes")["items"]
        plan_ms = []
        for _ in range(50):
            t0 = time.perf_counter()
            plan = plan_tp_groups(nodes, 8, args.nodes)
            plan_ms.append((time.perf_counter() - t0) * 1e3)
        inv = hive_inventory(nodes)
        res["plan_ms"] = {"p50": _pct(plan_ms, 0.5), "p99": _pct(plan_ms, 0.99)}
        res["plan_tp8_groups"] = len(plan)
        res["plan_groups_on_distinct_hives"] = len({p["hive"] for p in plan}) == len(plan)
        res["hives"] = len(inv)

        # -- kubelet-side device-plugin RPCs
        for k in kubelets.values():
            assert k.wait(lambda: k.registrations and k.device_lists, timeout=30)
        pref_us, alloc_us = [], []
        churn = {"allocations": 0, "single_hive": 0, "quad_checked": 0, "quad_direct": 0}
        quad_of = lambda bdf_idx: bdf_idx % 2  # noqa: E731
        for name, k in kubelets.items():
            sock = os.path.join(k.dir, k.registrations[-1].endpoint)
            ids = [x[0] for x in k.device_lists[-1][1]]
            cl = PluginClient(sock)
            try:
                if len(ids) == 8:
                    for _ in range(args.iters):
                        q = pb["PreferredAllocationRequest"]()
                        cq = q.container_requests.add()
                        cq.available_deviceIDs.extend(ids)
                        cq.allocation_size = 8
                        t0 = time.perf_counter()
                        cl.preferred(q, timeout=10)
                        pref_us.append((time.perf_counter() - t0) * 1e6)
                        a = pb["AllocateRequest"]()
                        a.container_requests.add().devices_ids.extend(ids)
                        t0 = time.perf_counter()
                        cl.allocate(a, timeout=10)
                        alloc_us.append((time.perf_counter() - t0) * 1e6)
                # churn: pods of random size come and go on this node
                free, held = list(ids), []
                for _ in range(args.iters):
                    if held and (rng.random() < 0.5 or not free):
                        free += held.pop(rng.randrange(len(held)))
                        continue
                    size = rng.choice([s for s in (1, 2, 4, 8) if s <= len(free)] or [0])
                    if size == 0:
                        continue
                    q = pb["PreferredAllocationRequest"]()
                    cq = q.container_requests.add()
                    cq.available_deviceIDs.extend(free)
                    cq.allocation_size = size
                    pick = list(cl.preferred(q, timeout=10).container_responses[0].deviceIDs)
                    a = pb["AllocateRequest"]()
                    a.container_requests.add().devices_ids.extend(pick)
                    resp = cl.allocate(a, timeout=10).container_responses[0]
                    churn["allocations"] += 1
                    churn["single_hive"] += resp.envs["BGC_AMD_GPU_SINGLE_XGMI_HIVE"] == "true"
                    free_quads = [sum(1 for x in free if quad_of(ids.index(x)) == qd) for qd in (0, 1)]
                    if name == "mi355x-1" and 2 <= size <= 4 and max(free_quads) >= size:
                        # a directly xGMI-linked set was available: did the plugin pick one?
                        churn["quad_checked"] += 1
                        churn["quad_direct"] += len({quad_of(ids.index(x)) for x in pick}) == 1
                    for x in pick:
                        free.remove(x)
                    held.append(pick)
            finally:
                cl.close()
        res["preferred_8_us"] = {"p50": _pct(pref_us, 0.5), "p99": _pct(pref_us, 0.99)}
        res["allocate_8_us"] = {"p50": _pct(alloc_us, 0.5), "p99": _pct(alloc_us, 0.99)}
        res["churn"] = churn
        res["churn_single_hive_share"] = round(churn["single_hive"] / max(1, churn["allocations"]), 4)
        res["two_quad_direct_xgmi_share"] = round(churn["quad_direct"] / max(1, churn["quad_checked"]), 4)
        res["processes_alive"] = {n: p.alive() for n, p in c.procs.items()}
    for k in kubelets.values():
        k.stop()
    return res


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nodes", type=int, default=4)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--real-gpu", action="store_true")
    ap.add_argument("--log-level", default="info")
    ap.add_argument("--json-out", default="")
    args = ap.parse_args(argv)
    res = run(args)
    line = json.dumps(res)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")
    print(line, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""xGMI-island-aware placement helpers for RCCL TP/DP/PP jobs (BASELINE config #4).

The node agent labels every MI355X node with its xGMI hive id, healthy GPU count and a
per-GPU topology annotation (native/gpu/node_agent.h).  These helpers turn those labels
into scheduling decisions and pod-spec fragments:

* ``hive_inventory(nodes)``        -> {hive_id: {"nodes": [...], "healthy": n}}
* ``plan_tp_groups(nodes, tp, n)`` -> place n tensor-parallel groups of size tp so that
                                      every group sits inside ONE xGMI island (TP all-reduce
                                      traffic stays on point-to-point xGMI links), DP/PP
                                      across islands is allowed.
* ``tp_pod_affinity(hive, gpus)``  -> nodeSelector/affinity/resources for a TP pod.

xGMI on MI355X is point-to-point (7 links per GPU), so a TP group must never straddle
hives; a group that would need more GPUs than one island has is rejected rather than
split.
"""
import json

LABEL_PREFIX = "amd.com/gpu"
RESOURCE = "amd.com/gpu"


def _labels(node):
    return node.get("metadata", {}).get("labels", {})


def node_schedulable(node):
    """False for cordoned nodes (``kubectl drain``/``cordon`` set spec.unschedulable)."""
    return not node.get("spec", {}).get("unschedulable", False)


def node_healthy_gpus(node):
    if not node_schedulable(node):
        return 0
    alloc = node.get("status", {}).get("allocatable", {}).get(RESOURCE)
    if alloc is not None:
        return int(alloc)
    return int(_labels(node).get(f"{LABEL_PREFIX}.healthy-count", "0"))


def node_hives(node):
    """Per-GPU hive ids from the topology annotation (falls back to the node label)."""
    ann = node.get("metadata", {}).get("annotations", {}).get(f"{LABEL_PREFIX}.topology")
    if ann:
        try:
            return [g["hive"] for g in json.loads(ann)]
        except (ValueError, KeyError, TypeError):
            pass
    hive = _labels(node).get(f"{LABEL_PREFIX}.xgmi-hive-id")
    count = int(_labels(node).get(f"{LABEL_PREFIX}.count", "0"))
    return [hive] * count if hive and hive != "mixed" else []


def hive_inventory(nodes):
    inv = {}
    for n in nodes:
        name = n["metadata"]["name"]
        hives = node_hives(n)
        healthy = node_healthy_gpus(n)
        if not hives:
            continue
        # attribute healthy GPUs proportionally when a node spans several hives
        per_hive = {}
        for h in hives:
            per_hive[h] = per_hive.get(h, 0) + 1
        total = len(hives)
        for h, cnt in per_hive.items():
            e = inv.setdefault(h, {"nodes": [], "healthy": 0, "gpus": 0})
            e["nodes"].append(name)
            e["gpus"] += cnt
            e["healthy"] += cnt if healthy >= total else min(cnt, healthy)
    return inv


def plan_tp_groups(nodes, tp, n_groups):
    """Greedy best-fit: each TP group goes to the island with the fewest free GPUs that
    still fits it (keeps large islands free for large groups). Returns a list of
    {"group": i, "hive": h, "node": node} or raises ValueError."""
    if tp < 1:
        raise ValueError("tp must be >= 1")
    free = {}
    node_of = {}
    for n in nodes:
        hives = node_hives(n)
        if not hives:
            continue
        healthy = node_healthy_gpus(n)
        for h in set(hives):
            key = (h, n["metadata"]["name"])
            free[key] = min(hives.count(h), healthy)
            node_of[key] = n["metadata"]["name"]
    plan = []
    for g in range(n_groups):
        fits = [(cnt, key) for key, cnt in free.items() if cnt >= tp]
        if not fits:
            raise ValueError(f"no xGMI island has {tp} free healthy GPUs for TP group {g} (free: {free})")
        cnt, key = min(fits)
        free[key] -= tp
        plan.append({"group": g, "hive": key[0], "node": node_of[key]})
    return plan


def tp_pod_affinity(hive_id, gpus):
    """Pod-spec fragment pinning a TP worker to one xGMI island."""
    return {
        "nodeSelector": {f"{LABEL_PREFIX}.xgmi-hive-id": hive_id, f"{LABEL_PREFIX}.product": "MI355X"},
        "resources": {"limits": {RESOURCE: str(gpus)}, "requests": {RESOURCE: str(gpus)}},
        "env": [{"name": "NCCL_IB_DISABLE", "value": "1"}, {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}],
    }

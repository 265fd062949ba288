"""RCCL-over-xGMI placement probe (north-star N5; BASELINE config #4).

Run one rank per GPU:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m bacchus_gpu_controller_amd.parallel.rccl_probe --sizes-mb 1,16,256,1024

Each rank:
  * reads its GPU's xGMI hive id through amdsmi (native backend) and all-gathers it, so a
    TP group that was NOT co-scheduled on one xGMI island is reported (and, with
    --require-single-hive, fails);
  * runs bf16 all-reduce over a size sweep with the `nccl` backend (= RCCL on ROCm),
    checks the result exactly, and reports algbw and busbw (busbw = algbw * 2(n-1)/n,
    the per-link figure comparable to the ~153 GB/s xGMI link rate);
  * reads its GPU's xGMI link write counters (amdsmi_get_link_metrics) before and after
    and compares the bytes that crossed xGMI with what the ring must have sent.

A TP=8 group on one hive should show busbw in the hundreds of GB/s; a group that fell
back to PCIe/NIC shows an order of magnitude less — the co-scheduling signal the node
agent's `amd.com/gpu.xgmi-hive-id` label is meant to protect.
"""
import argparse
import json
import os
import sys
import time


def busbw_factor(world):
    return 2.0 * (world - 1) / world if world > 1 else 1.0


def _bdf_key(bdf):
    """domain:bus:device of a PCI address, lower-case (torch reports no function number)."""
    b = (bdf or "").strip().lower()
    if b.count(":") == 1:  # "bb:dd.f" without a domain
        b = "0000:" + b
    return b.rsplit(".", 1)[0]


def device_bdf(local_device):
    """PCI address of a torch (HIP) device, e.g. "0000:05:00.0"."""
    import torch

    p = torch.cuda.get_device_properties(local_device)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"


def match_gpu(gpus, bdf=None, local_rank=0, allocated=None):
    """The amdsmi discovery entry of this rank's GPU.

    HIP renumbers the visible devices from 0 inside a container (HIP_VISIBLE_DEVICES or
    the device plugin's allocation), while amdsmi's ``hip_id`` is host-wide, so the match
    is by PCI address: ``bdf`` is this rank's device (``device_bdf``).  ``allocated`` is
    the device plugin's ``BGC_AMD_GPU_IDS`` (BDFs, or ``<bdf>-p<index>`` for compute
    partitions that share one); it narrows the candidates and tells partitions apart.
    ``hip_id == local_rank`` is the last resort, for hosts where neither is known."""
    cands = list(gpus)
    if allocated:
        keys = {_bdf_key(a.split("-p")[0]) for a in allocated}
        parts = {int(a.rsplit("-p", 1)[1]) for a in allocated if "-p" in a and a.rsplit("-p", 1)[1].isdigit()}
        narrowed = [g for g in cands if _bdf_key(g.get("bdf")) in keys and (not parts or g.get("index") in parts)]
        cands = narrowed or cands
    if bdf:
        same = [g for g in cands if _bdf_key(g.get("bdf")) == _bdf_key(bdf)]
        if len(same) == 1:
            return same[0]
        if len(same) > 1:  # partitions of one GPU: the hip ordinal among them
            cands = same
    for g in cands:
        if g.get("hip_id", g.get("index")) == local_rank:
            return g
    return cands[local_rank % len(cands)] if cands else None


def _allocated_ids():
    v = os.environ.get("BGC_AMD_GPU_IDS", "")
    return [x for x in v.split(",") if x] or None


def _rank_gpu(gpus, local_rank):
    try:
        bdf = device_bdf(local_rank)
    except Exception:  # noqa: BLE001 - no torch device (CPU rank)
        bdf = None
    return match_gpu(gpus, bdf, local_rank, _allocated_ids()), bdf


def local_hive_id(local_rank):
    try:
        from .. import native

        gpus = json.loads(native().gpu_backend("amdsmi", "").discover())
        g, _ = _rank_gpu(gpus, local_rank)
        return g["xgmi_hive_id"] if g else "unknown"
    except Exception as e:  # noqa: BLE001
        return f"unavailable:{type(e).__name__}"


def _amdsmi_index(backend, local_rank):
    gpus = json.loads(backend.discover())
    g, _ = _rank_gpu(gpus, local_rank)
    return g["index"] if g else local_rank % max(1, len(gpus))


def xgmi_write_kb(backend, index):
    """Cumulative KB this GPU has written over its xGMI links (amdsmi link metrics)."""
    t = json.loads(backend.sample(index, 2))
    return sum(l.get("write_kb", 0) for l in t.get("links", []) if l.get("type") == "xgmi")


def run(sizes_mb, iters=10, warmup=3, require_single_hive=False, dtype="bf16"):
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    if cuda:
        torch.cuda.set_device(local % torch.cuda.device_count())
    backend = "nccl" if cuda else "gloo"
    if world > 1 or not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29555")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        dist.init_process_group(backend=backend)
    out = sweep(sizes_mb, iters, warmup, dtype)
    dist.barrier()
    dist.destroy_process_group()
    if require_single_hive and not out["single_hive"]:
        raise SystemExit(f"TP group spans multiple xGMI hives: {out['hives']}")
    return out if rank == 0 else None


def sweep(sizes_mb, iters=10, warmup=3, dtype="bf16"):
    """The probe over an already initialised process group (every rank calls it; every
    rank gets the result). bench.py runs it after its timed region on N>1 GPUs."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    backend = dist.get_backend()
    cuda = backend == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    tdtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[dtype]

    def barrier():
        if cuda:
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()

    dev_index = torch.cuda.current_device() if cuda else local
    ident = {"hive": "cpu", "bdf": None, "amdsmi_bdf": None}
    if cuda:
        try:
            from .. import native

            g, bdf = _rank_gpu(json.loads(native().gpu_backend("amdsmi", "").discover()), dev_index)
            ident = {"hive": g["xgmi_hive_id"] if g else "unknown", "bdf": bdf, "amdsmi_bdf": g and g.get("bdf")}
        except Exception as e:  # noqa: BLE001
            ident["hive"] = f"unavailable:{type(e).__name__}"
    idents = [None] * world
    dist.all_gather_object(idents, ident)
    hives = [i["hive"] for i in idents]
    single_hive = len(set(hives)) == 1
    # xGMI traffic check: the link counters of this rank's GPU before and after the sweep.
    # A ring all-reduce writes 2(n-1)/n of the buffer per rank and iteration, so a group
    # that really runs over xGMI shows about that many bytes on its links.
    smi, smi_idx, kb0 = None, None, None
    if cuda:
        try:
            from .. import native

            smi = native().gpu_backend("amdsmi", "")
            smi_idx = _amdsmi_index(smi, dev_index)
            kb0 = xgmi_write_kb(smi, smi_idx)
        except Exception:  # noqa: BLE001
            smi = None
    expected_bytes = 0
    results = []
    for mb in sizes_mb:
        n = int(mb * (1 << 20) // torch.tensor([], dtype=tdtype).element_size())
        # small integers keep bf16 sums exact: every rank contributes (rank+1)
        buf = torch.full((n,), float(rank + 1), dtype=tdtype, device=dev)
        expect = float(world * (world + 1) // 2)
        for _ in range(warmup):
            buf.fill_(float(rank + 1))
            dist.all_reduce(buf)
        if cuda:
            torch.cuda.synchronize()
        times = []
        ok = True
        for _ in range(iters):
            buf.fill_(float(rank + 1))
            if cuda:
                torch.cuda.synchronize()
            barrier()
            t0 = time.perf_counter()
            dist.all_reduce(buf)
            if cuda:
                torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            ok = ok and bool(torch.all(buf == expect).item())
        t = sorted(times)[len(times) // 2]
        tmax = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        t = float(tmax.item())
        nbytes = n * buf.element_size()
        expected_bytes += busbw_factor(world) * nbytes * (warmup + iters) if world > 1 else 0
        algbw = nbytes / t / 1e9
        results.append({"size_mb": mb, "time_us": round(t * 1e6, 2), "algbw_gbps": round(algbw, 2),
                        "busbw_gbps": round(algbw * busbw_factor(world), 2), "correct": ok})
    wrote = None
    if smi is not None:
        try:
            wrote = (xgmi_write_kb(smi, smi_idx) - kb0) * 1024.0
        except Exception:  # noqa: BLE001
            wrote = None
    traffic = [None] * world
    dist.all_gather_object(traffic, {"xgmi_written_mb": None if wrote is None else round(wrote / 2**20, 1),
                                     "expected_mb": round(expected_bytes / 2**20, 1)})
    out = {"world_size": world, "backend": backend, "dtype": dtype, "hives": hives, "single_hive": single_hive,
           "devices": [{"bdf": i["bdf"], "amdsmi_bdf": i["amdsmi_bdf"]} for i in idents],
           "xgmi_traffic": traffic,
           # every rank's links carried at least half the ring's bytes (other tenants' traffic
           # only adds to the counters, so this can miss a fallback only on a shared box)
           "traffic_on_xgmi": world > 1 and all(t["xgmi_written_mb"] is not None and
                                                t["xgmi_written_mb"] >= 0.5 * t["expected_mb"] for t in traffic),
           "results": results, "max_busbw_gbps": max(r["busbw_gbps"] for r in results) if results else 0.0,
           "all_correct": all(r["correct"] for r in results)}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--sizes-mb", default="1,16,256")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--require-single-hive", action="store_true")
    args = ap.parse_args(argv)
    sizes = [float(s) for s in args.sizes_mb.split(",") if s]
    out = run(sizes, args.iters, args.warmup, args.require_single_hive, args.dtype)
    if out is not None:
        print(json.dumps(out), flush=True)
        if not out["all_correct"]:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""HBM walk cost in a fresh process: first vs repeated calls, and after the 1 GiB
bandwidth test (the node agent's order).  Writes gpurun_out/walk_probe.json."""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from bacchus_gpu_controller_amd import native  # noqa: E402

n = native()
out = []
for label in ("first", "second"):
    t = time.perf_counter()
    r = json.loads(n.diag_hbm_walk(0, 0.9, 4 << 30, 20000))
    out.append({"call": label, "wall_ms": (time.perf_counter() - t) * 1e3,
                **{k: r[k] for k in ("alloc_ms", "elapsed_ms", "bytes_covered", "write_gbps", "read_gbps", "mismatches")}})
t = time.perf_counter()
n.diag_hbm(0, 1 << 30, 2, 1)
out.append({"call": "hbm_1g", "wall_ms": (time.perf_counter() - t) * 1e3})
for chunk in (1 << 30, 16 << 30):
    t = time.perf_counter()
    r = json.loads(n.diag_hbm_walk(0, 0.9, chunk, 20000))
    out.append({"call": f"chunk_{chunk >> 30}g", "wall_ms": (time.perf_counter() - t) * 1e3,
                **{k: r[k] for k in ("alloc_ms", "elapsed_ms", "chunks", "mismatches")}})
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/walk_probe.json", "w"), indent=1)
print(json.dumps(out, indent=1))

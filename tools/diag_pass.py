"""One pass of every HIP diagnostic on device 0, as the node agent runs them (HBM
bandwidth, HBM walk, per-CU MFMA, MFMA GEMM vs host, GEMM soak, PCIe), for a rocprofv3
kernel trace of the whole set:

    rocprofv3 --kernel-trace --stats -d gpurun_out/diag_prof -- python3 tools/diag_pass.py OUT.json
"""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bacchus_gpu_controller_amd import ops  # noqa: E402

out = {}
for name, fn in (("hbm", lambda: ops.hbm(0, nbytes=1 << 30)),
                 ("hbm_walk", lambda: ops.hbm_walk(0)),
                 ("mfma", lambda: ops.mfma(0)),
                 ("gemm_check", lambda: ops.gemm_check(0, 1024, 1024, 1024)),
                 ("gemm_soak", lambda: ops.gemm_soak(0, 8192, 8192, 8192, launches=20)),
                 ("pcie", lambda: ops.pcie(0))):
    t0 = time.time()
    r = fn()
    r["wall_s"] = round(time.time() - t0, 3)
    out[name] = r
    print(name, r.get("passed"), r["wall_s"], flush=True)
with open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag_pass.json", "w") as f:
    json.dump(out, f, indent=1)

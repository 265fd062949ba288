"""One pass of every HIP diagnostic on device 0, as the node agent runs them (HBM
bandwidth, HBM walk, per-CU MFMA, MX fp8/fp4 tiles and rates, MFMA GEMM vs host, GEMM soak,
PCIe, a 2 s burn-in on the default MX fp4 path), for a rocprofv3 kernel trace of the whole set:

    rocprofv3 --kernel-trace --stats -d gpurun_out/diag_prof -- python3 tools/diag_pass.py OUT.json
"""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bacchus_gpu_controller_amd import ops  # noqa: E402



def _burn(dtype, ms=2000):
    from bacchus_gpu_controller_amd import native

    n = native()
    return json.loads(n.diag_burn(n.gpu_backend("amdsmi", ""), 0, 0, ms, 0x5EED, dtype))


out = {}
for name, fn in (("hbm", lambda: ops.hbm(0, nbytes=1 << 30)),
                 ("hbm_walk", lambda: ops.hbm_walk(0)),
                 ("mfma", lambda: ops.mfma(0)),
                 ("mfma_lowp", lambda: ops.mfma_lowp(0)),
                 ("gemm_check", lambda: ops.gemm_check(0, 1024, 1024, 1024)),
                 ("gemm_soak", lambda: ops.gemm_soak(0, 8192, 8192, 8192, launches=20)),
                 ("pcie", lambda: ops.pcie(0)),
                 ("burn_fp4", lambda: _burn("fp4"))):
    t0 = time.time()
    r = fn()
    r["wall_s"] = round(time.time() - t0, 3)
    out[name] = r
    print(name, r.get("passed"), r["wall_s"], flush=True)
with open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag_pass.json", "w") as f:
    json.dump(out, f, indent=1)

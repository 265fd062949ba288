"""One GEMM soak on the GPU box (for rocprofv3 runs): python3 tools/probes/soak_one.py M N K LAUNCHES."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bacchus_gpu_controller_amd import native  # noqa: E402

m, n, k, launches = (int(x) for x in sys.argv[1:5])
print(json.dumps(json.loads(native().diag_gemm_soak(0, m, n, k, launches))), flush=True)

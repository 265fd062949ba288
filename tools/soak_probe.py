"""GEMM soak on the GPU box: correctness at small sizes first, then the rate at 4096^3 and
8192^3 (LDS-tiled bf16 MFMA GEMM, exact checksums).  Writes one JSON file."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bacchus_gpu_controller_amd import native  # noqa: E402


def main(out_path):
    nat = native()
    res = []
    for m, n, k, launches in ((128, 128, 64, 1), (256, 384, 128, 2), (1024, 1024, 1024, 3), (4096, 4096, 4096, 10),
                              (8192, 8192, 8192, 10)):
        r = json.loads(nat.diag_gemm_soak(0, m, n, k, launches))
        print(json.dumps(r), flush=True)
        res.append(r)
        if not r["passed"]:
            break
    json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "soak_probe.json")

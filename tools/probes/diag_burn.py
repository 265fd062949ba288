"""Burn-in measurement on cuda:0: sustained MFMA load for N seconds with amdsmi sampling
(power, gfxclk, temperatures, throttle residency).  Sets the DiagFloors burn defaults.

    python3 tools/probes/diag_burn.py 10 gpurun_out/diag_burn.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bacchus_gpu_controller_amd import native  # noqa: E402


def main(secs, out):
    n = native()
    b = n.gpu_backend("amdsmi", "")
    runs = [json.loads(n.diag_burn(b, 0, 0, int(secs * 1000), 0x5eed + i)) for i in range(2)]
    print(json.dumps(runs, indent=1))
    with open(out, "w") as f:
        json.dump({"duration_s": secs, "runs": runs}, f, indent=1)


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 10, sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/diag_burn.json")

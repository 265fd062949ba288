"""PCIe link probe on the GPU box: amdsmi link capability/state (idle), then the
host<->device copy test with the link sampled while it runs.  Writes one JSON file."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bacchus_gpu_controller_amd import native  # noqa: E402


def main(out_path):
    nat = native()
    b = nat.gpu_backend("amdsmi", "")
    gpus = json.loads(b.discover())
    res = {"static": [{k: g.get(k) for k in ("index", "bdf", "pcie_max_width", "pcie_max_speed_mts", "pcie_max_gen")}
                      for g in gpus]}
    idle = json.loads(b.sample(0, 1))
    res["idle"] = {k: v for k, v in idle.items() if k.startswith("pcie")}
    runs = []
    for size_mb in (64, 256, 1024):
        t0 = time.time()
        runs.append(json.loads(nat.pcie_check(b, 0, 0, size_mb << 20)))
        runs[-1]["wall_s"] = round(time.time() - t0, 3)
    res["pcie_check"] = runs
    res["judged_default_floors"] = json.loads(nat.judge_diag(json.dumps({"pcie": runs[1]}), "{}"))
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "pcie_probe.json")

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
    for m, n, k, launches in ((128, 128, 64, 1), (256, 384, 128, 2), (256, 256, 64, 2), (768, 512, 320, 3),
                              (1024, 1024, 1024, 3), (4096, 4096, 4096, 10), (8192, 8192, 8192, 10)):
        r = json.loads(nat.diag_gemm_soak(0, m, n, k, launches))
        print(json.dumps(r), flush=True)
        res.append(r)
        if not r["passed"]:
            break
    if os.environ.get("SOAK_VS_TORCH", "1") == "1":
        # torch ships its own HIP runtime: measure it in a child process of its own
        import subprocess

        r = subprocess.run([sys.executable, __file__, "--torch"], capture_output=True, text=True, timeout=240)
        res.append({"torch_matmul": json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-500:]})
        print(json.dumps(res[-1]), flush=True)
    json.dump(res, open(out_path, "w"), indent=1)


def torch_rate():
    """The same shapes through torch.matmul (hipBLASLt), bf16 operands in {-1, 0, 1} like
    the soak's, 10 timed launches after 3 warm-ups: the library yardstick for the soak."""
    import torch

    out = []
    for s in (4096, 8192):
        a = torch.randint(-1, 2, (s, s), device="cuda").to(torch.bfloat16)
        b = torch.randint(-1, 2, (s, s), device="cuda").to(torch.bfloat16)
        for _ in range(3):
            c = a @ b
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(10):
            c = a @ b
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / 10
        out.append({"size": s, "ms": round(ms, 3), "tflops": round(2 * s ** 3 / ms / 1e9, 1)})
        del a, b, c
    return out


if __name__ == "__main__":
    if sys.argv[1:] == ["--torch"]:
        print(json.dumps(torch_rate()))
        sys.exit(0)
    main(sys.argv[1] if len(sys.argv) > 1 else "soak_probe.json")

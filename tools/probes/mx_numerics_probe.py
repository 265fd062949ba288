"""MX fp8/fp4 matrix-core numerics probe (MI355X, through gpurun): the block-scaled path on
caller codes (ops.mx_gemm) against an fp64 product of an independent decode, for several
operand dynamic ranges and scale spreads.  Reports the error relative to sum|a||b| (mag)
and to the largest single product, and how often the result equals the fp32-accumulated
exact per-128-K partials.  Writes gpurun_out/mx_numerics.json."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from bacchus_gpu_controller_amd import ops  # noqa: E402

FP4 = np.array([0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0, -0.0, -0.5, -1.0, -1.5, -2.0, -3.0, -4.0, -6.0])
V8 = torch.arange(256, dtype=torch.uint8).view(torch.float8_e4m3fn).to(torch.float64).numpy()
m, n, k = 64, 64, 512
rng = np.random.default_rng(7)
out = []


def fp8_codes(rows, emin, emax):
    e = rng.integers(emin, emax + 1, (rows, k))
    mant = rng.integers(0, 8, (rows, k))
    c = ((rng.integers(0, 2, (rows, k)) << 7) | (e << 3) | mant).astype(np.uint8)
    c[(c & 0x7F) == 0x7F] = 0x7E
    return c


for fmt, label, emin, emax, spread in (("fp8", "full range", 0, 15, 8), ("fp8", "full range, unit scales", 0, 15, 0),
                                       ("fp8", "exp 5..10 (2^-2..2^3)", 5, 10, 0), ("fp8", "exp 7..8 (1..4)", 7, 8, 0),
                                       ("fp8", "exp 7 (1..2), scales +-8", 7, 7, 8), ("fp4", "all codes", 0, 0, 8),
                                       ("fp4", "all codes, unit scales", 0, 0, 0)):
    sa = (127 + rng.integers(-spread, spread + 1, (m, k // 32))).astype(np.uint8)
    sb = (127 + rng.integers(-spread, spread + 1, (n, k // 32))).astype(np.uint8)
    if fmt == "fp8":
        a, bt = fp8_codes(m, emin, emax), fp8_codes(n, emin, emax)
        av, bv = V8[a], V8[bt]
    else:
        na, nb = rng.integers(0, 16, (m, k)), rng.integers(0, 16, (n, k))
        a = (na[:, 0::2] | (na[:, 1::2] << 4)).astype(np.uint8)
        bt = (nb[:, 0::2] | (nb[:, 1::2] << 4)).astype(np.uint8)
        av, bv = FP4[na], FP4[nb]
    A = av * np.repeat(np.exp2(sa.astype(np.float64) - 127), 32, axis=1)
    B = bv * np.repeat(np.exp2(sb.astype(np.float64) - 127), 32, axis=1)
    c = ops.mx_gemm(a, sa, bt, sb, fmt=fmt).astype(np.float64)
    ref = A @ B.T
    mag = np.abs(A) @ np.abs(B).T
    maxp = np.max(np.abs(A)[:, None, :] * np.abs(B)[None, :, :], axis=2)
    acc = np.zeros((m, n), dtype=np.float32)
    for k0 in range(0, k, 128):
        acc = (acc + (A[:, k0:k0 + 128] @ B[:, k0:k0 + 128].T).astype(np.float32)).astype(np.float32)
    err = np.abs(c - ref)
    r = {"fmt": fmt, "operands": label, "scale_spread_log2": spread,
         "err_over_mag_median": float(np.median(err / mag)), "err_over_mag_max": float((err / mag).max()),
         "err_over_max_product_median": float(np.median(err / maxp)),
         "fp32_bound_ratio_max": float((err / (4.0 * k * 5.96e-8 * mag)).max()),
         "equals_fp32_accum_of_exact_partials": float(np.mean(c == acc))}
    out.append(r)
    print(json.dumps(r), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/mx_numerics.json", "w"), indent=1)

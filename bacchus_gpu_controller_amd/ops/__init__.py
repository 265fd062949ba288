"""HIP/CDNA4 GPU health kernels (native/gpu/hip/gpu_diag.hip) exposed to Python.

These are the only compute kernels in the framework: the reference controller has none
(SURVEY §2.5).  They back the node agent's diagnostics before a GPU is advertised
(native/gpu/diag_runner.cc) and can be run by hand:

* ``hbm(device)``       — HBM3E pattern fill / copy / verify at streaming bandwidth
* ``hbm_walk(device)``  — address-in-data walk over most of the free HBM (stuck bits,
  aliased addresses), reporting the first bad address
* ``mfma(device)``      — exact-integer bf16 MFMA tiles on every CU + a throughput pass
* ``mfma_lowp(device)`` — the same for the MX block-scaled fp8 / fp4 matrix-core path
  (``v_mfma_scale_f32_16x16x128_f8f6f4``), with and without E8M0 block scales
* ``gemm_check(device)``— a bf16 GEMM on the matrix cores checked against exact row and
  column checksums (ABFT)
* ``gemm_soak(device)`` — the sustained-throughput soak: the 8-phase ping-pong GEMM
  (256x256 tiles) for ``launches`` launches, every result checksummed
* ``gemm_tiled(a, bt)`` — the soak's kernel on caller operands (A: MxK, Bt: NxK bf16),
  fp32 result; used to check the kernel against a PyTorch fp32 product
* ``mx_gemm(a, sa, bt, sbt, fmt)`` — the MX block-scaled matrix-core path on caller
  codes (fp8 e4m3 bytes or packed fp4 e2m1) and E8M0 scales; used to check the hardware's
  operand/scale layout against an independent PyTorch decode
* ``pcie(device)``      — host<->device copy bandwidth, pinned
* ``device_bdf(device)``— the HIP device's PCI address, to match it to amdsmi / kubelet

All fail loudly (RuntimeError) if ``libbgc_gpu_diag.so`` or the GPU is missing; there
is no CPU fallback.
"""
import json

import numpy as np

from .. import native


def library_path():
    return native().diag_library_path()


def device_count():
    return native().diag_device_count()


def device_arch(device=0):
    return native().diag_device_arch(device)


def device_bdf(device=0):
    return native().diag_device_bdf(device)


def hbm(device=0, nbytes=2 << 30, iters=3, seed=0x5EED):
    return json.loads(native().diag_hbm(device, nbytes, iters, seed))


def hbm_walk(device=0, fraction=0.9, chunk_bytes=4 << 30, budget_ms=20000, seed=0x5EED):
    return json.loads(native().diag_hbm_walk(device, fraction, chunk_bytes, budget_ms, seed))


def mfma(device=0, waves_per_cu=32, iters=4096, seed=0x5EED):
    return json.loads(native().diag_mfma(device, waves_per_cu, iters, seed))


def mfma_lowp(device=0, waves_per_cu=32, iters=4096, seed=0x5EED):
    """MX block-scaled fp8 (e4m3) and fp4 (e2m1) matrix-core tiles on every CU, with unit
    and random E8M0 block scales, checked exactly; then the dense fp8 and fp4 rates."""
    return json.loads(native().diag_mfma_lowp(device, waves_per_cu, iters, seed))


def gemm_check(device=0, m=4096, n=4096, k=4096, seed=0x5EED):
    return json.loads(native().diag_gemm_check(device, m, n, k, seed))


def gemm_soak(device=0, m=8192, n=8192, k=8192, launches=10, seed=0x5EED):
    return json.loads(native().diag_gemm_soak(device, m, n, k, launches, seed))


def pcie(device=0, nbytes=256 << 20, iters=5, seed=0x5EED):
    return json.loads(native().diag_pcie(device, nbytes, iters, seed))


def _bf16_bytes(x):
    """bf16 bits of a float array / tensor (round to nearest even), row-major."""
    try:
        import torch
        if isinstance(x, torch.Tensor):
            return x.detach().to("cpu", torch.bfloat16).contiguous().view(torch.int16).numpy().tobytes()
    except ImportError:
        pass
    f = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    return ((f + 0x7FFF + ((f >> 16) & 1)) >> 16).astype(np.uint16).tobytes()


def gemm_tiled(a, bt, device=0):
    """C = A @ Bt^T on the soak's kernels.  A is MxK, Bt is NxK; M and N must be
    multiples of 128 and K of 64 (the ping-pong kernel runs when M, N are multiples of
    256 and K of 128).  Returns an fp32 numpy array MxN."""
    m, k = a.shape
    n, k2 = bt.shape
    if k != k2:
        raise ValueError(f"inner dimensions differ: A is {m}x{k}, Bt is {n}x{k2}")
    c = native().diag_gemm_tiled(device, m, n, k, _bf16_bytes(a), _bf16_bytes(bt))
    return np.frombuffer(c, dtype=np.float32).reshape(m, n)


def mx_gemm(a, a_scales, bt, bt_scales, fmt="fp8", device=0):
    """C = sum_k a[m,k] 2^(sa[m,k/32]-127) * bt[n,k] 2^(sbt[n,k/32]-127) on the MX matrix
    cores (v_mfma_scale_f32_16x16x128_f8f6f4).  fp8: `a` M x K and `bt` N x K uint8 e4m3
    codes; fp4: M x K/2 and N x K/2 bytes of packed e2m1 codes (element 2i in the low
    nibble).  Scales: uint8 E8M0, M x K/32 and N x K/32.  M, N multiples of 16, K of 128.
    Returns an fp32 numpy array M x N."""
    code = {"fp8": 0, "fp4": 4}[fmt]
    a, bt = np.ascontiguousarray(a, dtype=np.uint8), np.ascontiguousarray(bt, dtype=np.uint8)
    sa, sb = np.ascontiguousarray(a_scales, dtype=np.uint8), np.ascontiguousarray(bt_scales, dtype=np.uint8)
    m, n = a.shape[0], bt.shape[0]
    k = sa.shape[1] * 32
    c = native().diag_mx_gemm(device, code, m, n, k, a.tobytes(), sa.tobytes(), bt.tobytes(), sb.tobytes())
    return np.frombuffer(c, dtype=np.float32).reshape(m, n)

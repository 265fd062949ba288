"""HIP/CDNA4 GPU health kernels (native/gpu/hip/gpu_diag.hip) exposed to Python.

These are the only compute kernels in the framework: the reference controller has none
(SURVEY §2.5).  They back the node agent's pre-advertisement health check:

* ``hbm(device)``  — HBM3E pattern fill / copy / verify at streaming bandwidth
* ``mfma(device)`` — exact-integer bf16 MFMA tiles on every CU + a throughput pass

Both fail loudly (RuntimeError) if ``libbgc_gpu_diag.so`` or the GPU is missing; there
is no CPU fallback.
"""
import json

from .. import native


def library_path():
    return native().diag_library_path()


def device_count():
    return native().diag_device_count()


def device_arch(device=0):
    return native().diag_device_arch(device)


def hbm(device=0, nbytes=2 << 30, iters=3, seed=0x5EED):
    return json.loads(native().diag_hbm(device, nbytes, iters, seed))


def mfma(device=0, waves_per_cu=32, iters=4096, seed=0x5EED):
    return json.loads(native().diag_mfma(device, waves_per_cu, iters, seed))

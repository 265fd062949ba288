"""Build driver for the native parts.

* C++ core, binaries and the pybind11 module: CMake + Ninja into ``build/`` (binaries
  land in ``bin/``, ``_native*.so`` next to this package).
* HIP/CDNA4 kernels: ``hipcc --offload-arch=gfx950`` into ``libbgc_gpu_diag.so`` (see
  ``native/gpu/hip/``).  hipcc cross-compiles without a GPU.

Everything is built in-tree so the artefacts travel with the repo snapshot to the GPU box.
"""
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

from .. import REPO_ROOT

BUILD_DIR = os.path.join(REPO_ROOT, "build")
PKG_DIR = os.path.join(REPO_ROOT, "bacchus_gpu_controller_amd")
HIP_DIR = os.path.join(REPO_ROOT, "native", "gpu", "hip")


def _run(cmd, **kw):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, **kw)


def _jobs():
    return str(min(16, max(1, (os.cpu_count() or 2))))


def build_core(build_type="Release"):
    if not os.path.exists(os.path.join(BUILD_DIR, "build.ninja")):
        _run(["cmake", "-S", REPO_ROOT, "-B", BUILD_DIR, "-G", "Ninja", f"-DCMAKE_BUILD_TYPE={build_type}"])
    _run(["ninja", "-C", BUILD_DIR, "-j", _jobs()])


def hip_sources():
    return sorted(glob.glob(os.path.join(HIP_DIR, "*.hip")) + glob.glob(os.path.join(HIP_DIR, "*.cc")))


def gpu_diag_path():
    return os.path.join(PKG_DIR, "libbgc_gpu_diag.so")


def build_hip(force=False):
    """Compile the HIP/CDNA4 health-diagnostic kernels (C ABI) for gfx950.

    The library is dlopen()ed by the node agent and by ``_native`` (native/gpu/diag.cc).
    ``-amdgpu-mfma-vgpr-form`` keeps MFMA accumulators in the unified VGPR file on gfx950,
    which removes the AGPR shuffles hipcc otherwise emits around the throughput loop.
    """
    srcs = hip_sources()
    if not srcs:
        return None
    out = gpu_diag_path()
    if not force and os.path.exists(out):
        newest = max(os.path.getmtime(s) for s in srcs + glob.glob(os.path.join(HIP_DIR, "*.h")))
        if os.path.getmtime(out) >= newest:
            return out
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-Wno-unused-result",
           f"-I{HIP_DIR}", *srcs, "-o", out + ".tmp"]
    _run(cmd)
    os.replace(out + ".tmp", out)
    return out


def ensure_built(hip=True):
    # pytest-xdist workers (and torchrun ranks) call this concurrently: serialize them,
    # two ninja runs in one build directory race on the same outputs.
    import fcntl

    os.makedirs(BUILD_DIR, exist_ok=True)
    with open(os.path.join(BUILD_DIR, ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        build_core()
        if hip:
            try:
                build_hip()
            except (subprocess.CalledProcessError, FileNotFoundError) as e:  # pragma: no cover
                print(f"warning: HIP build failed: {e}", file=sys.stderr)
                raise


if __name__ == "__main__":
    ensure_built()

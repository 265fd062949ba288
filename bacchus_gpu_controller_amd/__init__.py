"""bacchus-gpu-controller, MI355X-native edition.

A from-scratch rebuild of the bacchus-snu/bacchus-gpu-controller Kubernetes tenancy
controller (UserBootstrap CRD, admission webhook, reconciler, Google-Sheet quota
synchronizer) as native C++17 services, plus an MI355X node agent (amdsmi discovery,
telemetry side thread, HIP/CDNA4 health diagnostics) and an RCCL/xGMI placement probe.

Python is the test/bench surface:
  * ``native()``          -> the pybind11 module over the C++ core (``_native``)
  * ``models``            -> UserBootstrap object builders (CRD data model)
  * ``ops``               -> HIP/CDNA4 GPU health kernels (``libbgc_gpu_diag.so``, loaded by ``_native``)
  * ``parallel``          -> RCCL-over-xGMI all-reduce probe and hive topology
  * ``utils``             -> build + process helpers (binaries under ``bin/``)
  * ``testing``           -> fake Google OAuth2/Drive endpoint, cluster harness
  * ``bench``             -> churn benchmark driver used by ``bench.py`` (config #3), plus the
                             config #4 (``bench.tp8``) and config #5 (``bench.flap``) modes
"""
import importlib
import os

__version__ = "0.1.0"

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# BGC_BIN_DIR lets the test-suite run against sanitizer builds (tools/sanitize.sh).
BIN_DIR = os.environ.get("BGC_BIN_DIR") or os.path.join(REPO_ROOT, "bin")

_native_mod = None


def native():
    """Return the compiled C++ core module, building it first if needed."""
    global _native_mod
    if _native_mod is None and os.environ.get("BGC_NATIVE_MODULE"):
        # a sanitizer build of the module (tools/sanitize.sh asan-py): same name, other file
        from importlib import util as _util

        spec = _util.spec_from_file_location("bacchus_gpu_controller_amd._native",
                                                      os.environ["BGC_NATIVE_MODULE"])
        _native_mod = _util.module_from_spec(spec)
        spec.loader.exec_module(_native_mod)
    if _native_mod is None:
        try:
            _native_mod = importlib.import_module("bacchus_gpu_controller_amd._native")
        except ImportError:
            from .utils.build import ensure_built

            ensure_built()
            _native_mod = importlib.import_module("bacchus_gpu_controller_amd._native")
    return _native_mod


def binary(name):
    """Absolute path of a native binary (controller, admission, kube-lite, ...).
    BGC_BIN_<NAME> (e.g. BGC_BIN_CONTROLLER) substitutes one binary: A/B runs of one
    component's older build against the rest of this tree (tools/gpu_ab.sh)."""
    override = os.environ.get("BGC_BIN_" + name.upper().replace("-", "_"))
    if override:
        return override
    path = os.path.join(BIN_DIR, name)
    if not os.path.exists(path):
        from .utils.build import ensure_built

        ensure_built()
    return path

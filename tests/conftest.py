import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: multi-second integration test")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the C++ core/binaries (and HIP kernels) once per session, incrementally."""
    from bacchus_gpu_controller_amd.utils.build import ensure_built

    ensure_built()
    yield


@pytest.fixture(scope="session")
def nat():
    from bacchus_gpu_controller_amd import native

    return native()


@pytest.fixture(scope="session")
def reference_crd_path():
    p = "/root/reference/charts/bacchus-gpu-controller/templates/crd.yaml"
    return p if os.path.exists(p) else None

"""The sampling profiler (native/core/cpuprof.cc) writes a profile at exit that
tools/cpuprof_report.py symbolizes into native frames."""
import os
import subprocess
import sys

import pytest

from bacchus_gpu_controller_amd import REPO_ROOT
from bacchus_gpu_controller_amd.testing.cluster import Cluster

pytestmark = pytest.mark.slow


@pytest.mark.skipif(bool(os.environ.get("BGC_BIN_DIR")), reason="sanitizer builds own signal delivery")
def test_cpu_profile_of_kube_lite(tmp_path, monkeypatch):
    monkeypatch.setenv("BGC_CPU_PROFILE", str(tmp_path / "kl.%p.prof"))
    with Cluster(admission=False, controller=False) as c:
        for i in range(300):
            c.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": f"p{i}"}})
            c.admin.list("namespaces")
        pid = c.procs["apiserver"].p.pid
    prof = tmp_path / f"kl.{pid}.prof"
    assert prof.exists()
    head = prof.read_text().splitlines()[0]
    assert head.startswith("# bgc cpuprof v1") and "samples=" in head
    out = subprocess.run([sys.executable, os.path.join(REPO_ROOT, "tools", "cpuprof_report.py"), str(prof),
                          "--collapsed", str(tmp_path / "c.txt")], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "bgc::" in out.stdout  # frames resolved through the frame-pointer walk
    assert (tmp_path / "c.txt").read_text().strip()

"""Round-4 LeakSanitizer item, pinned down: a thread that used OpenSSL and
ends during process exit, after OpenSSL's atexit cleanup, leaks its per-thread state
(tools/probes/lsan_openssl_exit_race.cc).  bgc::process_init() turns that handler off
(OPENSSL_INIT_NO_ATEXIT); with it off the same program is clean."""
import os
import shutil
import subprocess

import pytest

from bacchus_gpu_controller_amd import REPO_ROOT

SRC = os.path.join(REPO_ROOT, "tools", "probes", "lsan_openssl_exit_race.cc")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("no g++")
    out = str(tmp_path_factory.mktemp("lsan") / "race")
    p = subprocess.run([gxx, "-std=c++17", "-g", "-fsanitize=address", SRC, "-o", out, "-lcrypto", "-lpthread"],
                       capture_output=True, text=True, timeout=120)
    if p.returncode != 0:
        pytest.skip("cannot build with -fsanitize=address: " + p.stderr[-500:])
    return out


def run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1")
    env.pop("LD_PRELOAD", None)
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=60, env=env)


def test_openssl_cleanup_at_exit_leaks_a_late_threads_state(exe):
    p = run(exe)
    if "LeakSanitizer has encountered a fatal error" in p.stderr or "ptrace" in p.stderr:
        pytest.skip("LeakSanitizer cannot run here")
    assert "Direct leak" in p.stderr and "CRYPTO_zalloc" in p.stderr, p.stderr[-2000:]


def test_no_atexit_cleanup_is_clean(exe):
    p = run(exe, "no-atexit")
    assert p.returncode == 0 and "leak" not in p.stderr.lower(), p.stderr[-2000:]

"""The asynchronous log writer never makes a logging thread wait for stderr I/O.

Round 5 found the batch write(2) running under the buffer lock (native/core/log.cc): a
stderr that blocks (a container runtime's pipe read slowly, a log file under writeback
throttling) then stalled every thread that logs a line.  Here stderr is a pipe nobody
reads: the pipe fills after 64 KiB and the writer thread blocks in write(2), but 8 threads
logging 256 KiB more (under the writer's 1 MiB synchronous-flush bound) never wait."""
import os
import subprocess
import sys

from bacchus_gpu_controller_amd import REPO_ROOT

CHILD = """
import sys
sys.path.insert(0, {root!r})
from bacchus_gpu_controller_amd import native
nat = native()
nat.log_burst(1, 200, 500)           # ~100 KiB: fills the unread pipe, the writer blocks
worst = nat.log_burst(8, 64, 500)    # ~256 KiB more while it is blocked
print(f"{{worst:.3f}}", flush=True)
"""


def test_loggers_do_not_wait_for_a_blocked_stderr():
    p = subprocess.Popen([sys.executable, "-c", CHILD.format(root=REPO_ROOT)], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, env=dict(os.environ, RUST_LOG="info"))
    try:
        line = p.stdout.readline().decode().strip()  # stderr is not read until this arrives
        assert line, "the child never reported: its loggers blocked on stderr"
        assert float(line) < 500.0, f"a LOG_INFO call waited {line} ms"
    finally:
        p.stderr.read()  # let it flush and exit
        p.wait(timeout=30)

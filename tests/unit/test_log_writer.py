"""The asynchronous log writer never makes a logging thread wait for stderr I/O.

Round 5 found the batch write(2) running under the buffer lock (native/core/log.cc), and
round 6 the same stall on the ERROR path: an ERROR line (every admission deny,
reference src/admission.rs:277-279,285-289; every error_policy, src/controller.rs:157-175)
or a full 1 MiB buffer flushed synchronously and waited for stderr while holding the
buffer lock, so every other logging thread waited too.

Here stderr is a pipe nobody reads: it fills after 64 KiB and the writer thread blocks in
write(2).  Then, with it blocked:
  * 8 threads log 256 KiB of INFO with one ERROR line among them;
  * 8 threads log ~2.4 MiB of INFO, past the 1 MiB bound: lines are dropped and counted.
No LOG_* call may take 50 ms.  Once the parent drains stderr, every line that was kept
comes out in the order it was logged, the drop is reported in one line, and lines logged
after the unblock all arrive, in order."""
import os
import re
import subprocess
import sys
import threading

from bacchus_gpu_controller_amd import REPO_ROOT

CHILD = """
import sys
sys.path.insert(0, {root!r})
from bacchus_gpu_controller_amd import native
nat = native()
nat.log_burst(1, 200, 500, tag="fill")                    # ~100 KiB: the writer blocks
err = nat.log_burst(8, 64, 500, error_at=10, tag="err")   # 256 KiB incl. one ERROR line
big = nat.log_burst(8, 600, 500, tag="big")               # ~2.4 MiB: past the 1 MiB bound
print(f"{{err:.3f}} {{big:.3f}} {{nat.log_lines_dropped()}}", flush=True)
sys.stdin.readline()                                      # the parent now drains stderr
nat.log_flush()                                           # wait until it has
nat.log_burst(1, 100, 20, tag="after")
nat.log_flush()
"""

LINE = re.compile(r"(INFO|ERROR) burst: (\w+) (\d+) (\d+) x+$")


def test_loggers_never_wait_for_a_blocked_stderr():
    p = subprocess.Popen([sys.executable, "-c", CHILD.format(root=REPO_ROOT)], stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=dict(os.environ, RUST_LOG="info"))
    err_chunks = []
    try:
        line = p.stdout.readline().decode().strip()  # stderr is not read until this arrives
        assert line, "the child never reported: its loggers blocked on stderr"
        err_ms, big_ms, dropped = line.split()
        assert float(err_ms) < 50.0, f"a LOG_* call waited {err_ms} ms with an ERROR line in the burst"
        assert float(big_ms) < 50.0, f"a LOG_INFO call waited {big_ms} ms past the 1 MiB bound"
        assert int(dropped) > 0, "2.4 MiB behind a blocked stderr dropped nothing"
        reader = threading.Thread(target=lambda: err_chunks.append(p.stderr.read()))
        reader.start()
        p.stdin.write(b"go\n")
        p.stdin.flush()
        reader.join(timeout=60)
        assert p.wait(timeout=30) == 0
    finally:
        if p.poll() is None:
            p.kill()
    text = b"".join(err_chunks).decode()
    last = {}
    levels = {}
    notices = []
    for ln in text.splitlines():
        m = LINE.search(ln)
        if not m:
            if "log lines dropped" in ln:
                notices.append(ln)
            continue
        lvl, tag, t, i = m.group(1), m.group(2), int(m.group(3)), int(m.group(4))
        key = (tag, t)
        assert i > last.get(key, -1), f"{tag} thread {t}: line {i} after line {last[key]}"
        last[key] = i
        levels[(tag, t, i)] = lvl
    assert levels.get(("err", 0, 10)) == "ERROR", "the ERROR line never reached stderr"
    assert all(last.get(("err", t)) == 63 for t in range(8)), "lines of the ERROR burst were lost"
    assert last.get(("after", 0)) == 99 and sum(1 for k in levels if k[0] == "after") == 100
    assert len(notices) >= 1, "no 'log lines dropped' notice after stderr drained"
    reported = sum(int(re.search(r"(\d+) log lines dropped", n).group(1)) for n in notices)
    assert reported == int(dropped)
    kept_big = sum(1 for k in levels if k[0] == "big")
    assert kept_big + int(dropped) == 8 * 600

"""Round-6 observability surfaces, and the process start-up checks.

* /debug/trace: per-tenant stage marks, armed by name prefix, kept per thread; a request
  through kube-lite, the admission server and the controller leaves its marks in each.
* /debug/stalls and bgc_stall_*: every service runs a 1 ms oversleep sampler.
* Threads carry names (per-thread CPU in the bench's busiest_threads).
* BGC_DIE_WITH_PARENT naming a PID that is not the parent fails loudly.
"""
import os
import subprocess

import pytest
import requests

from bacchus_gpu_controller_amd import BIN_DIR
from bacchus_gpu_controller_amd.bench import attribution
from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

pytestmark = pytest.mark.slow


def _tenant(c, name):
    c.as_user(f"oidc:{name}", ["gpu"]).create(
        "userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap", "metadata": {"name": name}, "spec": {}})


def test_trace_marks_follow_a_tenant_through_every_process():
    with Cluster() as c:
        ctl = f"http://127.0.0.1:{c.controller_port}"
        adm = f"https://127.0.0.1:{c.admission_port}"
        ca = os.path.join(c.cert_dir, "ca.crt")
        ends = [(c.server, c.verify), (ctl, None), (adm, ca)]
        for base, verify in ends:
            assert requests.post(base + "/debug/trace", data="tr-", timeout=5, verify=verify).status_code == 200
        _tenant(c, "tr-alice")
        _tenant(c, "other")  # not under the armed prefix: no marks
        wait_for(lambda: c.admin.get_or_none("namespaces", "tr-alice"), desc="namespace")
        dumps = [requests.delete(base + "/debug/trace", timeout=5, verify=verify).json() for base, verify in ends]
        stages = {st for d in dumps for n, st, _ in d["marks"] if n == "tr-alice"}
        assert not any(n == "other" for d in dumps for n, _, _ in d["marks"])
        # kube-lite: the create's receipt, webhook call and commit; each watch delivery
        for step in ("recv", "hook0", "hook1", "commit", "resp"):
            assert any(s.startswith("kl.userbootstraps.POST.") and s.endswith("." + step) for s in stages), step
        assert any(s.startswith("kl.watch.userbootstraps.controller.") for s in stages), stages
        assert "adm.review0.CREATE" in stages and "adm.review1.CREATE" in stages
        assert {"ctl.primary_event", "ctl.reconcile0", "ctl.apply.namespaces.send"} <= stages, stages
        # the marks join into one timeline (CLOCK_MONOTONIC shared by the processes)
        timeline = attribution.group_marks(dumps)["tr-alice"]
        t = {st: ts for ts, st in reversed(timeline)}  # first occurrence
        assert t["adm.review0.CREATE"] < t["ctl.primary_event"] < t["ctl.apply.namespaces.send"]
        # taken: a second read is empty and disarmed
        again = requests.get(c.server + "/debug/trace", timeout=5, verify=c.verify).json()
        assert again["marks"] == [] and again["armed"] is False


def test_watch_sections_are_timed_on_both_ends(monkeypatch):
    """A watch event's delay splits into kube-lite's write plus the transport and the reader
    (sent -> the controller's read) and the parse (read -> event), with the write itself
    (sent -> written) beside it; the
    watch writer's and the watcher's own sections are kept as slow sections past
    BGC_STALL_RECORD_US (0 here: every one)."""
    monkeypatch.setenv("BGC_STALL_RECORD_US", "0")
    with Cluster(admission=False) as c:
        ctl = f"http://127.0.0.1:{c.controller_port}"
        ends = [(c.server, c.verify), (ctl, None)]
        for base, verify in ends:
            assert requests.post(base + "/debug/trace", data="ws-", timeout=5, verify=verify).status_code == 200
            requests.delete(base + "/debug/stalls", timeout=5, verify=verify)
        _tenant(c, "ws-bob")
        wait_for(lambda: c.admin.get_or_none("namespaces", "ws-bob"), desc="namespace")
        dumps = [requests.delete(base + "/debug/trace", timeout=5, verify=verify).json() for base, verify in ends]
        t = {}
        for ts, st in attribution.group_marks(dumps)["ws-bob"]:
            t.setdefault(st, ts)
        sent, written = "kl.watch.userbootstraps.controller.sent", "kl.watch.userbootstraps.controller.written"
        # ".written" is read after the write returned: the reader may already have the bytes
        assert t[sent] <= t[written] and t[sent] <= t["ctl.primary_read"] <= t["ctl.primary_event"], t
        slow = {base: requests.get(base + "/debug/stalls", timeout=5, verify=verify).json()["slow"]
                for base, verify in ends}
        assert any(what == "kw:userbootstraps write" for _, _, what in slow[c.server]), slow[c.server][:5]
        assert any(what == "w:userbootstraps event" for _, _, what in slow[ctl]), slow[ctl][:5]
        # and the bench's attribution reads them as sections overlapping a segment
        stall_dumps = [dict(requests.get(base + "/debug/stalls", timeout=5, verify=verify).json(), process=p)
                       for (base, verify), p in zip(ends, ("kube-lite", "controller"))]
        got = attribution.analyze(dumps, stall_dumps)
        assert "controller w:userbootstraps event" in got["slow_sections"], got["slow_sections"]
        assert got["watch_writes"]["userbootstraps.controller"]["n"] >= 1, got["watch_writes"]


def test_lock_sections_of_watchers_and_workers(monkeypatch):
    """BGC_LOCK_SECTION_US (0 here: every one): the controller's watchers time their store
    apply and queue add, its workers their queue finish, and the synchronizer's watcher its
    own; /debug/stalls serves them as slow sections (the round-6 work-queue finding)."""
    from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle

    monkeypatch.setenv("BGC_LOCK_SECTION_US", "0")
    google = FakeGoogle().start()
    try:
        google.set_rows([{"id_username": "ls-carol"}])
        with Cluster(admission=False) as c:
            c.start_synchronizer(google, interval=3600, extra_env={"CONF_WATCH": "true"})
            ctl, sync = f"http://127.0.0.1:{c.controller_port}", f"http://127.0.0.1:{c.sync_port}"
            _tenant(c, "ls-carol")
            wait_for(lambda: c.admin.get_or_none("namespaces", "ls-carol"), desc="namespace")

            def sections(base):
                return {what for _, _, what in requests.get(base + "/debug/stalls", timeout=5).json()["slow"]}

            wait_for(lambda: {"w:userbootstraps store", "w:userbootstraps queue", "reconcile queue",
                              "w:namespaces store"} <= sections(ctl), desc="controller lock sections")
            wait_for(lambda: {"w:userbootstraps store", "w:userbootstraps queue"} <= sections(sync),
                     desc="synchronizer lock sections")
    finally:
        google.stop()


def test_every_service_runs_a_stall_sampler_and_names_its_threads():
    with Cluster() as c:
        for base, verify, proc in ((f"http://127.0.0.1:{c.controller_port}", None, "controller"),
                                   (f"https://127.0.0.1:{c.admission_port}", os.path.join(c.cert_dir, "ca.crt"),
                                    "admission"),
                                   (c.server, c.verify, "apiserver")):
            m = requests.get(base + "/metrics", timeout=5, verify=verify).text
            assert "bgc_stall_oversleep_seconds_count" in m and "bgc_log_lines_dropped_total 0" in m, proc
            st = requests.get(base + "/debug/stalls", timeout=5, verify=verify).json()
            assert st["running"] is True and st["ticks"] > 0, (proc, st)
            pid = c.procs[proc].p.pid

            def names():
                out = set()
                for t in os.listdir(f"/proc/{pid}/task"):
                    try:
                        out.add(open(f"/proc/{pid}/task/{t}/comm").read().strip())
                    except OSError:
                        pass  # the thread exited meanwhile
                return out

            want = {"stall-sampler"} | ({"reconcile", "w:userbootstrap"} if proc == "controller" else set())
            # the controller starts its workers once its caches synced (slow on a sanitizer build)
            wait_for(lambda: want <= names(), timeout=30, desc=f"{proc} thread names {want}")


def test_die_with_parent_naming_another_pid_fails_loudly():
    """A service started under a wrapper (its parent is not the PID the harness named) used
    to exit 0 at once, which read as a clean stop."""
    env = dict(os.environ, BGC_DIE_WITH_PARENT="1", CONF_LISTEN_ADDR="127.0.0.1", CONF_LISTEN_PORT="0")
    p = subprocess.run([os.path.join(BIN_DIR, "controller")], env=env, capture_output=True, text=True, timeout=30)
    assert p.returncode == 3, (p.returncode, p.stderr[-500:])
    assert "BGC_DIE_WITH_PARENT=1 but the parent process is" in p.stderr

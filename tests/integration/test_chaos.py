"""Crash-restart chaos (every process is stateless, a restart re-lists).

Tenants onboard continuously while the controller, the admission webhook and the
synchronizer are each SIGKILLed (no graceful shutdown) and restarted, as the kubelet
would.  Creates that hit the dead webhook fail (failurePolicy: Fail) and the client
retries them.  At the end every tenant must be fully provisioned, with exactly one set of
children, and no other namespaces must have appeared.
"""
import signal
import threading
import time

import pytest

from bacchus_gpu_controller_amd.testing.cluster import Cluster
from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle
from bacchus_gpu_controller_amd.testing.kubeapi import ApiError, wait_for

pytestmark = pytest.mark.slow

N = 48


def _ready(c, name):
    ub = c.admin.get_or_none("userbootstraps", name)
    rq = c.admin.get_or_none("resourcequotas", name, name)
    rb = c.admin.get_or_none("rolebindings", name, name)
    return bool(ub and (ub.get("status") or {}).get("synchronized_with_sheet") and rq
                and rq["spec"]["hard"].get("requests.amd.com/gpu") == "1" and rb)


def test_components_killed_mid_churn_converge():
    names = [f"chaos{i:02d}" for i in range(N)]
    google = FakeGoogle().start()
    google.set_rows([{"id_username": n, "gpu": 1} for n in names])
    try:
        with Cluster(controller_env={"CONF_ERROR_REQUEUE_MS": "200"}) as c:
            c.start_synchronizer(google, interval=60, extra_env={"CONF_WATCH": "true", "CONF_SHEET_POLL_MS": "500"})
            created, webhook_refusals, errors = [], [], []

            def creator():
                for n in names:
                    api = c.as_user(f"oidc:{n}", ["gpu"])
                    deadline = time.time() + 60
                    while True:
                        try:
                            api.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                                          "metadata": {"name": n}, "spec": {}})
                            created.append(n)
                            break
                        except ApiError as e:
                            if e.code == 500 and "webhook" in e.message and time.time() < deadline:
                                webhook_refusals.append(n)  # admission is down: retry, as a client would
                                time.sleep(0.1)
                                continue
                            errors.append(f"{n}: {e.code} {e.message}")
                            return
                    time.sleep(0.05)

            t = threading.Thread(target=creator)
            t.start()
            kills = []

            def kill_and_restart(name, restart, pause):
                c.procs[name].p.send_signal(signal.SIGKILL)
                c.procs[name].p.wait(10)
                kills.append(name)
                time.sleep(pause)
                restart()

            wait_for(lambda: len(created) >= 8, timeout=30, desc="8 creates")
            kill_and_restart("controller", c.start_controller, 0.5)
            wait_for(lambda: len(created) >= 16, timeout=30, desc="16 creates")
            kill_and_restart("admission", c.start_admission, 1.0)
            wait_for(lambda: len(created) >= 28, timeout=60, desc="28 creates")
            kill_and_restart("synchronizer", lambda: c.start_synchronizer(
                google, interval=60, extra_env={"CONF_WATCH": "true", "CONF_SHEET_POLL_MS": "500"}), 0.5)
            wait_for(lambda: len(created) >= 40, timeout=60, desc="40 creates")
            kill_and_restart("controller", c.start_controller, 0.2)
            t.join(120)
            assert not errors, errors
            assert sorted(created) == names
            wait_for(lambda: all(_ready(c, n) for n in names), timeout=60, interval=0.2, desc="every tenant Ready")
            assert kills == ["controller", "admission", "synchronizer", "controller"]
            # exactly one set of children per tenant, nothing else created
            ns = {x["metadata"]["name"] for x in c.admin.list("namespaces")["items"]}
            assert {n for n in ns if n.startswith("chaos")} == set(names)
            for n in names:
                assert len(c.admin.list("resourcequotas", namespace=n)["items"]) == 1
                assert len(c.admin.list("rolebindings", namespace=n)["items"]) == 1
            # the webhook was down for a while, so at least one create had to be retried
            assert webhook_refusals
    finally:
        google.stop()

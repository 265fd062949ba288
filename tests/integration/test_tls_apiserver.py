"""Components reach an HTTPS apiserver through kubeconfigs (kube-client's inference path:
$KUBECONFIG -> certificate-authority + tokenFile, both relative to the kubeconfig), the
way they do in a real cluster, instead of the plain-HTTP test overrides."""
import os
import time

import pytest
import requests

from bacchus_gpu_controller_amd import native
from bacchus_gpu_controller_amd.testing.cluster import CONTROLLER_TOKEN, Cluster, free_port
from bacchus_gpu_controller_amd.testing.fake_google import FakeGoogle
from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

pytestmark = pytest.mark.slow


def test_onboarding_over_https_with_kubeconfigs():
    google = FakeGoogle().start()
    try:
        google.set_rows([{"id_username": "tina", "gpu": 4}])
        with Cluster(tls_apiserver=True, controller_env={"CONF_REQUEUE_SECS": "5"}) as c:
            assert c.server.startswith("https://")
            with pytest.raises(requests.exceptions.SSLError):
                requests.get(c.server + "/version", timeout=5)  # not trusted without the cluster CA
            c.start_node_agent(node_name="mi355x-0", backend="mock")
            c.start_synchronizer(google, interval=1)
            c.as_user("oidc:tina", ["gpu"]).create(
                "userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                   "metadata": {"name": "tina"}, "spec": {}})
            rq = wait_for(lambda: c.admin.get_or_none("resourcequotas", "tina", "tina"), timeout=10, desc="quota")
            assert rq["spec"]["hard"]["requests.amd.com/gpu"] == "4"
            wait_for(lambda: c.admin.get_or_none("rolebindings", "tina", "tina"), timeout=10, desc="rolebinding")
            node = wait_for(lambda: c.admin.get_or_none("nodes", "mi355x-0"), desc="node")
            assert node["metadata"]["labels"]["amd.com/gpu.product"] == "MI355X"
            managers = {m["manager"] for m in c.admin.get("namespaces", "tina")["metadata"]["managedFields"]}
            assert "bacchus-gpu-controller.bacchus.io" in managers
    finally:
        google.stop()


def test_untrusted_apiserver_certificate_is_rejected():
    with Cluster(tls_apiserver=True, admission=False, controller=False) as c:
        other_ca = native().make_ca_and_leaf("evil", ["127.0.0.1"], 1)["ca_cert"]
        bad_ca = os.path.join(c.workdir, "other-ca.crt")
        with open(bad_ca, "w") as f:
            f.write(other_ca)
        port = free_port()
        env = {"CONF_LISTEN_ADDR": "127.0.0.1", "CONF_LISTEN_PORT": str(port), "RUST_LOG": "info",
               "KUBECONFIG": c.write_kubeconfig(CONTROLLER_TOKEN, "controller-badca", ca_file=bad_ca)}
        p = c.start_process("controller", "controller", env)
        c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                          "metadata": {"name": "mallory"}, "spec": {"kube_username": "m"}})
        wait_for(lambda: "certificate verify failed" in p.output(),
                 timeout=15, desc="TLS verification failure logged")
        time.sleep(0.5)
        assert c.admin.get_or_none("namespaces", "mallory") is None

"""Process-level harness: kube-lite + the native admission/controller/synchronizer/
node-agent binaries wired together the way the Helm chart wires them in a real cluster
(webhook registered through a MutatingWebhookConfiguration with a caBundle, TLS to the
webhook, service-account tokens for each component).

Used by tests/integration and by bench.py.
"""
import base64
import json
import os
import re
import socket
import subprocess
import tempfile
import threading
import time

import requests

from .. import REPO_ROOT, binary, native
from .kubeapi import KubeApi, wait_for

NAMESPACE = "bgc"
RELEASE = "bgc"
WEBHOOK_SERVICE = f"{RELEASE}-admission"

ADMIN_TOKEN = "admin-token"
CONTROLLER_TOKEN = "controller-token"
SYNC_TOKEN = "synchronizer-token"
NODE_AGENT_TOKEN = "node-agent-token"


_issued_ports = set()


def free_port():
    """A port nothing listens on, never one this process handed out before: the OS may
    return a just-released port again, and two components told to listen on the same port
    would have one fail to bind while the other answers its health checks."""
    while True:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if p not in _issued_ports:
            _issued_ports.add(p)
            return p


# glibc malloc: a deeper per-thread cache (default 7 chunks per size class) keeps the
# services' many short-lived JSON allocations off the shared arenas.  Measured on the
# MI355X box: +14% CR/s, -12% control-plane CPU per CR (profiles/archive/malloc_tunables_r1/);
# 64 per class keeps that at half the cached memory of 1024 (profiles/archive/tcache_ab_r1/).
# The container image sets the same value (Dockerfile ENV).  Only the thread cache is set
# here (mallopt has no knob for it): arenas, heap growth and trimming are set in one place,
# bgc::tune_malloc (native/core/process.cc).
SERVICE_GLIBC_TUNABLES = "glibc.malloc.tcache_count=64:glibc.malloc.tcache_max=16384"


class Proc:
    def __init__(self, name, cmd, env, workdir):
        self.name = name
        # a restarted or second replica gets a log of its own: truncating the path another
        # instance still writes at its own offset interleaves both (and NUL-fills the gap)
        self.log_path = os.path.join(workdir, f"{name}.log")
        n = 1
        while os.path.exists(self.log_path):
            self.log_path = os.path.join(workdir, f"{name}.{n}.log")
            n += 1
        self.log = open(self.log_path, "wb")
        full_env = dict(os.environ)
        full_env.setdefault("GLIBC_TUNABLES", SERVICE_GLIBC_TUNABLES)
        # tests and the bench read exact latency samples (/debug/samples/<name>); the
        # binaries and the chart leave them off
        full_env.setdefault("CONF_DEBUG_ENDPOINTS", "true")
        full_env.update(env)
        # The service SIGTERMs itself when this process dies (bgc::process_init reads
        # BGC_DIE_WITH_PARENT), so a test run killed by a timeout leaves no services behind.
        # The kernel's parent-death signal follows the starting *thread*: main thread only.
        if threading.current_thread() is threading.main_thread():
            full_env.setdefault("BGC_DIE_WITH_PARENT", str(os.getpid()))
        self.p = subprocess.Popen(cmd, env=full_env, stdout=self.log, stderr=subprocess.STDOUT,
                                  start_new_session=True)

    def alive(self):
        return self.p.poll() is None

    def stop(self, timeout=15):
        if self.p.poll() is None:
            self.p.terminate()
            try:
                self.p.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                self.p.kill()
                self.p.wait()
        self.log.close()
        return self.p.returncode

    def output(self):
        try:
            with open(self.log_path, "rb") as f:
                return f.read().decode(errors="replace")
        except OSError:
            return ""


def webhook_configuration(ca_pem, port, timeout_seconds=10):
    """What charts/bacchus-gpu-controller/templates/webhook.yaml renders (reference
    templates/webhook.yaml:1-27), with cert-manager's CA injection done inline."""
    return {
        "apiVersion": "admissionregistration.k8s.io/v1",
        "kind": "MutatingWebhookConfiguration",
        "metadata": {"name": RELEASE},
        "webhooks": [{
            "name": f"{RELEASE}-admission.bacchus.io",
            "rules": [{"apiGroups": ["bacchus.io"], "apiVersions": ["v1"], "resources": ["userbootstraps"],
                       "scope": "*", "operations": ["CREATE", "UPDATE", "DELETE"]}],
            "clientConfig": {"service": {"namespace": NAMESPACE, "name": WEBHOOK_SERVICE, "path": "/mutate",
                                         "port": port},
                             "caBundle": base64.b64encode(ca_pem.encode()).decode()},
            "timeoutSeconds": timeout_seconds,
            "sideEffects": "None",
            "admissionReviewVersions": ["v1"],
            "failurePolicy": "Fail",
        }],
    }


class Cluster:
    def __init__(self, workdir=None, admission=True, controller=True, controller_env=None, admission_env=None,
                 apiserver_args=None, log_level="warn", tls_apiserver=False):
        """tls_apiserver: kube-lite serves HTTPS with its own CA and every component reaches it
        through a kubeconfig (certificate-authority + tokenFile, paths relative to the
        kubeconfig) instead of the BGC_KUBE_* test overrides."""
        self._tmp = None
        keep = os.environ.get("BGC_CLUSTER_LOGDIR")  # keep component logs (sanitizer runs)
        if workdir is None and keep:
            os.makedirs(keep, exist_ok=True)
            # named after the running test (truncated: unix socket paths go under it), so a
            # sanitizer report leads back to it
            test = os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0].rsplit("::", 1)[-1]
            prefix = "cluster-" + re.sub(r"[^A-Za-z0-9_.-]", "_", test)[:32] + "-" if test else "cluster-"
            workdir = tempfile.mkdtemp(prefix=prefix, dir=keep)
        if workdir is None:
            self._tmp = tempfile.TemporaryDirectory(prefix="bgc-cluster-")
            workdir = self._tmp.name
        self.workdir = workdir
        self.want_admission = admission
        self.want_controller = controller
        self.controller_env = controller_env or {}
        self.admission_env = admission_env or {}
        self.apiserver_args = apiserver_args or []
        self.log_level = log_level
        self.tls_apiserver = tls_apiserver
        self.verify = True
        self.procs = {}
        self.server = None
        self.ca_pem = None
        self.admission_port = None
        self.controller_port = None

    # ------------------------------------------------------------------ setup
    def _write_tokens(self):
        path = os.path.join(self.workdir, "tokens.csv")
        with open(path, "w") as f:
            f.write(f'{ADMIN_TOKEN},kubernetes-admin,uid-admin,"system:masters"\n')
            f.write(f'{CONTROLLER_TOKEN},system:serviceaccount:{NAMESPACE}:{RELEASE}-controller,uid-ctrl,"system:serviceaccounts"\n')
            f.write(f'{SYNC_TOKEN},system:serviceaccount:{NAMESPACE}:{RELEASE}-synchronizer,uid-sync,"system:serviceaccounts"\n')
            f.write(f'{NODE_AGENT_TOKEN},system:serviceaccount:{NAMESPACE}:{RELEASE}-node-agent,uid-na,"system:serviceaccounts"\n')
        return path

    def _certs(self):
        dns = [f"{WEBHOOK_SERVICE}.{NAMESPACE}", f"{WEBHOOK_SERVICE}.{NAMESPACE}.svc", "localhost", "127.0.0.1"]
        b = native().make_ca_and_leaf(WEBHOOK_SERVICE, dns, 90)
        d = os.path.join(self.workdir, "cert")
        os.makedirs(d, exist_ok=True)
        for k, fn in (("cert", "tls.crt"), ("key", "tls.key"), ("ca_cert", "ca.crt"), ("ca_key", "ca.key")):
            with open(os.path.join(d, fn), "w") as f:
                f.write(b[k])
        self.ca_pem = b["ca_cert"]
        self.cert_dir = d
        return d

    def start(self):
        tokens = self._write_tokens()
        self.admission_port = free_port() if self.want_admission else 1
        port_file = os.path.join(self.workdir, "apiserver.port")
        args = [binary("kube-lite"), "--port", "0", "--port-file", port_file, "--token-file", tokens,
                "--no-anonymous", "--bookmark-ms", "1000",
                "--service-override", f"{NAMESPACE}/{WEBHOOK_SERVICE}=127.0.0.1:{self.admission_port}"]
        if self.tls_apiserver:
            args += self._apiserver_certs()
        args += self.apiserver_args
        self.procs["apiserver"] = Proc("apiserver", args, {"RUST_LOG": self.log_level}, self.workdir)
        wait_for(lambda: os.path.exists(port_file), 20, desc="kube-lite port file")
        scheme = "https" if self.tls_apiserver else "http"
        self.server = f"{scheme}://127.0.0.1:{open(port_file).read().strip()}"
        self.admin = KubeApi(self.server, ADMIN_TOKEN, verify=self.verify)
        self.admin.create("namespaces", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": NAMESPACE}})
        self.admin.create("customresourcedefinitions", json.loads(native().crd_json()))
        if self.want_admission:
            self._certs()
            self.start_admission()
            self.admin.create("mutatingwebhookconfigurations", webhook_configuration(self.ca_pem, self.admission_port))
        if self.want_controller:
            self.start_controller()
        return self

    def _apiserver_certs(self):
        b = native().make_ca_and_leaf("kube-apiserver", ["kubernetes", "kubernetes.default.svc", "localhost",
                                                         "127.0.0.1"], 30)
        d = os.path.join(self.workdir, "apiserver-pki")
        os.makedirs(d, exist_ok=True)
        for k, fn in (("cert", "apiserver.crt"), ("key", "apiserver.key"), ("ca_cert", "ca.crt")):
            with open(os.path.join(d, fn), "w") as f:
                f.write(b[k])
        self.apiserver_ca = os.path.join(d, "ca.crt")
        self.verify = self.apiserver_ca
        return ["--tls-cert", os.path.join(d, "apiserver.crt"), "--tls-key", os.path.join(d, "apiserver.key")]

    def write_kubeconfig(self, token, name, ca_file=None):
        """kubeconfig for one component: relative certificate-authority and tokenFile (both
        resolved against the kubeconfig's directory, like client-go)."""
        d = os.path.join(self.workdir, "kubeconfigs", name)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "token"), "w") as f:
            f.write(token + "\n")
        with open(os.path.join(d, "ca.crt"), "w") as f:
            f.write(open(ca_file or self.apiserver_ca).read())
        path = os.path.join(d, "config")
        with open(path, "w") as f:
            f.write(f"""apiVersion: v1
kind: Config
clusters:
- name: kube-lite
  cluster:
    server: {self.server}
    certificate-authority: ca.crt
users:
- name: {name}
  user:
    tokenFile: token
contexts:
- name: {name}@kube-lite
  context:
    cluster: kube-lite
    user: {name}
current-context: {name}@kube-lite
""")
        return path

    def component_env(self, token, port):
        env = {"CONF_LISTEN_ADDR": "127.0.0.1", "CONF_LISTEN_PORT": str(port), "RUST_LOG": self.log_level}
        if self.tls_apiserver:
            name = {CONTROLLER_TOKEN: "controller", SYNC_TOKEN: "synchronizer",
                    NODE_AGENT_TOKEN: "node-agent"}.get(token, "admin")
            env["KUBECONFIG"] = self.write_kubeconfig(token, name)
        else:
            env.update({"BGC_KUBE_SERVER": self.server, "BGC_KUBE_TOKEN": token})
        return env

    def start_admission(self):
        env = {
            "CONF_LISTEN_ADDR": "127.0.0.1", "CONF_LISTEN_PORT": str(self.admission_port),
            "CONF_CERT_PATH": os.path.join(self.cert_dir, "tls.crt"),
            "CONF_KEY_PATH": os.path.join(self.cert_dir, "tls.key"),
            "CONF_OIDC_USERNAME_PREFIX": "oidc:", "CONF_DEFAULT_ROLE_NAME": "edit",
            "CONF_AUTHORIZED_GROUP_NAMES": "gpu,admin", "RUST_LOG": self.log_level,
        }
        env.update(self.admission_env)
        self.procs["admission"] = Proc("admission", [binary("admission")], env, self.workdir)
        ca = os.path.join(self.cert_dir, "ca.crt")
        adm = self.procs["admission"]
        wait_for(lambda: adm.alive() and requests.get(f"https://127.0.0.1:{self.admission_port}/health", verify=ca,
                                                      timeout=1).text == "pong", 20, desc="admission /health")

    def start_controller(self, extra_env=None):
        self.controller_port = free_port()
        env = self.component_env(CONTROLLER_TOKEN, self.controller_port)
        env.update(self.controller_env)
        env.update(extra_env or {})
        self.procs["controller"] = Proc("controller", [binary("controller")], env, self.workdir)
        proc = self.procs["controller"]
        wait_for(lambda: proc.alive() and requests.get(f"http://127.0.0.1:{self.controller_port}/health",
                                                       timeout=1).text == "pong", 20, desc="controller /health")

    def start_synchronizer(self, google, interval=60, server_name="mi355x-01", extra_env=None, wait_healthy=True):
        """Start the native synchronizer against a FakeGoogle (testing/fake_google.py)."""
        key_path = os.path.join(self.workdir, "key.json")
        with open(key_path, "w") as f:
            f.write(google.service_account_json())
        self.sync_port = free_port()
        env = self.component_env(SYNC_TOKEN, self.sync_port)
        env.update({"CONF_GOOGLE_SERVICE_ACCOUNT_JSON_PATH": key_path, "CONF_GOOGLE_FILE_ID": google.file_id,
                    "CONF_SYNC_INTERVAL_SECS": str(interval), "CONF_GPU_SERVER_NAME": server_name})
        env.update(google.env())
        env.update(extra_env or {})
        p = self.start_process("synchronizer", "synchronizer", env)
        if wait_healthy:
            wait_for(lambda: p.alive() and requests.get(f"http://127.0.0.1:{self.sync_port}/health",
                                                        timeout=1).text == "pong", 20, desc="synchronizer /health")
        return p

    def start_node_agent(self, node_name="mi355x-0", max_gpus=0, backend="auto", n_mock_gpus=8, extra_env=None,
                         poll_interval_ms=1000, hive_id=None, proc_name=None, fixture_obj=None):
        """Start the native node agent; amdsmi when available, else a mock MI355X hive.
        Several agents (one per synthetic node) may run side by side: each gets its own
        fixture file (`self.fixtures[node_name]`), process name and port."""
        fixture = os.path.join(self.workdir, f"gpus-{node_name}.json")
        fx = (json.dumps(fixture_obj) if fixture_obj is not None
              else native().default_mi355x_fixture(n_mock_gpus, *([hive_id] if hive_id is not None else [])))
        with open(fixture, "w") as f:
            f.write(fx)
        self.fixtures = getattr(self, "fixtures", {})
        self.fixtures[node_name] = fixture
        port = free_port()
        self.node_agent_port = port
        self.node_agent_ports = getattr(self, "node_agent_ports", {})
        self.node_agent_ports[node_name] = port
        env = self.component_env(NODE_AGENT_TOKEN, port)
        env.update({"CONF_NODE_NAME": node_name, "CONF_GPU_BACKEND": backend, "CONF_MOCK_FIXTURE_PATH": fixture,
                    "CONF_MAX_GPUS": str(max_gpus), "CONF_CREATE_NODE": "true",
                    "CONF_POLL_INTERVAL_MS": str(poll_interval_ms)})
        env.update(extra_env or {})
        p = self.start_process(proc_name or "node-agent", "node-agent", env)
        wait_for(lambda: requests.get(f"http://127.0.0.1:{port}/health", timeout=1).text == "pong",
                 60, desc=f"node-agent {node_name} /health")
        return p

    def set_gpu_fixture(self, node_name, fixture_obj):
        """Atomically replace a mock node's GPU fixture (the agent reloads it on mtime change)."""
        path = self.fixtures[node_name]
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(fixture_obj, f)
        os.replace(tmp, path)

    def start_process(self, name, exe, env):
        # BGC_WRAP_<EXE>="tool args --" (e.g. BGC_WRAP_NODE_AGENT="rocprofv3 --marker-trace -d
        # out --"): profile one component of a running stack; the program stays right after
        # "--", as rocprofv3 requires
        wrap = os.environ.get("BGC_WRAP_" + exe.upper().replace("-", "_"), "").split()
        self.procs[name] = Proc(name, wrap + [binary(exe)], env, self.workdir)
        return self.procs[name]

    # ------------------------------------------------------------------ access
    def as_user(self, username, groups=()):
        return KubeApi(self.server, ADMIN_TOKEN, as_user=username, as_groups=list(groups), verify=self.verify)

    def fault(self, rules, append=False):
        r = requests.post(self.server + "/_kl/faults" + ("?append=true" if append else ""), json=rules, timeout=5, verify=self.verify)
        r.raise_for_status()

    def clear_faults(self):
        requests.delete(self.server + "/_kl/faults", timeout=5, verify=self.verify)

    def compact_and_drop_watches(self):
        requests.post(self.server + "/_kl/compact", timeout=5, verify=self.verify).raise_for_status()
        requests.post(self.server + "/_kl/drop-watches", timeout=5, verify=self.verify).raise_for_status()

    def stats(self):
        return requests.get(self.server + "/_kl/stats", timeout=5, verify=self.verify).json()

    def samples(self, component, name):
        port = {"apiserver": None, "controller": self.controller_port}.get(component)
        base = self.server if component == "apiserver" else f"http://127.0.0.1:{port}"
        return requests.get(f"{base}/debug/samples/{name}", timeout=5, verify=self.verify).json()

    def stop(self):
        codes = {}
        for name in reversed(list(self.procs)):
            codes[name] = self.procs[name].stop()
        if self._tmp:
            self._tmp.cleanup()
        return codes

    def logs(self):
        return {n: p.output() for n, p in self.procs.items()}

    def __enter__(self):
        try:
            return self.start()
        except Exception:
            for n, p in self.procs.items():
                print(f"--- {n} ---\n{p.output()[-4000:]}")
            self.stop()
            raise

    def __exit__(self, *exc):
        if exc[0] is not None:
            for n, p in self.procs.items():
                print(f"--- {n} log tail ---\n{p.output()[-3000:]}")
        self.stop()

"""kube-client `Client::try_default()` credential sources (reference src/controller.rs:224,
src/synchronizer.rs:392; kube-client 0.84 with the reference's features), against kube-lite
over HTTPS:

* `users[].user.exec` credential plugins (client.authentication.k8s.io v1 and v1beta1):
  KUBERNETES_EXEC_INFO, a relative command path, env, provideClusterInfo, the token cached
  until its expirationTimestamp, and a fresh credential after a 401;
* a multi-file $KUBECONFIG merged as client-go merges it (first definition wins, relative
  paths relative to the defining file);
* auth-provider oidc (the stored id-token) and gcp (access-token, then cmd-path).
"""
import json
import os
import stat
import sys
import textwrap

import pytest

from bacchus_gpu_controller_amd.testing.cluster import ADMIN_TOKEN, Cluster

pytestmark = pytest.mark.slow

PLUGIN = textwrap.dedent("""\
    #!{python}
    # fake exec credential plugin: token from a file, every call logged
    import datetime, json, os, sys
    d = os.path.dirname(os.path.abspath(__file__))
    info = json.loads(os.environ["KUBERNETES_EXEC_INFO"])
    with open(os.path.join(d, "calls.jsonl"), "a") as f:
        f.write(json.dumps({{"info": info, "args": sys.argv[1:], "env": os.environ.get("PLUGIN_MODE")}}) + "\\n")
    tokens = open(os.path.join(d, "tokens")).read().split()
    n = sum(1 for _ in open(os.path.join(d, "calls.jsonl")))
    tok = tokens[min(n, len(tokens)) - 1]
    ttl = float(os.environ.get("PLUGIN_TTL", "3600"))
    exp = (datetime.datetime.now(datetime.timezone.utc) + datetime.timedelta(seconds=ttl)).strftime("%Y-%m-%dT%H:%M:%SZ")
    print(json.dumps({{"apiVersion": info["apiVersion"], "kind": "ExecCredential",
                      "status": {{"token": tok, "expirationTimestamp": exp}}}}))
    """)


def _write(path, text, exe=False):
    with open(path, "w") as f:
        f.write(text)
    if exe:
        os.chmod(path, os.stat(path).st_mode | stat.S_IXUSR)
    return path


def _cluster_kubeconfig(c, path, user_block, ca="ca.crt"):
    d = os.path.dirname(path)
    _write(os.path.join(d, "ca.crt"), open(c.apiserver_ca).read())
    return _write(path, f"""apiVersion: v1
kind: Config
clusters:
- name: kl
  cluster:
    server: {c.server}
    certificate-authority: {ca}
users:
- name: u
  user:
{textwrap.indent(user_block, "    ")}
contexts:
- name: ctx
  context: {{cluster: kl, user: u}}
current-context: ctx
""")


def _plugin_dir(tmp_path, tokens):
    d = tmp_path / "plugin"
    d.mkdir()
    _write(str(d / "plugin.py"), PLUGIN.format(python=sys.executable), exe=True)
    _write(str(d / "tokens"), "\n".join(tokens) + "\n")
    return d


def _calls(d):
    p = d / "calls.jsonl"
    return [json.loads(l) for l in open(p)] if p.exists() else []


@pytest.mark.parametrize("api_version", ["client.authentication.k8s.io/v1", "client.authentication.k8s.io/v1beta1"])
def test_exec_plugin_authenticates_and_caches(nat, tmp_path, api_version):
    with Cluster(admission=False, controller=False, tls_apiserver=True) as c:
        pd = _plugin_dir(tmp_path, [ADMIN_TOKEN])
        kc = _cluster_kubeconfig(c, str(pd / "config"), f"""exec:
  apiVersion: {api_version}
  command: ./plugin.py
  args: [get-token, --cluster=kl]
  env: [{{name: PLUGIN_MODE, value: test}}]
  provideClusterInfo: true
  interactiveMode: Never""")
        parsed = nat.kubeconfig_parse(kc)
        assert parsed["exec"]["command"] == str(pd / "plugin.py")  # relative to the kubeconfig
        results, refreshes, source = nat.kube_request(kc, "GET", "/api/v1/namespaces", 3)
        assert [s for s, _ in results] == [200, 200, 200]
        assert refreshes == 1  # cached: the token is valid for an hour
        calls = _calls(pd)
        assert len(calls) == 1 and calls[0]["args"] == ["get-token", "--cluster=kl"] and calls[0]["env"] == "test"
        info = calls[0]["info"]
        assert info["kind"] == "ExecCredential" and info["apiVersion"] == api_version
        assert info["spec"]["interactive"] is False and info["spec"]["cluster"]["server"] == c.server
        assert "certificate-authority-data" in info["spec"]["cluster"]


def test_exec_plugin_401_refreshes_the_credential(nat, tmp_path):
    """The first credential is stale: the apiserver answers 401, the client runs the
    plugin again and retries with the new token (client-go's refresh on 401)."""
    with Cluster(admission=False, controller=False, tls_apiserver=True) as c:
        pd = _plugin_dir(tmp_path, ["revoked-token", ADMIN_TOKEN])
        kc = _cluster_kubeconfig(c, str(pd / "config"), """exec:
  apiVersion: client.authentication.k8s.io/v1
  command: ./plugin.py""")
        results, refreshes, _ = nat.kube_request(kc, "GET", "/api/v1/namespaces", 2)
        assert [s for s, _ in results] == [200, 200]
        assert refreshes == 2 and len(_calls(pd)) == 2


def test_exec_plugin_expired_token_is_refetched(nat, tmp_path, monkeypatch):
    with Cluster(admission=False, controller=False, tls_apiserver=True) as c:
        pd = _plugin_dir(tmp_path, [ADMIN_TOKEN])
        monkeypatch.setenv("PLUGIN_TTL", "5")  # expires within the client's 10 s margin
        kc = _cluster_kubeconfig(c, str(pd / "config"), """exec:
  apiVersion: client.authentication.k8s.io/v1
  command: ./plugin.py""")
        results, refreshes, _ = nat.kube_request(kc, "GET", "/api/v1/namespaces", 3)
        assert [s for s, _ in results] == [200, 200, 200]
        # one fetch when the client is built (a plugin may return a client certificate,
        # which the TLS context needs), then one per request: each found the cached token
        # inside the 10 s expiry margin
        assert refreshes == 4


def test_exec_plugin_failure_is_reported(nat, tmp_path):
    with Cluster(admission=False, controller=False, tls_apiserver=True) as c:
        d = tmp_path / "bad"
        d.mkdir()
        _write(str(d / "fail.sh"), "#!/bin/sh\necho 'login required' >&2\nexit 3\n", exe=True)
        kc = _cluster_kubeconfig(c, str(d / "config"), """exec:
  apiVersion: client.authentication.k8s.io/v1
  command: ./fail.sh""")
        with pytest.raises(Exception, match="exit 3.*login required"):
            nat.kube_request(kc, "GET", "/api/v1/namespaces", 1)


def test_multi_file_kubeconfig_merge(nat, tmp_path):
    """KUBECONFIG=a:b — the context in a names a cluster defined in b; the user in a reads
    a tokenFile relative to a, the cluster in b a CA relative to b; a later file's
    redefinition of a name is ignored."""
    with Cluster(admission=False, controller=False, tls_apiserver=True) as c:
        a, b = tmp_path / "a", tmp_path / "b"
        a.mkdir()
        b.mkdir()
        _write(str(a / "tok"), ADMIN_TOKEN + "\n")
        _write(str(b / "ca.pem"), open(c.apiserver_ca).read())
        _write(str(a / "config"), """apiVersion: v1
kind: Config
current-context: admin@kl
contexts:
- name: admin@kl
  context: {cluster: kl, user: admin}
users:
- name: admin
  user: {tokenFile: tok}
""")
        _write(str(b / "config"), f"""apiVersion: v1
kind: Config
current-context: other
clusters:
- name: kl
  cluster: {{server: "{c.server}", certificate-authority: ca.pem}}
users:
- name: admin
  user: {{token: wrong-token}}
contexts:
- name: other
  context: {{cluster: kl, user: admin}}
""")
        results, _, source = nat.kube_request(f"{a}/config:{tmp_path}/missing:{b}/config", "GET", "/api/v1/namespaces", 1)
        assert results[0][0] == 200
        assert source == f"kubeconfig:{a}/config:{b}/config"


def test_auth_provider_oidc_and_gcp(nat, tmp_path):
    with Cluster(admission=False, controller=False, tls_apiserver=True) as c:
        d = tmp_path / "ap"
        d.mkdir()
        kc = _cluster_kubeconfig(c, str(d / "oidc"), f"""auth-provider:
  name: oidc
  config: {{client-id: kubernetes, id-token: "{ADMIN_TOKEN}", idp-issuer-url: "https://idp.example"}}""")
        assert nat.kube_request(kc, "GET", "/api/v1/namespaces", 1)[0][0][0] == 200
        # gcp: the cached access-token has expired, so cmd-path runs and token-key picks the token
        _write(str(d / "gcloud.sh"), "#!/bin/sh\necho '{\"credential\": {\"access_token\": \"" + ADMIN_TOKEN +
               "\", \"token_expiry\": \"2099-01-01T00:00:00Z\"}}'\n", exe=True)
        kc = _cluster_kubeconfig(c, str(d / "gcp"), f"""auth-provider:
  name: gcp
  config:
    access-token: stale
    expiry: "2000-01-01T00:00:00Z"
    cmd-path: {d}/gcloud.sh
    cmd-args: config config-helper --format=json
    token-key: "{{.credential.access_token}}"
    expiry-key: "{{.credential.token_expiry}}\"""")
        results, refreshes, _ = nat.kube_request(kc, "GET", "/api/v1/namespaces", 2)
        assert [s for s, _ in results] == [200, 200] and refreshes == 1


def test_controller_binary_runs_on_an_exec_plugin_kubeconfig(tmp_path):
    """End to end: the controller authenticates through an exec plugin and reconciles."""
    from bacchus_gpu_controller_amd.testing.cluster import CONTROLLER_TOKEN
    from bacchus_gpu_controller_amd.testing.kubeapi import wait_for

    with Cluster(admission=False, controller=False, tls_apiserver=True) as c:
        pd = _plugin_dir(tmp_path, [CONTROLLER_TOKEN])
        kc = _cluster_kubeconfig(c, str(pd / "config"), """exec:
  apiVersion: client.authentication.k8s.io/v1beta1
  command: ./plugin.py""")
        c.start_controller(extra_env={"KUBECONFIG": kc})
        c.admin.create("userbootstraps", {"apiVersion": "bacchus.io/v1", "kind": "UserBootstrap",
                                          "metadata": {"name": "exec-user"}, "spec": {"kube_username": "exec-user"}})
        wait_for(lambda: c.admin.get_or_none("namespaces", "exec-user"), timeout=15, desc="namespace via exec creds")
        assert _calls(pd)  # the plugin really ran


def test_exec_plugin_install_hint_and_interactive_mode(nat, tmp_path):
    """client-go parity: a missing command reports the kubeconfig's installHint, and a
    plugin that insists on a terminal (interactiveMode: Always) is refused, since the
    services never have one."""
    with Cluster(admission=False, controller=False, tls_apiserver=True) as c:
        d = tmp_path / "hint"
        d.mkdir()
        kc = _cluster_kubeconfig(c, str(d / "missing"), """exec:
  apiVersion: client.authentication.k8s.io/v1
  command: bgc-no-such-credential-helper
  installHint: "install it with: apt install bgc-credential-helper\"""")
        assert nat.kubeconfig_parse(kc)["exec"]["install_hint"].startswith("install it with")
        with pytest.raises(Exception, match="(?s)cannot run.*install it with: apt install"):
            nat.kube_request(kc, "GET", "/api/v1/namespaces", 1)
        pd = _plugin_dir(tmp_path, [ADMIN_TOKEN])
        kc = _cluster_kubeconfig(c, str(pd / "config"), """exec:
  apiVersion: client.authentication.k8s.io/v1
  command: ./plugin.py
  interactiveMode: Always""")
        with pytest.raises(Exception, match="interactive mode"):
            nat.kube_request(kc, "GET", "/api/v1/namespaces", 1)
        assert not _calls(pd)  # refused before running it


CERT_PLUGIN = textwrap.dedent("""\
    #!{python}
    # fake exec plugin that hands out client certificates: the n-th call returns cert<n>
    # (the last one from then on), each valid for PLUGIN_TTL seconds
    import datetime, json, os
    d = os.path.dirname(os.path.abspath(__file__))
    info = json.loads(os.environ["KUBERNETES_EXEC_INFO"])
    with open(os.path.join(d, "calls.jsonl"), "a") as f:
        f.write("{{}}\\n")
    n = sum(1 for _ in open(os.path.join(d, "calls.jsonl")))
    k = min(n, int(open(os.path.join(d, "count")).read()))
    exp = (datetime.datetime.now(datetime.timezone.utc)
           + datetime.timedelta(seconds=float(os.environ.get("PLUGIN_TTL", "3600")))).strftime("%Y-%m-%dT%H:%M:%SZ")
    print(json.dumps({{"apiVersion": info["apiVersion"], "kind": "ExecCredential",
                      "status": {{"clientCertificateData": open(os.path.join(d, f"cert{{k}}.pem")).read(),
                                  "clientKeyData": open(os.path.join(d, f"key{{k}}.pem")).read(),
                                  "expirationTimestamp": exp}}}}))
    """)


def _openssl(*args, cwd):
    import subprocess

    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True)


def _client_pki(d, users):
    """A client CA (the apiserver's --client-ca-file) and one certificate per (CN, O)."""
    _openssl("req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:P-256", "-nodes", "-keyout", "ca.key",
             "-out", "ca.crt", "-days", "1", "-subj", "/CN=bgc-test-client-ca", cwd=d)
    for i, (cn, org) in enumerate(users, 1):
        _openssl("req", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:P-256", "-nodes", "-keyout", f"key{i}.pem",
                 "-out", f"c{i}.csr", "-subj", f"/O={org}/CN={cn}", cwd=d)
        _openssl("x509", "-req", "-in", f"c{i}.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial",
                 "-out", f"cert{i}.pem", "-days", "1", cwd=d)
    _write(os.path.join(d, "count"), str(len(users)))
    return os.path.join(d, "ca.crt")


def test_exec_plugin_client_certificate_rotation(nat, tmp_path, monkeypatch):
    """An exec plugin that issues short-lived client certificates: when a
    refresh returns a new certificate, the client rebuilds its TLS context, so the next
    requests present the new certificate instead of failing on the expired one.  kube-lite
    authenticates x509 client certificates (--client-ca-file: CN = user, O = groups) and
    answers SelfSubjectReview, which shows which certificate each request carried."""
    d = tmp_path / "certplugin"
    d.mkdir()
    ca = _client_pki(str(d), [("cert-admin-a", "system:masters"), ("cert-admin-b", "system:masters")])
    with Cluster(admission=False, controller=False, tls_apiserver=True,
                 apiserver_args=["--client-ca-file", ca]) as c:
        _write(str(d / "plugin.py"), CERT_PLUGIN.format(python=sys.executable), exe=True)
        kc = _cluster_kubeconfig(c, str(d / "config"), """exec:
  apiVersion: client.authentication.k8s.io/v1
  command: ./plugin.py""")
        review = "/apis/authentication.k8s.io/v1/selfsubjectreviews"
        # a long-lived certificate: fetched once, then cached
        results, refreshes, _ = nat.kube_request(kc, "POST", review, 2)
        users = [json.loads(b)["status"]["userInfo"]["username"] for _, b in results]
        assert [s for s, _ in results] == [201, 201] and users == ["cert-admin-a"] * 2 and refreshes == 1
        assert "system:masters" in json.loads(results[0][1])["status"]["userInfo"]["groups"]
        # certificates that expire within the client's 10 s margin: every request refreshes,
        # the second fetch hands out certificate b, and the requests carry b from then on
        os.unlink(d / "calls.jsonl")
        monkeypatch.setenv("PLUGIN_TTL", "5")
        results, refreshes, _ = nat.kube_request(kc, "POST", review, 3)
        users = [json.loads(b)["status"]["userInfo"]["username"] for _, b in results]
        assert [s for s, _ in results] == [201] * 3 and users == ["cert-admin-b"] * 3, users
        assert refreshes == 4
        # the cert user is an admin like any other: it can list
        results, _, _ = nat.kube_request(kc, "GET", "/api/v1/namespaces", 1)
        assert results[0][0] == 200

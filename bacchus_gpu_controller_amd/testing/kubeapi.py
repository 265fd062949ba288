"""Tiny Kubernetes REST client for tests and the bench harness (plain requests).

Only what the tests need: typed paths, CRUD, JSON/merge patch, server-side apply,
impersonation headers and polling helpers.  The production clients are native C++
(native/kube/client.cc); this one exists so tests can act as kubectl would.
"""
import json
import time

import requests

RESOURCES = {
    # plural: (group, version, namespaced)
    "namespaces": ("", "v1", False),
    "resourcequotas": ("", "v1", True),
    "nodes": ("", "v1", False),
    "pods": ("", "v1", True),
    "configmaps": ("", "v1", True),
    "leases": ("coordination.k8s.io", "v1", True),
    "secrets": ("", "v1", True),
    "serviceaccounts": ("", "v1", True),
    "events": ("", "v1", True),
    "roles": ("rbac.authorization.k8s.io", "v1", True),
    "rolebindings": ("rbac.authorization.k8s.io", "v1", True),
    "clusterroles": ("rbac.authorization.k8s.io", "v1", False),
    "clusterrolebindings": ("rbac.authorization.k8s.io", "v1", False),
    "userbootstraps": ("bacchus.io", "v1", False),
    "customresourcedefinitions": ("apiextensions.k8s.io", "v1", False),
    "mutatingwebhookconfigurations": ("admissionregistration.k8s.io", "v1", False),
}


class ApiError(Exception):
    def __init__(self, code, body):
        self.code = code
        self.body = body
        try:
            self.status = json.loads(body)
        except ValueError:
            self.status = {"message": body}
        super().__init__(f"{code}: {self.status.get('message', body)}")

    @property
    def message(self):
        return self.status.get("message", "")

    @property
    def reason(self):
        return self.status.get("reason", "")


def path_for(plural, name=None, namespace=None, sub=None):
    group, version, namespaced = RESOURCES[plural]
    base = f"/api/{version}" if not group else f"/apis/{group}/{version}"
    if namespaced and namespace:
        base += f"/namespaces/{namespace}"
    base += f"/{plural}"
    if name:
        base += f"/{name}"
    if sub:
        base += f"/{sub}"
    return base


class KubeApi:
    def __init__(self, server, token=None, as_user=None, as_groups=None, timeout=15, verify=True):
        self.server = server.rstrip("/")
        self.s = requests.Session()
        self.s.verify = verify  # CA bundle path for an HTTPS apiserver
        self.timeout = timeout
        if token:
            self.s.headers["Authorization"] = f"Bearer {token}"
        self.s.headers["Accept"] = "application/json"
        self._imp = []
        if as_user:
            self._imp.append(("Impersonate-User", as_user))
            for g in as_groups or []:
                self._imp.append(("Impersonate-Group", g))

    def _req(self, method, path, body=None, ctype="application/json", params=None):
        headers = {"Content-Type": ctype} if body is not None else {}
        # requests can't repeat a header name via dict; build a list of tuples
        hdrs = list(headers.items()) + self._imp
        data = body if isinstance(body, (str, bytes)) or body is None else json.dumps(body)
        prepared = requests.Request(method, self.server + path, data=data, params=params).prepare()
        for k, v in self.s.headers.items():
            prepared.headers.setdefault(k, v)
        # multi-valued Impersonate-Group: comma-join is NOT equivalent, so send one per header
        # by using the raw http.client path through requests' underlying adapter.
        for k, v in hdrs:
            if k in prepared.headers and k == "Impersonate-Group":
                prepared.headers[k] = prepared.headers[k] + "," + v
            else:
                prepared.headers[k] = v
        r = self.s.send(prepared, timeout=self.timeout)
        if r.status_code >= 300:
            raise ApiError(r.status_code, r.text)
        return r.json() if r.text else None

    # -- verbs --
    def get(self, plural, name, namespace=None):
        return self._req("GET", path_for(plural, name, namespace))

    def get_or_none(self, plural, name, namespace=None):
        try:
            return self.get(plural, name, namespace)
        except ApiError as e:
            if e.code == 404:
                return None
            raise

    def list(self, plural, namespace=None, label_selector=None, field_selector=None):
        params = {k: v for k, v in (("labelSelector", label_selector), ("fieldSelector", field_selector)) if v} or None
        return self._req("GET", path_for(plural, None, namespace), params=params)

    def create(self, plural, obj, namespace=None, field_manager=None):
        params = {"fieldManager": field_manager} if field_manager else None
        return self._req("POST", path_for(plural, None, namespace), obj, params=params)

    def replace(self, plural, name, obj, namespace=None, sub=None):
        return self._req("PUT", path_for(plural, name, namespace, sub), obj)

    def json_patch(self, plural, name, ops, namespace=None, sub=None):
        return self._req("PATCH", path_for(plural, name, namespace, sub), ops, "application/json-patch+json")

    def merge_patch(self, plural, name, patch, namespace=None, sub=None, field_manager=None):
        params = {"fieldManager": field_manager} if field_manager else None
        return self._req("PATCH", path_for(plural, name, namespace, sub), patch, "application/merge-patch+json",
                         params=params)

    def apply(self, plural, name, obj, manager, force=False, namespace=None, sub=None):
        params = {"fieldManager": manager}
        if force:
            params["force"] = "true"
        return self._req("PATCH", path_for(plural, name, namespace, sub), obj, "application/apply-patch+yaml",
                         params=params)

    def delete(self, plural, name, namespace=None):
        return self._req("DELETE", path_for(plural, name, namespace))

    def raw(self, method, path, body=None, ctype="application/json"):
        return self._req(method, path, body, ctype)


def wait_for(fn, timeout=10.0, interval=0.02, desc="condition"):
    deadline = time.time() + timeout
    last = None
    while time.time() < deadline:
        try:
            last = fn()
            if last:
                return last
        except (ApiError, requests.RequestException, OSError, KeyError) as e:
            last = e
        time.sleep(interval)
    raise AssertionError(f"timed out waiting for {desc}; last={last!r}")

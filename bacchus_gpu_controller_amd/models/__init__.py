"""UserBootstrap data model (reference src/crd.rs:9-42) as plain-dict builders.

The authoritative schema is generated natively (native/crd/schema.cc, `crdgen`);
these helpers build objects that conform to it, for tests, the bench and operators'
scripts.
"""
import json

from .. import native

GROUP = "bacchus.io"
VERSION = "v1"
API_VERSION = f"{GROUP}/{VERSION}"
KIND = "UserBootstrap"
PLURAL = "userbootstraps"


def user_bootstrap(name, kube_username=None, quota=None, role=None, rolebinding=None, status=None):
    spec = {}
    if kube_username is not None:
        spec["kube_username"] = kube_username
    if quota is not None:
        spec["quota"] = quota
    if role is not None:
        spec["role"] = role
    if rolebinding is not None:
        spec["rolebinding"] = rolebinding
    obj = {"apiVersion": API_VERSION, "kind": KIND, "metadata": {"name": name}, "spec": spec}
    if status is not None:
        obj["status"] = status
    return obj


def rolebinding(role_name, subjects, kind="ClusterRole"):
    """RoleBinding without metadata (crd.rs:37-42): {role_ref, subjects}."""
    return {"role_ref": {"apiGroup": "rbac.authorization.k8s.io", "kind": kind, "name": role_name},
            "subjects": [{"apiGroup": "rbac.authorization.k8s.io", "kind": "User", "name": s} for s in subjects]}


def gpu_quota(gpus, cpu, memory_gi, storage_gi, partitions=0, gpu_resource="amd.com/gpu",
              partition_resource="amd.com/gpu-partition"):
    """The synchronizer's quota mapping (native sync/sheet.cc) as a ResourceQuotaSpec."""
    row = {"gpu_request": gpus, "cpu_request": cpu, "memory_request": memory_gi, "storage_request": storage_gi,
           "mig_request": partitions}
    return json.loads(native().quota_spec(row, gpu_resource, partition_resource))


def schema():
    return json.loads(native().ub_schema_json())


def crd():
    return json.loads(native().crd_json())


def validate(obj):
    """Structural-schema errors as (path, kind, detail) tuples; [] when valid."""
    return native().validate_ub(json.dumps(obj))

#include "kube/resource.h"

#include "core/http.h"

namespace bgc::kube {

std::string ResourceType::collection_path(const std::string& ns) const {
  if (namespaced && !ns.empty()) return prefix() + "/namespaces/" + http::url_encode(ns) + "/" + plural;
  return prefix() + "/" + plural;
}

std::string ResourceType::object_path(const std::string& ns, const std::string& name) const {
  return collection_path(namespaced ? ns : "") + "/" + http::url_encode(name);
}

std::string object_key(const ResourceType& rt, const std::string& ns, const std::string& name) {
  return rt.key(ns, name);
}

namespace types {
// group, version, kind, plural, namespaced, has_status
const ResourceType Namespace{"", "v1", "Namespace", "namespaces", false, true};
const ResourceType ResourceQuota{"", "v1", "ResourceQuota", "resourcequotas", true, true};
const ResourceType Role{"rbac.authorization.k8s.io", "v1", "Role", "roles", true, false};
const ResourceType RoleBinding{"rbac.authorization.k8s.io", "v1", "RoleBinding", "rolebindings", true, false};
const ResourceType ClusterRole{"rbac.authorization.k8s.io", "v1", "ClusterRole", "clusterroles", false, false};
const ResourceType ClusterRoleBinding{"rbac.authorization.k8s.io", "v1", "ClusterRoleBinding", "clusterrolebindings", false, false};
const ResourceType UserBootstrap{"bacchus.io", "v1", "UserBootstrap", "userbootstraps", false, true};
const ResourceType Node{"", "v1", "Node", "nodes", false, true};
const ResourceType Pod{"", "v1", "Pod", "pods", true, true};
const ResourceType Lease{"coordination.k8s.io", "v1", "Lease", "leases", true, false};
const ResourceType ConfigMap{"", "v1", "ConfigMap", "configmaps", true, false};
const ResourceType Secret{"", "v1", "Secret", "secrets", true, false};
const ResourceType ServiceAccount{"", "v1", "ServiceAccount", "serviceaccounts", true, false};
const ResourceType Event{"", "v1", "Event", "events", true, false};
const ResourceType CustomResourceDefinition{"apiextensions.k8s.io", "v1", "CustomResourceDefinition",
                                            "customresourcedefinitions", false, true};
const ResourceType MutatingWebhookConfiguration{"admissionregistration.k8s.io", "v1", "MutatingWebhookConfiguration",
                                                "mutatingwebhookconfigurations", false, false};

const std::vector<const ResourceType*>& builtin() {
  static const std::vector<const ResourceType*> all = {
      &Namespace, &ResourceQuota, &Role, &RoleBinding, &ClusterRole, &ClusterRoleBinding, &Node, &Pod, &Lease,
      &ConfigMap, &Secret, &ServiceAccount, &Event, &CustomResourceDefinition, &MutatingWebhookConfiguration};
  return all;
}
}  // namespace types

}  // namespace bgc::kube

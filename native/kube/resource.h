// Kubernetes resource type descriptors and REST paths.
#pragma once

#include <string>
#include <vector>

namespace bgc::kube {

struct ResourceType {
  std::string group;    // "" for core
  std::string version;  // "v1"
  std::string kind;     // "Namespace"
  std::string plural;   // "namespaces"
  bool namespaced = false;
  bool has_status = false;

  std::string api_version() const { return group.empty() ? version : group + "/" + version; }
  std::string prefix() const { return group.empty() ? "/api/" + version : "/apis/" + group + "/" + version; }
  // Collection path; ns empty => all namespaces (for namespaced types).
  std::string collection_path(const std::string& ns = "") const;
  std::string object_path(const std::string& ns, const std::string& name) const;
  std::string key(const std::string& ns, const std::string& name) const { return namespaced ? ns + "/" + name : name; }
};

namespace types {
extern const ResourceType Namespace;
extern const ResourceType ResourceQuota;
extern const ResourceType Role;
extern const ResourceType RoleBinding;
extern const ResourceType ClusterRole;
extern const ResourceType ClusterRoleBinding;
extern const ResourceType UserBootstrap;
extern const ResourceType Node;
extern const ResourceType Pod;
extern const ResourceType Lease;
extern const ResourceType ConfigMap;
extern const ResourceType Secret;
extern const ResourceType ServiceAccount;
extern const ResourceType Event;
extern const ResourceType CustomResourceDefinition;
extern const ResourceType MutatingWebhookConfiguration;
const std::vector<const ResourceType*>& builtin();
}  // namespace types

// Object key helpers ("ns/name" or "name").
std::string object_key(const ResourceType& rt, const std::string& ns, const std::string& name);

}  // namespace bgc::kube

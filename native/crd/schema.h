// UserBootstrap CRD model, OpenAPI v3 schema generation and structural validation.
//
// Reference: src/crd.rs:9-42 (types + kube derive attributes) and src/crdgen.rs:3-8
// (serde_yaml of `UserBootstrap::crd()`).  The schema is generated the way
// kube-derive + schemars do it: the UserBootstrap Rust types are modelled here, the
// embedded k8s-openapi type schemas (k8s_openapi_defs.cc) are inlined, `Option<T>`
// becomes `nullable: true`, field doc comments override type descriptions, and every
// map is emitted with sorted keys (k8s-openapi JSONSchemaProps / BTreeMap order).
#pragma once

#include <string>
#include <vector>

#include "core/json.h"

namespace bgc::crd {

extern const char* const kK8sOpenApiDefs;

constexpr const char* kGroup = "bacchus.io";
constexpr const char* kVersion = "v1";
constexpr const char* kApiVersion = "bacchus.io/v1";
constexpr const char* kKind = "UserBootstrap";
constexpr const char* kPlural = "userbootstraps";
constexpr const char* kSingular = "userbootstrap";
constexpr const char* kShortName = "ub";

const json::Value& k8s_definitions();
// Resolves `$ref`s against k8s_definitions(); sibling keys override the target's.
json::Value inline_refs(const json::Value& schema);
// Inlined schema of one k8s type (e.g. "Subject", "RoleRef", "ResourceQuotaSpec").
json::Value k8s_type_schema(const std::string& name);

const json::Value& userbootstrap_schema();  // openAPIV3Schema
json::Value userbootstrap_crd();            // CustomResourceDefinition object
std::string crd_yaml();                     // == reference crdgen output

// ---------------------------------------------------------------------------
// Structural validation.
struct ValidationError {
  std::string path;    // e.g. "spec.kube_username"
  std::string kind;    // "type" | "required" | "format" | "null"
  std::string detail;  // human readable
};

struct ValidateOptions {
  // serde semantics (k8s-openapi Deserialize): `metadata` of embedded objects defaults
  // instead of being required, as in `unwrap_or_default()`.
  bool serde = false;
};

std::vector<ValidationError> validate(const json::Value& value, const json::Value& schema,
                                      const ValidateOptions& opts = {});

// serde_json-style message for the first error, e.g.
//   "invalid type: integer `5`, expected a string at spec.kube_username"
std::string serde_error_message(const json::Value& value, const ValidationError& e);

// Typed view of a (parsed) UserBootstrap.  Parsing mirrors `DynamicObject::try_parse`
// (reference src/admission.rs:341-347): structural type errors are reported, unknown
// fields are ignored.
struct RoleBindingSpec {
  json::Value role_ref;  // {apiGroup, kind, name}
  json::Value subjects;  // null or array
};

struct UserBootstrap {
  json::Value raw;  // original object
  std::string name;
  std::string uid;
  std::string resource_version;
  bool has_kube_username = false;
  std::string kube_username;
  bool has_quota = false;
  json::Value quota;  // ResourceQuotaSpec
  bool has_role = false;
  json::Value role;
  bool has_rolebinding = false;
  RoleBindingSpec rolebinding;
  bool has_status = false;
  bool synchronized_with_sheet = false;
};

// Throws std::runtime_error with a serde-style message on type errors.
UserBootstrap parse_userbootstrap(const json::Value& obj);

// The same validation as parse_userbootstrap, returning only which spec fields are set (no
// copies): what the admission policy needs on every review.  Pointers alias `obj`.
struct UserBootstrapShape {
  const std::string* kube_username = nullptr;  // null when absent or null
  bool has_quota = false;
  bool has_role = false;
  bool has_rolebinding = false;
};
UserBootstrapShape inspect_userbootstrap(const json::Value& obj);

bool is_rfc3339(const std::string& s);

}  // namespace bgc::crd

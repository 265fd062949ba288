// Field sets for server-side apply (SSA-lite): leaf paths of an object, with the
// associative-list rules Kubernetes uses for metadata (ownerReferences keyed by uid,
// finalizers as a set); every other list is atomic.
//
// Path syntax: RFC 6901 tokens joined by '/', with keyed list items as "[uid=<v>]" and
// set items as "[=<json value>]".
#pragma once

#include <map>
#include <set>
#include <string>
#include <vector>

#include "core/json.h"

namespace bgc::apiserver {

using FieldSet = std::set<std::string>;

// Leaves of `obj` (ignoring apiVersion/kind/metadata.{name,namespace,resourceVersion,
// uid,generation,creationTimestamp,managedFields} and status unless include_status).
FieldSet leaves(const json::Value& obj, bool include_status = false);
const json::Value* get_path(const json::Value& root, const std::string& path);
bool remove_path(json::Value& root, const std::string& path);
void set_path(json::Value& root, const std::string& path, const json::Value& v);
// Leaves whose value differs between `before` and `after` (added or changed), and
// those removed.
void diff_leaves(const json::Value& before, const json::Value& after, FieldSet& changed, FieldSet& removed,
                 bool include_status = false);
// diff_leaves restricted to the top-level member `key` (paths keep their "/key" prefix),
// for writes that can change nothing else, such as a status subresource write.
void diff_member_leaves(const json::Value& before, const json::Value& after, const std::string& key,
                        FieldSet& changed, FieldSet& removed);
// Human-readable ".spec.hard.cpu" form for conflict messages.
std::string display_path(const std::string& path);
// metadata.managedFields[].fieldsV1 rendering of a set.
json::Value fields_v1(const FieldSet& fs);

}  // namespace bgc::apiserver

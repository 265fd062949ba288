// YAML support.
//
// * `emit` reproduces the exact block style that serde_yaml 0.9 (libyaml emitter,
//   unlimited line width, unicode on) produces, because `crdgen` must print the CRD
//   byte-for-byte like the reference (reference src/crdgen.rs:3-8, output checked in
//   at charts/bacchus-gpu-controller/templates/crd.yaml).
// * `parse` is a pragmatic YAML 1.2 subset reader (block/flow collections, all scalar
//   styles, comments, multi-document) used for kubeconfig files and manifests.
#pragma once

#include <string>
#include <vector>

#include "core/json.h"

namespace bgc::yaml {

class Error : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// Emits one YAML document (no leading `---`), serde_yaml::to_string style.
std::string emit(const json::Value& v);

// Parses the first document.
json::Value parse(const std::string& text);
// Parses every document in a stream (empty documents skipped).
std::vector<json::Value> parse_all(const std::string& text);

}  // namespace bgc::yaml

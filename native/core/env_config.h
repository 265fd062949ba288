// envy-compatible configuration: every field `foo_bar` is read from `CONF_FOO_BAR`
// (reference: `envy::prefixed("CONF_")` in src/controller.rs:220,
// src/admission.rs:138, src/synchronizer.rs:386). A missing required field or an
// unparsable number aborts startup with an error naming the field.
#pragma once

#include <cstdint>
#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

namespace bgc {

class ConfigError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class EnvConfig {
 public:
  explicit EnvConfig(std::string prefix = "CONF_");
  // Snapshot from a map instead of the process environment (tests/bindings).
  EnvConfig(std::string prefix, std::map<std::string, std::string> env);

  std::string str(const std::string& field) const;  // required
  std::string str_or(const std::string& field, const std::string& dflt) const;
  uint16_t u16(const std::string& field) const;
  uint64_t u64(const std::string& field) const;
  uint64_t u64_or(const std::string& field, uint64_t dflt) const;
  double f64_or(const std::string& field, double dflt) const;
  bool boolean_or(const std::string& field, bool dflt) const;
  // Comma-separated list; NO trimming, so "" -> [""] (reference
  // src/admission.rs:41-50 comma_separated_deserialize).
  std::vector<std::string> comma_list(const std::string& field) const;
  std::optional<std::string> raw(const std::string& field) const;

  static std::string env_name(const std::string& prefix, const std::string& field);

 private:
  std::string prefix_;
  std::optional<std::map<std::string, std::string>> env_;
};

std::vector<std::string> split_comma(const std::string& s);

}  // namespace bgc

#include "core/env_config.h"

#include <cctype>
#include <charconv>
#include <cstdlib>

namespace bgc {

EnvConfig::EnvConfig(std::string prefix) : prefix_(std::move(prefix)) {}
EnvConfig::EnvConfig(std::string prefix, std::map<std::string, std::string> env)
    : prefix_(std::move(prefix)), env_(std::move(env)) {}

std::string EnvConfig::env_name(const std::string& prefix, const std::string& field) {
  std::string out = prefix;
  for (char c : field) out.push_back(static_cast<char>(std::toupper(static_cast<unsigned char>(c))));
  return out;
}

std::optional<std::string> EnvConfig::raw(const std::string& field) const {
  std::string name = env_name(prefix_, field);
  if (env_) {
    auto it = env_->find(name);
    if (it == env_->end()) return std::nullopt;
    return it->second;
  }
  const char* v = std::getenv(name.c_str());
  if (!v) return std::nullopt;
  return std::string(v);
}

std::string EnvConfig::str(const std::string& field) const {
  auto v = raw(field);
  if (!v) throw ConfigError("missing value for field " + field);
  return *v;
}

std::string EnvConfig::str_or(const std::string& field, const std::string& dflt) const {
  auto v = raw(field);
  return v ? *v : dflt;
}

template <typename T>
static T parse_unsigned(const std::string& field, const std::string& s) {
  T v{};
  auto r = std::from_chars(s.data(), s.data() + s.size(), v);
  if (s.empty() || r.ec != std::errc() || r.ptr != s.data() + s.size()) {
    throw ConfigError("invalid value for field " + field + ": \"" + s + "\"");
  }
  return v;
}

uint16_t EnvConfig::u16(const std::string& field) const { return parse_unsigned<uint16_t>(field, str(field)); }
uint64_t EnvConfig::u64(const std::string& field) const { return parse_unsigned<uint64_t>(field, str(field)); }

uint64_t EnvConfig::u64_or(const std::string& field, uint64_t dflt) const {
  auto v = raw(field);
  return v ? parse_unsigned<uint64_t>(field, *v) : dflt;
}

double EnvConfig::f64_or(const std::string& field, double dflt) const {
  auto v = raw(field);
  if (!v) return dflt;
  char* end = nullptr;
  double d = std::strtod(v->c_str(), &end);
  if (v->empty() || end != v->c_str() + v->size()) {
    throw ConfigError("invalid value for field " + field + ": \"" + *v + "\"");
  }
  return d;
}

bool EnvConfig::boolean_or(const std::string& field, bool dflt) const {
  auto v = raw(field);
  if (!v) return dflt;
  if (*v == "true" || *v == "1") return true;
  if (*v == "false" || *v == "0") return false;
  throw ConfigError("invalid value for field " + field + ": \"" + *v + "\"");
}

std::vector<std::string> split_comma(const std::string& s) {
  std::vector<std::string> out;
  size_t start = 0;
  while (true) {
    size_t c = s.find(',', start);
    out.push_back(s.substr(start, c == std::string::npos ? std::string::npos : c - start));
    if (c == std::string::npos) break;
    start = c + 1;
  }
  return out;
}

std::vector<std::string> EnvConfig::comma_list(const std::string& field) const {
  return split_comma(str(field));
}

}  // namespace bgc

// Kubernetes resource quantities (k8s.io/apimachinery/pkg/api/resource): the apiserver
// stores a quantity in canonical form ("1000m" comes back as "1", "1024Mi" as "1Gi"), so
// comparing what the controller applied with what the server holds needs their values.
#pragma once

#include <optional>
#include <string>
#include <string_view>

namespace bgc::kube {

// Value of a quantity string: <signed decimal number><suffix>, the suffix one of the binary
// SI (Ki Mi Gi Ti Pi Ei), the decimal SI (n u m "" k M G T P E) or a decimal exponent
// (e3, E-2).  nullopt when `s` is not a quantity.
std::optional<long double> parse_quantity(std::string_view s);
// Both parse and have the same value (relative tolerance 1e-12).
bool same_quantity(std::string_view a, std::string_view b);
// The form the apiserver stores and returns (apimachinery Quantity.String /
// CanonicalizeBytes): the value rounded up to 1n, written with the suffix family it was
// given in (binary SI below 1Ki, or not a whole number, falls back to decimal SI), the
// mantissa the smallest integer, the decimal exponent a multiple of 3: "1000m" -> "1",
// "0.5" -> "500m", "2000" -> "2k", "1024Mi" -> "1Gi", "0.5Ki" -> "512", "1.5e3" -> "1500".
// nullopt when `s` is not a quantity or its value is out of this implementation's range.
std::optional<std::string> canonical_quantity(std::string_view s);

}  // namespace bgc::kube

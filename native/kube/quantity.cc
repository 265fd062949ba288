#include "kube/quantity.h"

#include <algorithm>
#include <cctype>
#include <cmath>

namespace bgc::kube {

std::optional<long double> parse_quantity(std::string_view s) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  long double v = 0;
  size_t digits = 0;
  while (i < s.size() && std::isdigit(static_cast<unsigned char>(s[i]))) {
    v = v * 10 + (s[i++] - '0');
    ++digits;
  }
  if (i < s.size() && s[i] == '.') {
    ++i;
    long double scale = 0.1L;
    while (i < s.size() && std::isdigit(static_cast<unsigned char>(s[i]))) {
      v += (s[i++] - '0') * scale;
      scale /= 10;
      ++digits;
    }
  }
  if (digits == 0) return std::nullopt;
  const std::string_view suffix = s.substr(i);
  long double mult = 1;
  if (suffix.empty()) {
  } else if (suffix.size() == 2 && suffix[1] == 'i') {
    static constexpr char kBin[] = "KMGTPE";
    const char* p = nullptr;
    for (const char* c = kBin; *c; ++c)
      if (*c == suffix[0]) p = c;
    if (!p) return std::nullopt;
    mult = std::pow(1024.0L, static_cast<long double>(p - kBin + 1));
  } else if ((suffix[0] == 'e' || suffix[0] == 'E') && suffix.size() > 1) {  // "1E" alone is exa
    size_t j = 1;
    bool eneg = false;
    if (j < suffix.size() && (suffix[j] == '+' || suffix[j] == '-')) eneg = suffix[j++] == '-';
    if (j == suffix.size()) return std::nullopt;
    int e = 0;
    for (; j < suffix.size(); ++j) {
      if (!std::isdigit(static_cast<unsigned char>(suffix[j])) || e > 100) return std::nullopt;
      e = e * 10 + (suffix[j] - '0');
    }
    mult = std::pow(10.0L, static_cast<long double>(eneg ? -e : e));
  } else if (suffix.size() == 1) {
    switch (suffix[0]) {
      case 'n': mult = 1e-9L; break;
      case 'u': mult = 1e-6L; break;
      case 'm': mult = 1e-3L; break;
      case 'k': mult = 1e3L; break;
      case 'M': mult = 1e6L; break;
      case 'G': mult = 1e9L; break;
      case 'T': mult = 1e12L; break;
      case 'P': mult = 1e15L; break;
      case 'E': mult = 1e18L; break;
      default: return std::nullopt;
    }
  } else {
    return std::nullopt;
  }
  v *= mult;
  return neg ? -v : v;
}

bool same_quantity(std::string_view a, std::string_view b) {
  const auto x = parse_quantity(a), y = parse_quantity(b);
  if (!x || !y) return false;
  const long double scale = std::max<long double>(1.0L, std::max(std::fabs(*x), std::fabs(*y)));
  return std::fabs(*x - *y) <= 1e-12L * scale;
}

}  // namespace bgc::kube

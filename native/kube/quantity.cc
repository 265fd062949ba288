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

namespace {

using i128 = __int128;
constexpr i128 kNano = 1000000000;
constexpr int kMaxDigits = 36;  // 10^36 < 2^120: every product below stays in range

enum class Format { BinarySI, DecimalSI, DecimalExponent };

i128 pow10(int n) {
  i128 v = 1;
  while (n-- > 0) v *= 10;
  return v;
}

std::string to_string(i128 v) {
  if (v == 0) return "0";
  std::string out;
  for (; v > 0; v /= 10) out.push_back(static_cast<char>('0' + static_cast<int>(v % 10)));
  std::reverse(out.begin(), out.end());
  return out;
}

int digit_count(i128 v) {
  int n = 0;
  for (; v > 0; v /= 10) ++n;
  return n;
}

}  // namespace

std::optional<std::string> canonical_quantity(std::string_view s) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  i128 mant = 0;
  int frac = 0, digits = 0;
  bool sticky = false;  // a non-zero fraction digit past the kept precision
  bool any = false;
  for (bool in_frac = false; i < s.size(); ++i) {
    if (s[i] == '.' && !in_frac) {
      in_frac = true;
      continue;
    }
    if (!std::isdigit(static_cast<unsigned char>(s[i]))) break;
    any = true;
    const int d = s[i] - '0';
    if (mant == 0 && d == 0 && !in_frac) continue;  // leading zeros
    if (digits < kMaxDigits) {
      mant = mant * 10 + d;
      if (mant > 0) ++digits;
      if (in_frac) ++frac;
    } else if (!in_frac) {
      return std::nullopt;
    } else if (d != 0) {
      sticky = true;
    }
  }
  if (!any) return std::nullopt;
  const std::string_view suffix = s.substr(i);
  Format fmt = Format::DecimalSI;
  int e10 = 0, k1024 = 0;
  if (suffix.empty()) {
  } else if (suffix.size() == 2 && suffix[1] == 'i') {
    const std::string_view kBin = "KMGTPE";
    const size_t p = kBin.find(suffix[0]);
    if (p == std::string_view::npos) return std::nullopt;
    fmt = Format::BinarySI;
    k1024 = static_cast<int>(p) + 1;
  } else if ((suffix[0] == 'e' || suffix[0] == 'E') && suffix.size() > 1) {
    size_t j = 1;
    bool eneg = false;
    if (suffix[j] == '+' || suffix[j] == '-') eneg = suffix[j++] == '-';
    if (j == suffix.size()) return std::nullopt;
    for (; j < suffix.size(); ++j) {
      if (!std::isdigit(static_cast<unsigned char>(suffix[j])) || e10 > 100) return std::nullopt;
      e10 = e10 * 10 + (suffix[j] - '0');
    }
    if (eneg) e10 = -e10;
    fmt = Format::DecimalExponent;
  } else if (suffix.size() == 1) {
    const std::string_view kDec = "num kMGTPE";
    const size_t p = kDec.find(suffix[0]);
    if (p == std::string_view::npos || suffix[0] == ' ') return std::nullopt;
    e10 = (static_cast<int>(p) - 3) * 3;
  } else {
    return std::nullopt;
  }
  // the value in units of 1n, rounded up (away from zero) as the apiserver does
  i128 nano = 0;
  const int p = 9 - frac + e10;
  if (mant != 0) {
    i128 num = mant;
    for (int k = 0; k < k1024; ++k) {
      if (num > pow10(kMaxDigits) / 1024) return std::nullopt;
      num *= 1024;
    }
    if (p >= 0) {
      // dropped digits would be worth 1n or more: out of range
      if (sticky || digit_count(num) + p > kMaxDigits) return std::nullopt;
      nano = num * pow10(p);
    } else if (-p > kMaxDigits) {
      nano = 1;  // below 1n: rounds up to 1n
    } else {
      const i128 den = pow10(-p);
      nano = num / den + ((num % den != 0 || sticky) ? 1 : 0);
    }
  } else if (sticky) {
    nano = 1;
  }
  if (nano == 0) return std::string("0");
  const std::string sign = neg ? "-" : "";
  if (fmt == Format::BinarySI && (nano < 1024 * kNano || nano % kNano != 0)) fmt = Format::DecimalSI;
  if (fmt == Format::BinarySI) {
    i128 v = nano / kNano;
    int k = 0;
    while (k < 6 && v % 1024 == 0) {
      v /= 1024;
      ++k;
    }
    std::string out = sign + to_string(v);
    if (k > 0) {
      out.push_back("KMGTPE"[k - 1]);
      out.push_back('i');
    }
    return out;
  }
  i128 m = nano;
  int e = -9;
  while (m % 10 == 0) {
    m /= 10;
    ++e;
  }
  const int r = ((e % 3) + 3) % 3;
  for (int k = 0; k < r; ++k) m *= 10;
  e -= r;
  std::string out = sign + to_string(m);
  if (fmt == Format::DecimalSI && e >= -9 && e <= 18) {
    static const char* kSuffix[] = {"n", "u", "m", "", "k", "M", "G", "T", "P", "E"};
    out += kSuffix[(e + 9) / 3];
  } else if (e != 0) {
    out += "e" + std::to_string(e);
  }
  return out;
}

}  // namespace bgc::kube

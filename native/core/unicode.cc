#include "core/unicode.h"

namespace bgc::unicode {

namespace {

// Decodes the code point at s[i]; *len gets its byte length (1 for an invalid byte, whose
// value is returned as 0xFFFFFFFF so it never matches a class).
char32_t decode(std::string_view s, size_t i, size_t* len) {
  constexpr char32_t kInvalid = 0xFFFFFFFF;
  const unsigned char c = static_cast<unsigned char>(s[i]);
  *len = 1;
  if (c < 0x80) return c;
  size_t n;  // continuation bytes
  if (c >= 0xC2 && c <= 0xDF) n = 1;
  else if (c >= 0xE0 && c <= 0xEF) n = 2;
  else if (c >= 0xF0 && c <= 0xF4) n = 3;
  else return kInvalid;
  if (i + n >= s.size()) return kInvalid;
  char32_t cp = c & (0x3F >> n);
  for (size_t k = 1; k <= n; ++k) {
    const unsigned char x = static_cast<unsigned char>(s[i + k]);
    if ((x & 0xC0) != 0x80) return kInvalid;
    cp = (cp << 6) | (x & 0x3F);
  }
  // overlong forms, surrogates and code points past U+10FFFF are invalid
  if ((n == 2 && cp < 0x800) || (n == 3 && (cp < 0x10000 || cp > 0x10FFFF)) || (cp >= 0xD800 && cp <= 0xDFFF)) {
    return kInvalid;
  }
  *len = n + 1;
  return cp;
}

void encode(char32_t cp, std::string& out) {
  if (cp < 0x80) {
    out += static_cast<char>(cp);
  } else if (cp < 0x800) {
    out += static_cast<char>(0xC0 | (cp >> 6));
    out += static_cast<char>(0x80 | (cp & 0x3F));
  } else if (cp < 0x10000) {
    out += static_cast<char>(0xE0 | (cp >> 12));
    out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
    out += static_cast<char>(0x80 | (cp & 0x3F));
  } else {
    out += static_cast<char>(0xF0 | (cp >> 18));
    out += static_cast<char>(0x80 | ((cp >> 12) & 0x3F));
    out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
    out += static_cast<char>(0x80 | (cp & 0x3F));
  }
}

}  // namespace

bool is_white_space(char32_t c) {
  return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

std::string_view trim(std::string_view s) {
  size_t b = 0;
  while (b < s.size()) {
    size_t len;
    if (!is_white_space(decode(s, b, &len))) break;
    b += len;
  }
  size_t e = s.size();
  while (e > b) {
    size_t start = e - 1;  // back to the lead byte of the last code point (at most 3 steps)
    while (start > b && e - start < 4 && (static_cast<unsigned char>(s[start]) & 0xC0) == 0x80) --start;
    size_t len;
    const char32_t cp = decode(s, start, &len);
    if (start + len != e || !is_white_space(cp)) break;
    e = start;
  }
  return s.substr(b, e - b);
}

char32_t to_lower(char32_t c) {
  if (c < 0x80) return c >= 'A' && c <= 'Z' ? c + 32 : c;
  if (c >= 0xC0 && c <= 0xDE && c != 0xD7) return c + 32;  // Latin-1 capitals (not ×)
  if (c >= 0x100 && c <= 0x17F) {  // Latin Extended-A: capital/small pairs
    if (c == 0x130 || c == 0x131 || c == 0x138 || c == 0x149 || c == 0x17F) return c;
    if (c == 0x178) return 0xFF;  // Ÿ -> ÿ
    const bool odd_capitals = (c >= 0x139 && c <= 0x148) || (c >= 0x179 && c <= 0x17E);
    if (odd_capitals) return c % 2 == 1 ? c + 1 : c;
    return c % 2 == 0 ? c + 1 : c;
  }
  if (c >= 0x391 && c <= 0x3AB && c != 0x3A2) return c + 32;  // Greek capitals
  if (c == 0x386) return 0x3AC;
  if (c >= 0x388 && c <= 0x38A) return c + 37;
  if (c == 0x38C) return 0x3CC;
  if (c == 0x38E || c == 0x38F) return c + 63;
  if (c >= 0x400 && c <= 0x40F) return c + 80;  // Cyrillic Ѐ-Џ
  if (c >= 0x410 && c <= 0x42F) return c + 32;  // Cyrillic А-Я
  if (c >= 0xFF21 && c <= 0xFF3A) return c + 32;  // fullwidth Ａ-Ｚ
  return c;
}

std::string to_lower(std::string_view s) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size();) {
    size_t len;
    const char32_t cp = decode(s, i, &len);
    if (cp == 0xFFFFFFFF) {
      out += s[i];
    } else if (cp == 0x130) {
      out += "i\xCC\x87";  // İ -> i + combining dot above (Rust's full lowercase mapping)
    } else {
      encode(to_lower(cp), out);
    }
    i += len;
  }
  return out;
}

}  // namespace bgc::unicode

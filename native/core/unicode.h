// The slices of Rust's `str` Unicode behaviour the reference relies on, for UTF-8 text:
// `trim()` (White_Space code points at both ends) and `to_lowercase()` (reference
// src/synchronizer.rs:225-236: a sheet cell is approved when
// `authorized.trim().to_lowercase() == "o"`).  A Google Form can put a non-breaking or
// ideographic space around the cell's "O"; an ASCII-only trim would reject those rows.
#pragma once

#include <string>
#include <string_view>

namespace bgc::unicode {

// Unicode White_Space (PropList.txt): U+0009-000D, 0020, 0085, 00A0, 1680, 2000-200A,
// 2028, 2029, 202F, 205F, 3000.  (Zero-width U+200B and U+FEFF are not White_Space.)
bool is_white_space(char32_t c);
// `s` without leading and trailing White_Space code points.  Invalid UTF-8 bytes are
// never trimmed.
std::string_view trim(std::string_view s);
// Lower-case mapping of one code point: ASCII, Latin-1, Latin Extended-A, Greek, Cyrillic
// and fullwidth Latin (U+FF21-FF3A); every other code point maps to itself.
char32_t to_lower(char32_t c);
// `s` with to_lower applied to every code point (U+0130 becomes "i̇", as in Rust's full
// mapping).  Invalid UTF-8 bytes are copied unchanged.
std::string to_lower(std::string_view s);

}  // namespace bgc::unicode

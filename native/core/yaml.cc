#include "core/yaml.h"

#include <charconv>
#include <cstring>
#include <map>

namespace bgc::yaml {

using json::Type;
using json::Value;

// ===========================================================================
// Emitter (serde_yaml 0.9 / libyaml compatible block style)
// ===========================================================================
namespace {

struct Cp {
  uint32_t cp;
  size_t len;
};

Cp decode(std::string_view s, size_t i) {
  unsigned char c = static_cast<unsigned char>(s[i]);
  auto cont = [&](size_t k) -> uint32_t {
    return i + k < s.size() ? (static_cast<unsigned char>(s[i + k]) & 0x3F) : 0;
  };
  if (c < 0x80) return {c, 1};
  if ((c & 0xE0) == 0xC0) return {((c & 0x1Fu) << 6) | cont(1), 2};
  if ((c & 0xF0) == 0xE0) return {((c & 0x0Fu) << 12) | (cont(1) << 6) | cont(2), 3};
  return {((c & 0x07u) << 18) | (cont(1) << 12) | (cont(2) << 6) | cont(3), 4};
}

bool is_break(uint32_t c) { return c == '\r' || c == '\n' || c == 0x85 || c == 0x2028 || c == 0x2029; }
bool is_blankz(uint32_t c) { return c == ' ' || c == '\t' || is_break(c) || c == 0; }
bool is_printable(uint32_t c) {
  return c == 0x0A || (c >= 0x20 && c <= 0x7E) || (c >= 0xA0 && c <= 0xD7FF) ||
         (c >= 0xE000 && c <= 0xFFFD && c != 0xFEFF);
}

struct Analysis {
  bool multiline = false;
  bool flow_plain_allowed = false;
  bool block_plain_allowed = false;
  bool single_quoted_allowed = false;
  bool block_allowed = false;
};

// Port of the decision logic of libyaml's yaml_emitter_analyze_scalar (libyaml, MIT
// License, Copyright (c) 2017-2020 Ingy döt Net, (c) 2006-2016 Kirill Simonov): the
// scalar-style rules serde_yaml 0.9 inherits, re-implemented here so that crdgen's output
// is byte-identical to the reference's crd.yaml.
Analysis analyze(std::string_view s) {
  Analysis a;
  if (s.empty()) {
    a.block_plain_allowed = true;
    a.single_quoted_allowed = true;
    return a;
  }
  bool block_ind = false, flow_ind = false, line_breaks = false, special = false;
  bool leading_space = false, leading_break = false, trailing_space = false, trailing_break = false;
  bool break_space = false, space_break = false;
  bool prev_space = false, prev_break = false;
  if (s.rfind("---", 0) == 0 || s.rfind("...", 0) == 0) {
    block_ind = true;
    flow_ind = true;
  }
  bool preceded_by_ws = true;
  size_t i = 0;
  Cp first = decode(s, 0);
  bool followed_by_ws = first.len >= s.size() ? true : is_blankz(decode(s, first.len).cp);
  while (i < s.size()) {
    Cp c = decode(s, i);
    uint32_t ch = c.cp;
    if (i == 0) {
      if (std::strchr("#,[]{}&*!|>'\"%@`", static_cast<int>(ch)) && ch != 0) {
        flow_ind = true;
        block_ind = true;
      }
      if (ch == '?' || ch == ':') {
        flow_ind = true;
        if (followed_by_ws) block_ind = true;
      }
      if (ch == '-' && followed_by_ws) {
        flow_ind = true;
        block_ind = true;
      }
    } else {
      if (ch == ',' || ch == '?' || ch == '[' || ch == ']' || ch == '{' || ch == '}') flow_ind = true;
      if (ch == ':') {
        flow_ind = true;
        if (followed_by_ws) block_ind = true;
      }
      if (ch == '#' && preceded_by_ws) {
        flow_ind = true;
        block_ind = true;
      }
    }
    if (!is_printable(ch)) special = true;
    if (is_break(ch)) line_breaks = true;
    if (ch == ' ') {
      if (i == 0) leading_space = true;
      if (i + c.len == s.size()) trailing_space = true;
      if (prev_break) break_space = true;
      prev_space = true;
      prev_break = false;
    } else if (is_break(ch)) {
      if (i == 0) leading_break = true;
      if (i + c.len == s.size()) trailing_break = true;
      if (prev_space) space_break = true;
      prev_space = false;
      prev_break = true;
    } else {
      prev_space = false;
      prev_break = false;
    }
    preceded_by_ws = is_blankz(ch);
    i += c.len;
    if (i < s.size()) {
      Cp n = decode(s, i);
      followed_by_ws = i + n.len >= s.size() ? true : is_blankz(decode(s, i + n.len).cp);
    }
  }
  a.multiline = line_breaks;
  a.flow_plain_allowed = a.block_plain_allowed = a.single_quoted_allowed = a.block_allowed = true;
  if (leading_space || leading_break || trailing_space || trailing_break) {
    a.flow_plain_allowed = a.block_plain_allowed = false;
  }
  if (trailing_space) a.block_allowed = false;
  if (break_space) a.flow_plain_allowed = a.block_plain_allowed = a.single_quoted_allowed = false;
  if (space_break || special) {
    a.flow_plain_allowed = a.block_plain_allowed = a.single_quoted_allowed = a.block_allowed = false;
  }
  if (line_breaks) a.flow_plain_allowed = a.block_plain_allowed = false;
  if (flow_ind) a.flow_plain_allowed = false;
  if (block_ind) a.block_plain_allowed = false;
  return a;
}

// --- serde_yaml's "would this plain scalar resolve to a non-string?" checks ---
bool digits_but_not_number(std::string_view s) {
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) s.remove_prefix(1);
  if (s.size() <= 1 || s[0] != '0') return false;
  for (char c : s.substr(1)) {
    if (c < '0' || c > '9') return false;
  }
  return true;
}

bool is_null_word(std::string_view s) { return s == "~" || s == "null" || s == "Null" || s == "NULL"; }
bool is_bool_word(std::string_view s) {
  return s == "true" || s == "True" || s == "TRUE" || s == "false" || s == "False" || s == "FALSE";
}

bool all_in_radix(std::string_view s, int radix) {
  if (s.empty()) return false;
  for (char c : s) {
    int d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (c >= 'a' && c <= 'z') d = c - 'a' + 10;
    else if (c >= 'A' && c <= 'Z') d = c - 'A' + 10;
    else return false;
    if (d >= radix) return false;
  }
  return true;
}

bool is_int_word(std::string_view s) {
  std::string_view u = s;
  if (!u.empty() && (u[0] == '+' || u[0] == '-')) u.remove_prefix(1);
  if (u.rfind("0x", 0) == 0) return all_in_radix(u.substr(2), 16);
  if (u.rfind("0o", 0) == 0) return all_in_radix(u.substr(2), 8);
  if (u.rfind("0b", 0) == 0) return all_in_radix(u.substr(2), 2);
  if (!u.empty() && (u[0] == '+' || u[0] == '-')) return false;
  if (digits_but_not_number(s)) return false;
  return all_in_radix(u, 10);
}

// Rust f64::from_str grammar, finite results only (serde_yaml parse_f64).
bool is_float_word(std::string_view s) {
  if (s == ".inf" || s == ".Inf" || s == ".INF" || s == "+.inf" || s == "+.Inf" || s == "+.INF" ||
      s == "-.inf" || s == "-.Inf" || s == "-.INF" || s == ".nan" || s == ".NaN" || s == ".NAN") {
    return true;
  }
  std::string_view u = s;
  if (!u.empty() && (u[0] == '+' || u[0] == '-')) u.remove_prefix(1);
  size_t i = 0, digits = 0;
  while (i < u.size() && u[i] >= '0' && u[i] <= '9') ++i, ++digits;
  if (i < u.size() && u[i] == '.') {
    ++i;
    while (i < u.size() && u[i] >= '0' && u[i] <= '9') ++i, ++digits;
  }
  if (digits == 0) return false;
  if (i < u.size() && (u[i] == 'e' || u[i] == 'E')) {
    ++i;
    if (i < u.size() && (u[i] == '+' || u[i] == '-')) ++i;
    size_t ed = 0;
    while (i < u.size() && u[i] >= '0' && u[i] <= '9') ++i, ++ed;
    if (ed == 0) return false;
  }
  return i == u.size();
}

enum class Style { Any, Plain, SingleQuoted, DoubleQuoted, Literal };

class Emitter {
 public:
  std::string out;

  void document(const Value& v) {
    if (v.is_object() && !v.empty()) {
      mapping(v, 0, /*inline_first=*/true);
    } else if (v.is_array() && !v.empty()) {
      sequence(v, 0, true);
    } else {
      // a top-level block scalar's content sits at the default indentation (2), as in
      // libyaml; plain/quoted scalars ignore the indent
      scalar_node(v, 2, false);
    }
    // a literal scalar already ends with its own line break(s): another one would add a
    // blank line that keep-chomping ("|+") readers count as content
    if (out.empty() || out.back() != '\n') out.push_back('\n');
  }

 private:
  void write_indent(int indent) {
    if (!out.empty() && out.back() != '\n') out.push_back('\n');
    out.append(static_cast<size_t>(indent), ' ');
  }

  void mapping(const Value& m, int indent, bool inline_first) {
    const auto& keys = m.keys();
    const auto& vals = m.values();
    for (size_t i = 0; i < keys.size(); ++i) {
      if (!(i == 0 && inline_first)) write_indent(indent);
      string_scalar(keys[i], indent, /*simple_key=*/true);
      out.push_back(':');
      const Value& v = vals[i];
      if (v.is_object() && !v.empty()) {
        mapping(v, indent + 2, false);
      } else if (v.is_array() && !v.empty()) {
        sequence(v, indent, false);
      } else {
        out.push_back(' ');
        scalar_node(v, indent + 2, false);
      }
    }
  }

  void sequence(const Value& s, int indent, bool inline_first) {
    const auto& items = s.items();
    for (size_t i = 0; i < items.size(); ++i) {
      if (!(i == 0 && inline_first)) write_indent(indent);
      out.append("- ");
      const Value& v = items[i];
      if (v.is_object() && !v.empty()) {
        mapping(v, indent + 2, true);
      } else if (v.is_array() && !v.empty()) {
        sequence(v, indent + 2, true);
      } else {
        scalar_node(v, indent + 2, false);
      }
    }
  }

  void scalar_node(const Value& v, int block_indent, bool simple_key) {
    switch (v.type()) {
      case Type::Null: out.append("null"); return;
      case Type::Bool: out.append(v.as_bool() ? "true" : "false"); return;
      case Type::Int:
      case Type::UInt: out.append(v.dump()); return;
      case Type::Double: {
        double d = v.as_double();
        if (d != d) out.append(".nan");
        else if (d == 1.0 / 0.0) out.append(".inf");
        else if (d == -1.0 / 0.0) out.append("-.inf");
        else out.append(v.dump());
        return;
      }
      case Type::String: string_scalar(v.as_string(), block_indent, simple_key); return;
      case Type::Array: out.append("[]"); return;
      case Type::Object: out.append("{}"); return;
    }
  }

  void string_scalar(const std::string& s, int block_indent, bool simple_key) {
    Style requested;
    if (s.find('\n') != std::string::npos) {
      requested = Style::Literal;
    } else if (s.empty() || is_null_word(s) || is_bool_word(s) || is_int_word(s) ||
               is_float_word(s) || digits_but_not_number(s)) {
      requested = Style::SingleQuoted;
    } else {
      requested = Style::Any;
    }
    Analysis a = analyze(s);
    Style st = requested == Style::Any ? Style::Plain : requested;
    if (simple_key && a.multiline) st = Style::DoubleQuoted;
    if (st == Style::Plain) {
      if (!a.block_plain_allowed) st = Style::SingleQuoted;
      if (s.empty() && simple_key) st = Style::SingleQuoted;
    }
    if (st == Style::SingleQuoted && !a.single_quoted_allowed) st = Style::DoubleQuoted;
    if (st == Style::Literal && (!a.block_allowed || simple_key)) st = Style::DoubleQuoted;
    switch (st) {
      case Style::Plain: out.append(s); break;
      case Style::SingleQuoted: single_quoted(s); break;
      case Style::DoubleQuoted: double_quoted(s); break;
      case Style::Literal: literal(s, block_indent); break;
      default: out.append(s);
    }
  }

  void single_quoted(const std::string& s) {
    out.push_back('\'');
    for (char c : s) {
      if (c == '\'') out.append("''");
      else out.push_back(c);
    }
    out.push_back('\'');
  }

  void double_quoted(const std::string& s) {
    static const char kHex[] = "0123456789ABCDEF";
    out.push_back('"');
    size_t i = 0;
    while (i < s.size()) {
      Cp c = decode(s, i);
      uint32_t ch = c.cp;
      if (!is_printable(ch) || ch == 0xFEFF || is_break(ch) || ch == '"' || ch == '\\') {
        out.push_back('\\');
        switch (ch) {
          case 0x00: out.push_back('0'); break;
          case 0x07: out.push_back('a'); break;
          case 0x08: out.push_back('b'); break;
          case 0x09: out.push_back('t'); break;
          case 0x0A: out.push_back('n'); break;
          case 0x0B: out.push_back('v'); break;
          case 0x0C: out.push_back('f'); break;
          case 0x0D: out.push_back('r'); break;
          case 0x1B: out.push_back('e'); break;
          case 0x22: out.push_back('"'); break;
          case 0x5C: out.push_back('\\'); break;
          case 0x85: out.push_back('N'); break;
          case 0xA0: out.push_back('_'); break;
          case 0x2028: out.push_back('L'); break;
          case 0x2029: out.push_back('P'); break;
          default: {
            int width;
            if (ch <= 0xFF) {
              out.push_back('x');
              width = 2;
            } else if (ch <= 0xFFFF) {
              out.push_back('u');
              width = 4;
            } else {
              out.push_back('U');
              width = 8;
            }
            for (int k = width - 1; k >= 0; --k) out.push_back(kHex[(ch >> (4 * k)) & 0xF]);
          }
        }
      } else {
        out.append(s, i, c.len);
      }
      i += c.len;
    }
    out.push_back('"');
  }

  void literal(const std::string& s, int indent) {
    out.append("|");
    Cp first = decode(s, 0);
    if (first.cp == ' ' || is_break(first.cp)) out.push_back('2');
    // chomping indicator (yaml_emitter_write_block_scalar_hints)
    size_t n = s.size();
    auto prev_start = [&](size_t pos) {
      size_t p = pos;
      do {
        --p;
      } while (p > 0 && (static_cast<unsigned char>(s[p]) & 0xC0) == 0x80);
      return p;
    };
    size_t last = prev_start(n);
    if (!is_break(decode(s, last).cp)) {
      out.push_back('-');
    } else if (last == 0) {
      out.push_back('+');
    } else {
      size_t before = prev_start(last);
      if (is_break(decode(s, before).cp)) out.push_back('+');
    }
    out.push_back('\n');
    bool breaks = true;
    size_t i = 0;
    while (i < n) {
      Cp c = decode(s, i);
      if (is_break(c.cp)) {
        out.push_back('\n');
        breaks = true;
      } else {
        if (breaks) out.append(static_cast<size_t>(indent), ' ');
        out.append(s, i, c.len);
        breaks = false;
      }
      i += c.len;
    }
  }
};

}  // namespace

std::string emit(const Value& v) {
  Emitter e;
  e.document(v);
  return std::move(e.out);
}

// ===========================================================================
// Parser (YAML 1.2 subset)
// ===========================================================================
namespace {

struct Line {
  int indent;          // leading spaces
  std::string text;    // content after indentation (comments stripped for structure)
  std::string raw;     // full original line (for block scalars)
  int number;
};

Value resolve_plain(const std::string& s) {
  if (s.empty() || is_null_word(s)) return Value();
  if (s == "true" || s == "True" || s == "TRUE") return Value(true);
  if (s == "false" || s == "False" || s == "FALSE") return Value(false);
  if (is_int_word(s)) {
    std::string_view u = s;
    bool neg = false;
    if (u[0] == '+' || u[0] == '-') {
      neg = u[0] == '-';
      u.remove_prefix(1);
    }
    int radix = 10;
    if (u.rfind("0x", 0) == 0) radix = 16, u.remove_prefix(2);
    else if (u.rfind("0o", 0) == 0) radix = 8, u.remove_prefix(2);
    else if (u.rfind("0b", 0) == 0) radix = 2, u.remove_prefix(2);
    uint64_t v = 0;
    auto r = std::from_chars(u.data(), u.data() + u.size(), v, radix);
    if (r.ec == std::errc()) {
      if (neg) {
        if (v <= static_cast<uint64_t>(INT64_MAX) + 1) {
          return Value(static_cast<long long>(-static_cast<__int128>(v)));
        }
      } else {
        return Value(static_cast<unsigned long long>(v));
      }
    }
  }
  if (is_float_word(s)) {
    std::string t = s;
    if (t.find(".inf") != std::string::npos || t.find(".Inf") != std::string::npos ||
        t.find(".INF") != std::string::npos) {
      return Value(t[0] == '-' ? -1.0 / 0.0 : 1.0 / 0.0);
    }
    if (t.find(".nan") != std::string::npos || t.find(".NaN") != std::string::npos ||
        t.find(".NAN") != std::string::npos) {
      return Value(0.0 / 0.0);
    }
    if (t[0] == '+') t.erase(0, 1);
    double d = std::strtod(t.c_str(), nullptr);
    return Value(d);
  }
  return Value(s);
}

class Parser {
 public:
  explicit Parser(const std::string& text) { split(text); }

  bool next_document(Value& out) {
    // skip document separators / blank lines
    while (pos_ < lines_.size()) {
      const std::string& t = lines_[pos_].text;
      if (t.empty()) {
        ++pos_;
        continue;
      }
      if (lines_[pos_].indent == 0 && (t == "---" || t.rfind("--- ", 0) == 0)) {
        std::string rest = t.size() > 4 ? t.substr(4) : "";
        ++pos_;
        if (!rest.empty()) {
          out = parse_inline_value(rest, 0);
          return true;
        }
        continue;
      }
      if (lines_[pos_].indent == 0 && t == "...") {
        ++pos_;
        continue;
      }
      break;
    }
    if (pos_ >= lines_.size()) return false;
    out = parse_node(lines_[pos_].indent);
    return true;
  }

 private:
  [[noreturn]] void fail(const std::string& msg, int line) {
    throw Error("yaml: " + msg + " (line " + std::to_string(line) + ")");
  }

  static std::string strip_comment(const std::string& s) {
    bool in_s = false, in_d = false;
    for (size_t i = 0; i < s.size(); ++i) {
      char c = s[i];
      if (in_d) {
        if (c == '\\') ++i;
        else if (c == '"') in_d = false;
      } else if (in_s) {
        if (c == '\'') in_s = false;
      } else if (c == '"') {
        in_d = true;
      } else if (c == '\'') {
        in_s = true;
      } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
        std::string r = s.substr(0, i);
        while (!r.empty() && (r.back() == ' ' || r.back() == '\t')) r.pop_back();
        return r;
      }
    }
    std::string r = s;
    while (!r.empty() && (r.back() == ' ' || r.back() == '\t' || r.back() == '\r')) r.pop_back();
    return r;
  }

  void split(const std::string& text) {
    size_t start = 0;
    int num = 1;
    // a final line break terminates the last line; it does not start an empty one
    while (start < text.size()) {
      size_t nl = text.find('\n', start);
      std::string raw = text.substr(start, nl == std::string::npos ? std::string::npos : nl - start);
      if (!raw.empty() && raw.back() == '\r') raw.pop_back();
      int ind = 0;
      while (static_cast<size_t>(ind) < raw.size() && raw[static_cast<size_t>(ind)] == ' ') ++ind;
      std::string body = raw.substr(static_cast<size_t>(ind));
      lines_.push_back({ind, strip_comment(body), raw, num++});
      if (nl == std::string::npos) break;
      start = nl + 1;
    }
  }

  void skip_blank() {
    while (pos_ < lines_.size() && lines_[pos_].text.empty()) ++pos_;
  }

  bool at_doc_marker() const {
    if (pos_ >= lines_.size()) return false;
    const Line& l = lines_[pos_];
    return l.indent == 0 && (l.text == "---" || l.text.rfind("--- ", 0) == 0 || l.text == "...");
  }

  static bool is_seq_entry(const std::string& t) { return t == "-" || t.rfind("- ", 0) == 0; }

  // Finds the `: ` (or trailing `:`) that separates a mapping key, honouring quotes
  // and flow brackets. Returns npos when the text is not a mapping entry.
  static size_t find_key_colon(const std::string& t) {
    if (t.empty()) return std::string::npos;
    size_t i = 0;
    if (t[0] == '"' || t[0] == '\'') {
      char q = t[0];
      i = 1;
      while (i < t.size()) {
        if (q == '"' && t[i] == '\\') {
          i += 2;
          continue;
        }
        if (t[i] == q) {
          if (q == '\'' && i + 1 < t.size() && t[i + 1] == '\'') {
            i += 2;
            continue;
          }
          break;
        }
        ++i;
      }
      ++i;
      if (i < t.size() && t[i] == ':' && (i + 1 == t.size() || t[i + 1] == ' ')) return i;
      return std::string::npos;
    }
    if (t[0] == '[' || t[0] == '{') return std::string::npos;
    for (; i < t.size(); ++i) {
      if (t[i] == ':' && (i + 1 == t.size() || t[i + 1] == ' ' || t[i + 1] == '\t')) return i;
    }
    return std::string::npos;
  }

  std::string parse_key(const std::string& k, int line) {
    std::string key = k;
    while (!key.empty() && key.back() == ' ') key.pop_back();
    if (key.empty()) return key;
    if (key[0] == '"' || key[0] == '\'') {
      size_t p = 0;
      Value v = parse_flow(key, p, line);
      if (!v.is_string()) fail("bad key", line);
      return v.as_string();
    }
    return key;
  }

  Value parse_node(int indent) {
    skip_blank();
    if (pos_ >= lines_.size() || at_doc_marker()) return Value();
    const Line& l = lines_[pos_];
    if (l.indent < indent) return Value();
    if (is_seq_entry(l.text)) return parse_sequence(l.indent);
    if (find_key_colon(l.text) != std::string::npos) return parse_mapping(l.indent);
    // scalar / flow spanning lines
    int ind = l.indent;
    ++pos_;
    if (l.text[0] == '|' || l.text[0] == '>') return parse_block_scalar(l.text, ind, l.number);
    return parse_inline_value_cont(l.text, ind - 1, l.number);
  }

  Value parse_mapping(int indent) {
    Value m = Value::object();
    while (true) {
      skip_blank();
      if (pos_ >= lines_.size() || at_doc_marker()) break;
      const Line& l = lines_[pos_];
      if (l.indent < indent) break;
      if (l.indent > indent) fail("unexpected indentation", l.number);
      if (is_seq_entry(l.text)) break;
      size_t c = find_key_colon(l.text);
      if (c == std::string::npos) fail("expected a mapping key", l.number);
      std::string key = parse_key(l.text.substr(0, c), l.number);
      std::string rest = c + 1 < l.text.size() ? l.text.substr(c + 1) : "";
      size_t a = rest.find_first_not_of(" \t");
      rest = a == std::string::npos ? "" : rest.substr(a);
      int line_no = l.number;
      ++pos_;
      m.set(key, parse_value_after_indicator(rest, indent, line_no, /*in_map=*/true));
    }
    return m;
  }

  Value parse_sequence(int indent) {
    Value s = Value::array();
    while (true) {
      skip_blank();
      if (pos_ >= lines_.size() || at_doc_marker()) break;
      Line& l = lines_[pos_];
      if (l.indent != indent || !is_seq_entry(l.text)) {
        if (l.indent > indent) fail("unexpected indentation in sequence", l.number);
        break;
      }
      std::string rest = l.text.size() > 2 ? l.text.substr(2) : "";
      size_t a = rest.find_first_not_of(' ');
      int extra = a == std::string::npos ? 0 : static_cast<int>(a);
      rest = a == std::string::npos ? "" : rest.substr(a);
      int item_indent = indent + 2 + extra;
      if (!rest.empty() && (is_seq_entry(rest) || find_key_colon(rest) != std::string::npos)) {
        // Rewrite the current line in place as a nested block starting at item_indent.
        l.indent = item_indent;
        l.text = rest;
        s.push_back(parse_node(item_indent));
        continue;
      }
      int line_no = l.number;
      ++pos_;
      s.push_back(parse_value_after_indicator(rest, indent, line_no, false));
    }
    return s;
  }

  // Value following `key:` or `- `.
  Value parse_value_after_indicator(const std::string& rest, int parent_indent, int line_no, bool in_map) {
    std::string r = rest;
    // ignore tags like !!str / !foo (value kept as parsed)
    bool force_str = false;
    if (!r.empty() && r[0] == '!') {
      size_t sp = r.find(' ');
      std::string tag = r.substr(0, sp);
      force_str = tag == "!!str";
      r = sp == std::string::npos ? "" : r.substr(sp + 1);
    }
    if (!r.empty() && (r[0] == '&' || r[0] == '*')) fail("anchors/aliases are not supported", line_no);
    if (r.empty()) {
      skip_blank();
      if (pos_ >= lines_.size() || at_doc_marker()) return Value();
      const Line& n = lines_[pos_];
      if (n.indent > parent_indent) return parse_node(n.indent);
      if (in_map && n.indent == parent_indent && is_seq_entry(n.text)) return parse_sequence(n.indent);
      return Value();
    }
    if (r[0] == '|' || r[0] == '>') return parse_block_scalar(r, parent_indent, line_no);
    Value v = parse_inline_value_cont(r, parent_indent, line_no);
    if (force_str && !v.is_string()) {
      if (v.is_null()) return Value(r.substr(0));
      return Value(r);
    }
    return v;
  }

  // Inline scalar/flow value that may continue on more-indented following lines.
  Value parse_inline_value_cont(const std::string& first, int parent_indent, int line_no) {
    std::string text = first;
    char c0 = text[0];
    if (c0 == '[' || c0 == '{' || c0 == '"' || c0 == '\'') {
      // gather continuation lines until the flow/quoted value is complete
      while (!flow_complete(text) && pos_ < lines_.size()) {
        const Line& n = lines_[pos_];
        std::string piece = c0 == '"' || c0 == '\'' ? trim_left(n.raw) : n.text;
        if (piece.empty()) {
          text += "\n";
        } else {
          text += (text.back() == '\n' ? "" : " ") + piece;
        }
        ++pos_;
      }
      size_t p = 0;
      Value v = parse_flow(text, p, line_no);
      while (p < text.size() && text[p] == ' ') ++p;
      if (p != text.size()) fail("trailing characters after value", line_no);
      return v;
    }
    // plain multi-line scalar
    while (pos_ < lines_.size()) {
      const Line& n = lines_[pos_];
      if (n.text.empty()) {
        // blank line inside a plain scalar folds to a newline if followed by continuation
        size_t q = pos_;
        while (q < lines_.size() && lines_[q].text.empty()) ++q;
        if (q < lines_.size() && lines_[q].indent > parent_indent && !is_structural(lines_[q])) {
          for (size_t k = pos_; k < q; ++k) text += "\n";
          pos_ = q;
          continue;
        }
        break;
      }
      if (n.indent <= parent_indent || is_structural(n)) break;
      text += (text.back() == '\n' ? "" : " ") + n.text;
      ++pos_;
    }
    return resolve_plain(text);
  }

  bool is_structural(const Line& l) const {
    return is_seq_entry(l.text) || find_key_colon(l.text) != std::string::npos;
  }

  static std::string trim_left(const std::string& s) {
    size_t a = s.find_first_not_of(" \t");
    return a == std::string::npos ? "" : s.substr(a);
  }

  static bool flow_complete(const std::string& t) {
    int depth = 0;
    bool in_s = false, in_d = false;
    for (size_t i = 0; i < t.size(); ++i) {
      char c = t[i];
      if (in_d) {
        if (c == '\\') ++i;
        else if (c == '"') in_d = false;
        continue;
      }
      if (in_s) {
        if (c == '\'') {
          if (i + 1 < t.size() && t[i + 1] == '\'') ++i;
          else in_s = false;
        }
        continue;
      }
      if (c == '"') in_d = true;
      else if (c == '\'') in_s = true;
      else if (c == '[' || c == '{') ++depth;
      else if (c == ']' || c == '}') --depth;
    }
    return depth <= 0 && !in_s && !in_d;
  }

  Value parse_inline_value(const std::string& text, int line_no) {
    return parse_inline_value_cont(text, -1, line_no);
  }

  Value parse_block_scalar(const std::string& header, int parent_indent, int line_no) {
    bool folded = header[0] == '>';
    char chomp = 'c';
    int explicit_indent = 0;
    for (size_t i = 1; i < header.size(); ++i) {
      char c = header[i];
      if (c == '-') chomp = '-';
      else if (c == '+') chomp = '+';
      else if (c >= '1' && c <= '9') explicit_indent = c - '0';
      else if (c == ' ') break;
      else fail("bad block scalar header", line_no);
    }
    // determine content indentation
    int block_indent = -1;
    if (explicit_indent) block_indent = parent_indent + explicit_indent;
    std::vector<std::string> content;
    while (pos_ < lines_.size()) {
      const Line& n = lines_[pos_];
      bool blank = n.raw.find_first_not_of(' ') == std::string::npos;
      if (blank) {
        content.push_back("");
        ++pos_;
        continue;
      }
      if (block_indent < 0) {
        if (n.indent <= parent_indent) break;
        block_indent = n.indent;
      }
      if (n.indent < block_indent) break;
      content.push_back(n.raw.substr(static_cast<size_t>(block_indent)));
      ++pos_;
    }
    // trailing blank lines belong to the scalar only for chomping purposes; give the
    // ones beyond the content back to the structure.
    size_t trailing = 0;
    while (trailing < content.size() && content[content.size() - 1 - trailing].empty()) ++trailing;
    std::string body;
    size_t nonblank = content.size() - trailing;
    for (size_t i = 0; i < nonblank; ++i) {
      if (i) {
        if (folded && !content[i].empty() && !content[i - 1].empty() && content[i][0] != ' ' &&
            content[i - 1][0] != ' ') {
          body += " ";
        } else {
          body += "\n";
        }
      }
      body += content[i];
    }
    if (chomp == '-') {
      // strip
    } else if (chomp == '+') {
      if (nonblank) body += "\n";
      for (size_t i = 0; i < trailing; ++i) body += "\n";
    } else if (nonblank) {
      body += "\n";
    }
    return Value(body);
  }

  // ---- flow-style values (JSON-compatible superset) ----
  Value parse_flow(const std::string& t, size_t& p, int line_no) {
    skip_sp(t, p);
    if (p >= t.size()) return Value();
    char c = t[p];
    if (c == '[') {
      ++p;
      Value a = Value::array();
      skip_sp(t, p);
      if (p < t.size() && t[p] == ']') {
        ++p;
        return a;
      }
      while (true) {
        a.push_back(parse_flow(t, p, line_no));
        skip_sp(t, p);
        if (p < t.size() && t[p] == ',') {
          ++p;
          skip_sp(t, p);
          if (p < t.size() && t[p] == ']') {
            ++p;
            return a;
          }
          continue;
        }
        if (p < t.size() && t[p] == ']') {
          ++p;
          return a;
        }
        fail("expected , or ] in flow sequence", line_no);
      }
    }
    if (c == '{') {
      ++p;
      Value m = Value::object();
      skip_sp(t, p);
      if (p < t.size() && t[p] == '}') {
        ++p;
        return m;
      }
      while (true) {
        skip_sp(t, p);
        Value k = parse_flow_scalar(t, p, line_no, true);
        skip_sp(t, p);
        Value v;
        if (p < t.size() && t[p] == ':') {
          ++p;
          v = parse_flow(t, p, line_no);
        }
        m.set(k.is_string() ? k.as_string() : k.dump(), v);
        skip_sp(t, p);
        if (p < t.size() && t[p] == ',') {
          ++p;
          skip_sp(t, p);
          if (p < t.size() && t[p] == '}') {
            ++p;
            return m;
          }
          continue;
        }
        if (p < t.size() && t[p] == '}') {
          ++p;
          return m;
        }
        fail("expected , or } in flow mapping", line_no);
      }
    }
    return parse_flow_scalar(t, p, line_no, false);
  }

  static void skip_sp(const std::string& t, size_t& p) {
    while (p < t.size() && (t[p] == ' ' || t[p] == '\t' || t[p] == '\n')) ++p;
  }

  Value parse_flow_scalar(const std::string& t, size_t& p, int line_no, bool is_key) {
    if (p < t.size() && t[p] == '"') return Value(parse_double_quoted(t, p, line_no));
    if (p < t.size() && t[p] == '\'') {
      ++p;
      std::string out;
      while (true) {
        if (p >= t.size()) fail("unterminated single-quoted string", line_no);
        if (t[p] == '\'') {
          if (p + 1 < t.size() && t[p + 1] == '\'') {
            out.push_back('\'');
            p += 2;
            continue;
          }
          ++p;
          break;
        }
        if (t[p] == '\n') {
          fold_newlines(t, p, out);
          continue;
        }
        out.push_back(t[p++]);
      }
      return Value(out);
    }
    size_t start = p;
    bool in_flow = true;
    while (p < t.size()) {
      char c = t[p];
      if (in_flow && (c == ',' || c == ']' || c == '}')) break;
      if (c == ':' && (p + 1 >= t.size() || t[p + 1] == ' ' || t[p + 1] == ',' || (is_key && true))) {
        if (p + 1 >= t.size() || t[p + 1] == ' ' || t[p + 1] == ',' || t[p + 1] == '}' || t[p + 1] == ']') break;
      }
      ++p;
    }
    std::string s = t.substr(start, p - start);
    while (!s.empty() && s.back() == ' ') s.pop_back();
    return is_key ? Value(s) : resolve_plain(s);
  }

  static void fold_newlines(const std::string& t, size_t& p, std::string& out) {
    // line folding inside quoted scalars: single newline -> space, n newlines -> n-1 \n
    while (!out.empty() && (out.back() == ' ' || out.back() == '\t')) out.pop_back();
    size_t count = 0;
    while (p < t.size() && (t[p] == '\n' || t[p] == ' ' || t[p] == '\t')) {
      if (t[p] == '\n') ++count;
      ++p;
    }
    if (count <= 1) out.push_back(' ');
    else out.append(count - 1, '\n');
  }

  std::string parse_double_quoted(const std::string& t, size_t& p, int line_no) {
    ++p;
    std::string out;
    while (true) {
      if (p >= t.size()) fail("unterminated double-quoted string", line_no);
      char c = t[p];
      if (c == '"') {
        ++p;
        break;
      }
      if (c == '\n') {
        fold_newlines(t, p, out);
        continue;
      }
      if (c != '\\') {
        out.push_back(c);
        ++p;
        continue;
      }
      ++p;
      if (p >= t.size()) fail("bad escape", line_no);
      char e = t[p++];
      auto hex = [&](int n) {
        if (p + static_cast<size_t>(n) > t.size()) fail("bad escape", line_no);
        uint32_t v = 0;
        auto r = std::from_chars(t.data() + p, t.data() + p + n, v, 16);
        if (r.ec != std::errc()) fail("bad escape", line_no);
        p += static_cast<size_t>(n);
        return v;
      };
      uint32_t cp = 0;
      switch (e) {
        case '0': out.push_back('\0'); continue;
        case 'a': out.push_back('\a'); continue;
        case 'b': out.push_back('\b'); continue;
        case 't': case '\t': out.push_back('\t'); continue;
        case 'n': out.push_back('\n'); continue;
        case 'v': out.push_back('\v'); continue;
        case 'f': out.push_back('\f'); continue;
        case 'r': out.push_back('\r'); continue;
        case 'e': out.push_back('\x1b'); continue;
        case ' ': out.push_back(' '); continue;
        case '"': out.push_back('"'); continue;
        case '/': out.push_back('/'); continue;
        case '\\': out.push_back('\\'); continue;
        case 'N': cp = 0x85; break;
        case '_': cp = 0xA0; break;
        case 'L': cp = 0x2028; break;
        case 'P': cp = 0x2029; break;
        case 'x': cp = hex(2); break;
        case 'u': cp = hex(4); break;
        case 'U': cp = hex(8); break;
        case '\n': {
          // escaped line break: join without space
          while (p < t.size() && (t[p] == ' ' || t[p] == '\t')) ++p;
          continue;
        }
        default: fail("bad escape", line_no);
      }
      append_utf8(cp, out);
    }
    return out;
  }

  static void append_utf8(uint32_t cp, std::string& out) {
    if (cp < 0x80) {
      out.push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }

  std::vector<Line> lines_;
  size_t pos_ = 0;
};

}  // namespace

Value parse(const std::string& text) {
  Parser p(text);
  Value v;
  if (!p.next_document(v)) return Value();
  return v;
}

std::vector<Value> parse_all(const std::string& text) {
  Parser p(text);
  std::vector<Value> docs;
  Value v;
  while (p.next_document(v)) {
    if (!v.is_null()) docs.push_back(std::move(v));
    v = Value();
  }
  return docs;
}

}  // namespace bgc::yaml

#include "sync/sheet.h"

#include <algorithm>
#include <charconv>
#include <map>

#include "core/unicode.h"

namespace bgc::sync {

using json::Value;

std::string infer_header(const std::string& h) {
  auto has = [&](const char* s) { return h.find(s) != std::string::npos; };
  if (h == "타임스탬프") return "timestamp";
  if (h == "이름") return "name";
  if (h == "소속") return "department";
  if (has("SNUCSE ID")) return "id_username";
  if (has("사용할 서버")) return "gpu_server";
  if (has("GPU 개수")) return "gpu_request";
  if (has("vCPU 개수")) return "cpu_request";
  if (has("메모리")) return "memory_request";
  if (has("스토리지")) return "storage_request";
  if (has("MiG 개수")) return "mig_request";
  if (has("요청 사유")) return "description";
  if (has("승인")) return "authorized";
  if (has("이메일")) return "email";
  throw CsvHeaderError("csv header error: unknown header: \"" + h + "\"");
}

std::vector<std::vector<std::string>> parse_records(std::string_view t) {
  std::vector<std::vector<std::string>> out;
  std::vector<std::string> rec;
  std::string field;
  size_t i = 0;
  bool in_quotes = false;
  bool field_started = false;
  // skip a UTF-8 BOM
  if (t.size() >= 3 && static_cast<unsigned char>(t[0]) == 0xEF && static_cast<unsigned char>(t[1]) == 0xBB &&
      static_cast<unsigned char>(t[2]) == 0xBF) {
    i = 3;
  }
  auto end_record = [&]() {
    rec.push_back(field);
    field.clear();
    field_started = false;
    // an empty line is not a record (csv crate semantics)
    if (!(rec.size() == 1 && rec[0].empty())) out.push_back(rec);
    rec.clear();
  };
  while (i < t.size()) {
    char c = t[i];
    if (in_quotes) {
      if (c == '"') {
        if (i + 1 < t.size() && t[i + 1] == '"') {
          field.push_back('"');
          i += 2;
          continue;
        }
        in_quotes = false;
        ++i;
        continue;
      }
      field.push_back(c);
      ++i;
      continue;
    }
    if (c == '"' && !field_started) {
      in_quotes = true;
      field_started = true;
      ++i;
      continue;
    }
    if (c == ',') {
      rec.push_back(field);
      field.clear();
      field_started = false;
      ++i;
      continue;
    }
    if (c == '\r' || c == '\n') {
      end_record();
      if (c == '\r' && i + 1 < t.size() && t[i + 1] == '\n') ++i;
      ++i;
      continue;
    }
    field.push_back(c);
    field_started = true;
    ++i;
  }
  if (in_quotes) throw CsvParseError("csv parsing error: unterminated quoted field");
  if (field_started || !field.empty() || !rec.empty()) end_record();
  return out;
}

static bool parse_i64(const std::string& s, int64_t& out) {
  std::string_view v = s;
  if (!v.empty() && v[0] == '+') v.remove_prefix(1);  // Rust i64::from_str accepts '+'
  if (v.empty()) return false;
  auto r = std::from_chars(v.data(), v.data() + v.size(), out);
  return r.ec == std::errc() && r.ptr == v.data() + v.size();
}

std::vector<Row> parse_csv(std::string_view text, std::vector<std::string>* warnings) {
  auto records = parse_records(text);
  std::vector<Row> rows;
  if (records.empty()) return rows;
  std::vector<std::string> fields;
  for (const auto& h : records[0]) fields.push_back(infer_header(h));
  // column index per Row field (-1 = missing, -2 = duplicate)
  static const char* kNames[] = {"name", "department", "id_username", "gpu_server", "gpu_request", "cpu_request",
                                 "memory_request", "storage_request", "mig_request", "authorized"};
  std::map<std::string, int> col;
  for (const char* n : kNames) col[n] = -1;
  for (size_t c = 0; c < fields.size(); ++c) {
    auto it = col.find(fields[c]);
    if (it == col.end()) continue;
    it->second = it->second == -1 ? static_cast<int>(c) : -2;
  }
  for (size_t r = 1; r < records.size(); ++r) {
    const auto& rec = records[r];
    auto warn = [&](const std::string& msg) {
      if (warnings) warnings->push_back("row parsing error. skipping: record " + std::to_string(r) + ": " + msg);
    };
    if (rec.size() != fields.size()) {
      warn("found record with " + std::to_string(rec.size()) + " fields, but the previous record has " +
           std::to_string(fields.size()) + " fields");
      continue;
    }
    Row row;
    bool ok = true;
    auto str = [&](const char* n, std::string& dst) {
      int c = col[n];
      if (c == -1) {
        warn(std::string("missing field `") + n + "`");
        ok = false;
      } else if (c == -2) {
        warn(std::string("duplicate field `") + n + "`");
        ok = false;
      } else {
        dst = rec[static_cast<size_t>(c)];
      }
    };
    auto num = [&](const char* n, int64_t& dst) {
      std::string s;
      str(n, s);
      if (ok && !parse_i64(s, dst)) {
        warn(std::string("field `") + n + "`: invalid digit found in string \"" + s + "\"");
        ok = false;
      }
    };
    str("name", row.name);
    if (ok) str("department", row.department);
    if (ok) str("id_username", row.id_username);
    if (ok) str("gpu_server", row.gpu_server);
    if (ok) num("gpu_request", row.gpu_request);
    if (ok) num("cpu_request", row.cpu_request);
    if (ok) num("memory_request", row.memory_request);
    if (ok) num("storage_request", row.storage_request);
    if (ok) num("mig_request", row.mig_request);
    if (ok) str("authorized", row.authorized);
    if (ok) rows.push_back(std::move(row));
  }
  return rows;
}

bool is_authorized(const Row& r) {
  // `authorized.trim().to_lowercase() == "o"` with Rust's Unicode semantics
  // (synchronizer.rs:225-236): "\u00a0O" (a Google Form's non-breaking space) is approved,
  // the fullwidth "Ｏ" is not.
  return unicode::to_lower(unicode::trim(r.authorized)) == "o";
}

Value quota_spec(const Row& r, const QuotaKeys& keys) {
  std::map<std::string, std::string> hard;  // sorted like the reference's BTreeMap
  hard["requests.cpu"] = std::to_string(r.cpu_request);
  hard["requests.memory"] = std::to_string(r.memory_request) + "Gi";
  hard["limits.cpu"] = std::to_string(r.cpu_request);
  hard["limits.memory"] = std::to_string(r.memory_request) + "Gi";
  hard["requests." + keys.gpu_resource] = std::to_string(r.gpu_request);
  hard["requests.storage"] = std::to_string(r.storage_request) + "Gi";
  hard["requests." + keys.partition_resource] = std::to_string(r.mig_request);
  Value h = Value::object();
  for (auto& [k, v] : hard) h[k] = v;
  return Value::object({{"hard", h}});
}

RowIndex::RowIndex(const std::vector<Row>& rows, const std::string& gpu_server_name) {
  for (const auto& r : rows) {
    if (r.gpu_server.find(gpu_server_name) == std::string::npos) continue;
    ++target_rows_;
    if (is_authorized(r)) by_user_[r.id_username] = r;  // later rows win (last match)
  }
}

const Row* RowIndex::find(const std::string& id_username) const {
  auto it = by_user_.find(id_username);
  return it == by_user_.end() ? nullptr : &it->second;
}

}  // namespace bgc::sync

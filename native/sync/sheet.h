// Google-Form sheet model: RFC 4180 CSV reader, Korean header inference, typed rows
// and the quota mapping.  Reference: src/synchronizer.rs:63-169 (Row, try_infer_header,
// parse_csv) and :240-286 (quota map).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "core/json.h"

namespace bgc::sync {

class CsvHeaderError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class CsvParseError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

struct Row {
  std::string name;
  std::string department;
  std::string id_username;
  std::string gpu_server;
  int64_t gpu_request = 0;
  int64_t cpu_request = 0;
  int64_t memory_request = 0;
  int64_t storage_request = 0;
  int64_t mig_request = 0;
  std::string authorized;
};

// synchronizer.rs:97-143 — first matching rule wins; unknown => CsvHeaderError.
std::string infer_header(const std::string& header);

// RFC 4180 records (quoted fields, "" escapes, CRLF/LF, empty lines skipped). Throws
// CsvParseError on an unterminated quote.
std::vector<std::vector<std::string>> parse_records(std::string_view text);

// Header row is mapped with infer_header (any failure aborts the whole parse); each data
// row that does not deserialize (wrong field count, missing column, non-i64 number) is
// skipped with a warning (synchronizer.rs:158-166).
std::vector<Row> parse_csv(std::string_view text, std::vector<std::string>* warnings = nullptr);

bool is_authorized(const Row& r);  // authorized.trim().to_lowercase() == "o"

struct QuotaKeys {
  // N4: the reference's nvidia.com keys become configurable AMD resource names.
  std::string gpu_resource = "amd.com/gpu";
  std::string partition_resource = "amd.com/gpu-partition";
};

// {"hard": {...}} with keys in sorted (BTreeMap) order.
json::Value quota_spec(const Row& r, const QuotaKeys& keys);

// id_username -> last authorized row among rows whose gpu_server contains `server`
// (substring, so "" matches everything — synchronizer.rs:208-212, :225-236).  O(1)
// lookups instead of the reference's O(rows) reverse scan per UserBootstrap.
class RowIndex {
 public:
  RowIndex() = default;
  RowIndex(const std::vector<Row>& rows, const std::string& gpu_server_name);
  const Row* find(const std::string& id_username) const;
  size_t size() const { return by_user_.size(); }
  size_t target_rows() const { return target_rows_; }

 private:
  std::unordered_map<std::string, Row> by_user_;
  size_t target_rows_ = 0;
};

}  // namespace bgc::sync

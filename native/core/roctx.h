// roctx ranges (rocprofiler-sdk) resolved at runtime so `rocprofv3 --marker-trace`
// shows the node agent's telemetry hot path; a no-op when the library is absent.
#pragma once

namespace bgc::roctx {

void push(const char* name);
void pop();
void mark(const char* name);
bool available();

class Range {
 public:
  explicit Range(const char* name) { push(name); }
  ~Range() { pop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

}  // namespace bgc::roctx

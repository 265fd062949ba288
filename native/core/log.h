// Structured logging with RUST_LOG-compatible level control.
//
// The reference initialises `tracing_subscriber::fmt` without the env-filter feature
// (reference src/controller.rs:217, Cargo.toml:41), which interprets RUST_LOG as a
// `Targets` list: "info", "warn,controller=debug", ... default INFO.  Lines look like
//   2026-01-01T00:00:00.000000Z  INFO controller: reconciling alice
#pragma once

#include <atomic>
#include <cstdint>
#include <sstream>
#include <string>
#include <string_view>

namespace bgc::log {

enum class Level : int { Trace = 0, Debug = 1, Info = 2, Warn = 3, Error = 4, Off = 5 };

// Parses a Targets spec. Unknown directives are ignored (like tracing's lenient parse
// falling back to default on error).
void init_from_env(const char* var = "RUST_LOG");
void init(const std::string& spec);
bool enabled(Level lvl, std::string_view target);
void write(Level lvl, std::string_view target, std::string_view msg);
// Redirect output (tests); nullptr restores stderr.
void set_sink(void (*sink)(const std::string& line));
// Writes buffered lines now, waiting for stderr if it is blocked (lines go to stderr in
// batches from a writer thread; an ERROR line wakes it at once; exit flushes).  Logging
// calls themselves never wait for stderr.
void flush();
// Lines dropped because 1 MiB was already waiting for a blocked stderr (process lifetime).
uint64_t lines_dropped();

class Line {
 public:
  Line(Level l, std::string_view target) : lvl_(l), target_(target) {}
  ~Line() { write(lvl_, target_, os_.str()); }
  template <typename T>
  Line& operator<<(const T& v) {
    os_ << v;
    return *this;
  }

 private:
  Level lvl_;
  std::string_view target_;
  std::ostringstream os_;
};

}  // namespace bgc::log

// for-loop form: safe inside un-braced if/else (no dangling-else), evaluates once.
#define BGC_LOG(lvl, target)                                                                    \
  for (bool bgc_log_on_ = ::bgc::log::enabled(::bgc::log::Level::lvl, target); bgc_log_on_;    \
       bgc_log_on_ = false)                                                                     \
  ::bgc::log::Line(::bgc::log::Level::lvl, target)

#define LOG_ERROR(t) BGC_LOG(Error, t)
#define LOG_WARN(t) BGC_LOG(Warn, t)
#define LOG_INFO(t) BGC_LOG(Info, t)
#define LOG_DEBUG(t) BGC_LOG(Debug, t)
#define LOG_TRACE(t) BGC_LOG(Trace, t)

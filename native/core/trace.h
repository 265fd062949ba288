// Per-object stage timestamps for the bench's per-CR latency attribution.
//
// Every process of the stack (kube-lite, controller, synchronizer, admission, the load
// driver) marks the moments a traced tenant passes through it: request received, webhook
// answered, committed, watch event delivered, reconcile started, apply sent/answered, ...
// Timestamps are CLOCK_MONOTONIC nanoseconds (metrics::now_ns), which every process on the
// host shares, so the harness joins the marks of all processes into one timeline per tenant
// (bench/attribution.py) and names the stage where an apply->Ready tail was spent.
//
// Off by default and a no-op until armed: the harness arms it per latency window with a
// name prefix (POST /debug/trace, debug endpoints only), so only that window's tenants are
// recorded and the production binaries never keep marks.  The reference has nothing of the
// kind (`tracing` log lines only).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>

namespace bgc::trace {

// Cheap check for call sites that build a stage name: false unless armed.
bool armed();
// Records (name, stage, now) when armed and `name` starts with one of the armed prefixes.
void mark(std::string_view name, std::string_view stage);
void mark_at(std::string_view name, std::string_view stage, int64_t t_ns);
// Starts recording marks of names that start with one of the comma-separated prefixes in
// `prefix` (one per bench rank), at most `capacity` of them (further marks are counted as
// dropped); clears earlier marks.  No prefix disarms.
void arm(const std::string& prefix, size_t capacity = size_t{1} << 21);
void disarm();
// {"prefix":..,"armed":bool,"dropped":n,"marks":[[name,stage,t_ns],...]}; `take` also
// clears the marks and disarms.
std::string dump_json(bool take);

}  // namespace bgc::trace

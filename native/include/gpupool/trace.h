// Per-reconcile tracing (SURVEY.md §5 "Tracing / profiling": the reference has none).
//
// Every reconcile pass runs inside a trace::Trace opened by the Controller worker. Code inside the
// pass opens trace::Span scopes ("fetch", "observe", "claim", "drain", "status", ...) or reports
// externally-measured phases with trace::add_span (e.g. the node agent's probe time returned by the
// claim RPC). On close a trace:
//   * feeds gpupool_reconcile_span_seconds{kind,span} (Prometheus histogram),
//   * is kept in a bounded ring of recent traces served as JSON at /debug/traces,
//   * is logged as one JSON line (debug level, or info when slower than the slow threshold).
// The current trace is thread-local, so spans need no plumbing through call signatures; a Span
// opened with no trace active is a no-op.
#pragma once

#include <chrono>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "gpupool/json.h"

namespace gpupool {
namespace trace {

class Trace {
 public:
  // ``key`` is the work-queue key "Kind/ns/name"; the kind prefix labels the span histogram.
  explicit Trace(std::string key);
  ~Trace();  // finishes with result "unknown" if finish() was not called
  Trace(const Trace&) = delete;
  Trace& operator=(const Trace&) = delete;

  void add(const std::string& span, double ms);
  void attr(const std::string& k, Json v) { attrs_[k] = std::move(v); }
  void finish(const std::string& result);
  const std::string& id() const { return id_; }

  static Trace* current();

 private:
  std::string id_, key_, kind_;
  std::chrono::steady_clock::time_point t0_;
  double start_unix_;
  std::vector<std::pair<std::string, double>> spans_;
  Json attrs_ = Json::object();
  bool done_ = false;
  Trace* prev_;
};

class Span {
 public:
  explicit Span(std::string name);
  ~Span();
  Span(const Span&) = delete;
  Span& operator=(const Span&) = delete;

 private:
  std::string name_;
  std::chrono::steady_clock::time_point t0_;
};

// Adds an externally measured span to the current trace (no-op without one).
void add_span(const std::string& name, double ms);
// reconcileID of the current trace, or "" outside a reconcile.
std::string current_id();
// Most recent finished traces, newest first (at most ``n``; the ring keeps 256).
Json recent(size_t n = 64);
// Traces slower than this are logged at info level (default 1 s); others at debug.
void set_slow_threshold(std::chrono::milliseconds t);
// Clears the ring (tests).
void reset();

}  // namespace trace
}  // namespace gpupool

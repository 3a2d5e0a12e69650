#include "gpupool/trace.h"

#include <atomic>
#include <cstdio>
#include <deque>
#include <mutex>
#include <random>

#include "gpupool/log.h"
#include "gpupool/metrics.h"

namespace gpupool {
namespace trace {

namespace {

thread_local Trace* tl_current = nullptr;

constexpr size_t kRing = 4096;  // a bench run's timed passes + its secondary scenarios
std::mutex g_mu;
std::deque<Json> g_ring;  // newest at front
std::atomic<int64_t> g_slow_ms{1000};

HistogramVec& span_hist() {
  static HistogramVec& h = Registry::global().histogram(
      "gpupool_reconcile_span_seconds", "Time spent in one phase (span) of a reconcile pass.",
      exponential_buckets(0.0001, 2, 20));
  return h;
}

std::string new_id() {
  // 64-bit random, hex: unique enough to correlate log lines of one pass
  static std::atomic<uint64_t> seq{0};
  thread_local std::mt19937_64 rng{std::random_device{}() ^ (seq.fetch_add(1) * 0x9E3779B97F4A7C15ull)};
  char buf[17];
  std::snprintf(buf, sizeof buf, "%016llx", static_cast<unsigned long long>(rng()));
  return buf;
}

const Logger& trace_log() {
  static const Logger l("trace");
  return l;
}

}  // namespace

Trace::Trace(std::string key)
    : id_(new_id()), key_(std::move(key)), t0_(std::chrono::steady_clock::now()),
      start_unix_(std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count()),
      prev_(tl_current) {
  kind_ = key_.substr(0, key_.find('/'));
  tl_current = this;
}

Trace::~Trace() {
  if (!done_) finish("unknown");
  tl_current = prev_;
}

Trace* Trace::current() { return tl_current; }

void Trace::add(const std::string& span, double ms) {
  spans_.emplace_back(span, ms);
  span_hist().observe({{"kind", kind_}, {"span", span}}, ms / 1e3);
}

void Trace::finish(const std::string& result) {
  if (done_) return;
  done_ = true;
  double total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0_).count();
  Json spans = Json::array();
  for (const auto& [name, ms] : spans_) {
    Json s = Json::object();
    s["name"] = name;
    s["ms"] = ms;
    spans.push_back(std::move(s));
  }
  Json rec = Json::object();
  rec["reconcileID"] = id_;
  rec["key"] = key_;
  rec["start"] = start_unix_;
  rec["totalMs"] = total;
  rec["result"] = result;
  rec["spans"] = spans;
  if (attrs_.size() > 0) rec["attrs"] = attrs_;
  {
    std::lock_guard<std::mutex> g(g_mu);
    g_ring.push_front(rec);
    if (g_ring.size() > kRing) g_ring.pop_back();
  }
  LogLevel lvl = total >= static_cast<double>(g_slow_ms.load()) ? LogLevel::Info : LogLevel::Debug;
  trace_log().log(lvl, "reconcile trace", rec);
}

Span::Span(std::string name) : name_(std::move(name)), t0_(std::chrono::steady_clock::now()) {}

Span::~Span() {
  if (Trace* t = Trace::current())
    t->add(name_, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0_).count());
}

void add_span(const std::string& name, double ms) {
  if (Trace* t = Trace::current()) t->add(name, ms);
}

std::string current_id() {
  Trace* t = Trace::current();
  return t ? t->id() : std::string();
}

Json recent(size_t n) {
  std::lock_guard<std::mutex> g(g_mu);
  Json out = Json::array();
  for (size_t i = 0; i < g_ring.size() && i < n; ++i) out.push_back(g_ring[i]);
  return out;
}

void set_slow_threshold(std::chrono::milliseconds t) { g_slow_ms = t.count(); }

void reset() {
  std::lock_guard<std::mutex> g(g_mu);
  g_ring.clear();
}

}  // namespace trace
}  // namespace gpupool

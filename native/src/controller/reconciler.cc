// Pool reconciler base (status writes, finalizers, events, readiness metrics) and the
// Controller (work queue + workers). The kinds: mi355x_pool.cc, azure_pool.cc, job.cc.
#include "gpupool/reconciler.h"

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <random>
#include <sstream>

#include "gpupool/generated/schema_consts.h"
#include "gpupool/leader.h"
#include "reconcile_util.h"

namespace gpupool {

using namespace recutil;

namespace recutil {
std::string join(const std::vector<std::string>& v, const char* sep) {
  std::string out;
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) out += sep;
    out += v[i];
  }
  return out;
}

std::string short_id(const DeviceView& d) {
  std::string u = !d.hip_uuid.empty() ? d.hip_uuid : d.uuid;
  return u + "(#" + std::to_string(d.index) + ")";
}

HistogramVec& reconcile_hist() {
  static HistogramVec& h = Registry::global().histogram(
      "gpupool_reconcile_duration_seconds", "Time spent in one reconcile pass.", exponential_buckets(0.0005, 2, 18));
  return h;
}
HistogramVec& to_ready_hist() {
  static HistogramVec& h = Registry::global().histogram(
      "gpupool_reconcile_to_ready_seconds",
      "From the first reconcile of a spec generation to the status write that reports it Ready.",
      exponential_buckets(0.001, 2, 18));
  return h;
}
CounterVec& reconcile_total() {
  static CounterVec& c = Registry::global().counter("gpupool_reconcile_total", "Reconcile passes by kind and result.");
  return c;
}
GaugeVec& ready_gauge() {
  static GaugeVec& g = Registry::global().gauge("gpupool_ready_replicas", "status.readyReplicas per pool.");
  return g;
}
GaugeVec& quota_gauge() {
  static GaugeVec& g = Registry::global().gauge(
      "gpupool_namespace_quota_units",
      "Namespace ResourceQuota of a pool resource (type=hard) and the units pools use or reserve (type=used).");
  return g;
}
GaugeVec& desired_gauge() {
  static GaugeVec& g = Registry::global().gauge("gpupool_desired_replicas", "spec.replicas per pool.");
  return g;
}

// Pool-level GPU utilisation (Prometheus + Grafana, GPU调度平台搭建.md:800), aggregated from the
// agents' telemetry of the pool's claimed GPUs at every reconcile pass (steady-state resync).
struct UtilGauges {
  GaugeVec& gfx = Registry::global().gauge("gpupool_pool_gfx_activity_percent",
                                           "Mean GFX (compute) activity of the pool's GPUs.");
  GaugeVec& umc = Registry::global().gauge("gpupool_pool_umc_activity_percent",
                                           "Mean memory-controller (HBM) activity of the pool's GPUs.");
  GaugeVec& power = Registry::global().gauge("gpupool_pool_power_watts", "Summed socket power of the pool's GPUs.");
  GaugeVec& vram_used = Registry::global().gauge("gpupool_pool_vram_used_bytes", "Summed VRAM in use on the pool's GPUs.");
  GaugeVec& vram_total = Registry::global().gauge("gpupool_pool_vram_total_bytes", "Summed VRAM of the pool's GPUs.");
};
UtilGauges& util_gauges() {
  static UtilGauges g;
  return g;
}

void set_util_gauges(const Labels& l, const std::vector<DeviceView>& mine) {
  double gfx = 0, umc = 0, power = 0, used = 0, total = 0;
  int n = 0;
  for (const auto& d : mine) {
    if (!d.telemetry.is_object()) continue;
    ++n;
    gfx += d.telemetry["gfxActivity"].as_double(0);
    umc += d.telemetry["umcActivity"].as_double(0);
    power += d.telemetry["powerW"].as_double(0);
    used += d.telemetry["memUsedBytes"].as_double(0);
    total += d.telemetry["memTotalBytes"].as_double(0);
  }
  UtilGauges& g = util_gauges();
  g.gfx.set(l, n ? gfx / n : 0);
  g.umc.set(l, n ? umc / n : 0);
  g.power.set(l, power);
  g.vram_used.set(l, used);
  g.vram_total.set(l, total);
}

void erase_util_gauges(const Labels& l) {
  UtilGauges& g = util_gauges();
  for (GaugeVec* v : {&g.gfx, &g.umc, &g.power, &g.vram_used, &g.vram_total}) v->erase(l);
}
}  // namespace recutil

// ================================================================== base
PoolReconcilerBase::PoolReconcilerBase(KubeClient& client, Informer& pools, EventRecorder* events,
                                       ReconcilerOptions opts, std::string kind, ResourceRef res)
    : client_(client), pools_(pools), events_(events), opts_(opts), kind_(std::move(kind)), res_(std::move(res)),
      finalizer_(gen::kFinalizer), log_(Logger("reconciler").with("kind", kind_)) {}

void PoolReconcilerBase::write_status_(const Json& obj, const Json& status) {
  trace::Span span("status");
  if (!leader_fence_ok()) throw std::runtime_error("not writing status: leadership not renewed in time");
  Json cur = obj;
  const std::string ns = obj.path("metadata.namespace").as_string();
  const std::string name = obj.path("metadata.name").as_string();
  if (cur["status"] == status) return;  // semantically unchanged: no write, no watch churn
  for (int attempt = 0; attempt < 6; ++attempt) {
    Json upd = cur;
    upd["status"] = status;
    try {
      Json out = client_.update(res_, ns, upd, "status");
      std::vector<std::string> place{status["nodeName"].as_string()};
      for (const auto& n : status["nodes"].elements()) place.push_back(n.as_string());
      const std::string uid = out.path("metadata.uid").as_string();
      {
        std::lock_guard<std::mutex> g(mu_);
        own_rv_[uid] = out.path("metadata.resourceVersion").as_string();
        own_place_[uid] = std::move(place);
      }
      on_status_written_(out);
      return;
    } catch (const KubeError& e) {
      if (!e.conflict()) throw;
      cur = client_.get(res_, ns, name);  // fresh read, then re-apply our status
      if (cur["status"] == status) return;
      Json mine = Json::object();
      mine["status"] = status;
      stale_placement_check_(obj, cur, &mine);
    }
  }
  throw KubeError(409, "Conflict", "status update kept conflicting for " + ns + "/" + name);
}

// A pass observes where the pool's GPUs live from status.nodeName / status.nodes of the object it
// read. When the informer served an object older than the stored one (it lags this reconciler's
// own writes) and the stored placement differs, every conclusion of the pass may be wrong — e.g.
// "no GPUs anywhere" when the named node's agent is down but the stale copy named no node. Such a
// pass must not land its status or drop its finalizer: it fails with a conflict and re-runs on the
// fresh object. Same placement — or a status write whose own placement matches the fresh one (the
// pass found the GPUs where they are, the usual case right after this reconciler's own write) —
// and the write is retried.
void PoolReconcilerBase::stale_placement_check_(const Json& seen, const Json& fresh, const Json* writing) {
  auto placement = [](const Json& o) {
    std::vector<std::string> p{o.path("status.nodeName").as_string()};
    for (const auto& n : o.path("status.nodes").elements()) p.push_back(n.as_string());
    return p;
  };
  const auto now = placement(fresh);
  if (placement(seen) != now && !(writing && placement(*writing) == now))
    throw KubeError(409, "Conflict",
                    "pass ran on a stale copy of " + fresh.path("metadata.namespace").as_string() + "/" +
                        fresh.path("metadata.name").as_string() + " (status placement changed): re-running");
}

bool PoolReconcilerBase::own_status_write(const Json& obj) {
  const std::string uid = obj.path("metadata.uid").as_string();
  std::lock_guard<std::mutex> g(mu_);
  auto it = own_rv_.find(uid);
  return it != own_rv_.end() && !it->second.empty() && it->second == obj.path("metadata.resourceVersion").as_string();
}

// Finalizer edits carry the object's resourceVersion (the list is replaced as a whole, so a
// concurrent edit must not be lost). The informer cache can lag the apiserver — most often behind
// this reconciler's own status write — and a stale version is a 409: then the object is read
// fresh and the edit retried against it, instead of failing the pass into rate-limited backoff
// until the watch catches up (seen as hundreds of 409s when 48 pools were created at once).
Json PoolReconcilerBase::edit_finalizers_(const Json& obj, bool add) {
  Json cur = obj;
  for (int attempt = 0;; ++attempt) {
    ObjectMeta m = ObjectMeta::from(cur);
    if (m.has_finalizer(finalizer_) == add) return cur;
    Json fins = Json::array();
    for (const auto& f : m.finalizers)
      if (f != finalizer_) fins.push_back(f);
    if (add) fins.push_back(finalizer_);
    Json patch = Json::object();
    patch["metadata"]["finalizers"] = fins;
    patch["metadata"]["resourceVersion"] = m.resource_version;  // optimistic concurrency
    try {
      return client_.patch_merge(res_, m.ns, m.name, patch);
    } catch (const KubeError& e) {
      if (!e.conflict() || attempt >= 3) throw;
      cur = client_.get(res_, m.ns, m.name);
      if (!add) stale_placement_check_(obj, cur);  // removal was decided from obj's placement
    }
  }
}

Json PoolReconcilerBase::ensure_finalizer_(const Json& obj) {
  if (ObjectMeta::from(obj).has_finalizer(finalizer_)) return obj;
  trace::Span span("finalizer");
  return edit_finalizers_(obj, true);
}

Json PoolReconcilerBase::remove_finalizer_(const Json& obj) { return edit_finalizers_(obj, false); }

// The stored object, read through the API server: a status written from what the pass could NOT
// observe (an unreachable agent) is built on the newest status — the informer copy may predate this
// reconciler's own last write and would carry no devices to keep. Falls back to ``obj``.
Json PoolReconcilerBase::fresh_(const Json& obj) {
  try {
    Json cur = client_.get(res_, obj.path("metadata.namespace").as_string(), obj.path("metadata.name").as_string());
    if (cur.path("metadata.uid") == obj.path("metadata.uid")) return cur;
  } catch (const std::exception&) {
  }
  return obj;
}

void PoolReconcilerBase::event_(const Json& obj, const std::string& type, const std::string& reason,
                                const std::string& msg) {
  if (events_ && opts_.emit_events) events_->record(obj, type, reason, msg);
}

void PoolReconcilerBase::note_generation_(const ObjectMeta& m) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = pending_.find(m.uid);
  if (it == pending_.end() || it->second.first != m.generation) pending_[m.uid] = {m.generation, clock_t_::now()};
}

void PoolReconcilerBase::observe_ready_(const ObjectMeta& m, bool ready, int64_t desired) {
  Labels l{{"kind", kind_}, {"pool", m.key()}};
  desired_gauge().set(l, static_cast<double>(desired));
  note_generation_(m);
  std::lock_guard<std::mutex> g(mu_);
  auto it = pending_.find(m.uid);
  if (ready && ready_gen_[m.uid] != m.generation) {
    ready_gen_[m.uid] = m.generation;
    double s = std::chrono::duration<double>(clock_t_::now() - it->second.second).count();
    to_ready_hist().observe({{"kind", kind_}}, s);
    log_.info("pool ready", Json::object().set("pool", m.key()).set("generation", m.generation).set("reconcileToReadySeconds", s));
  }
}

void PoolReconcilerBase::forget_(const std::string& uid) {
  std::lock_guard<std::mutex> g(mu_);
  pending_.erase(uid);
  ready_gen_.erase(uid);
  own_rv_.erase(uid);
  own_place_.erase(uid);
}

std::vector<std::string> PoolReconcilerBase::written_placement_(const std::string& uid) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = own_place_.find(uid);
  return it == own_place_.end() ? std::vector<std::string>{} : it->second;
}

// ================================================================== Controller
Controller::Controller(int workers) : workers_(workers) {}

Controller::~Controller() { stop(); }

void Controller::add_reconciler(PoolReconcilerBase* r) { by_kind_[r->kind()] = r; }

void Controller::enqueue(const std::string& kind, const std::string& ns, const std::string& name) {
  q_.add(kind + "/" + ns + "/" + name);
}

void Controller::enqueue_after(const std::string& kind, const std::string& ns, const std::string& name, ms d) {
  q_.add_after(kind + "/" + ns + "/" + name, d);
}

void Controller::start() {
  for (int i = 0; i < workers_; ++i) threads_.emplace_back([this] { worker_(); });
}

void Controller::stop() {
  q_.shutdown();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
}

void Controller::worker_() {
  std::string key;
  double waited_ms = 0;
  while (q_.get(&key, &waited_ms)) {
    auto s1 = key.find('/');
    auto s2 = key.find('/', s1 + 1);
    std::string kind = key.substr(0, s1), ns = key.substr(s1 + 1, s2 - s1 - 1), name = key.substr(s2 + 1);
    auto it = by_kind_.find(kind);
    if (it == by_kind_.end()) {
      q_.forget(key);
      q_.done(key);
      continue;
    }
    if (!leader_fence_ok()) {  // paused past the renew deadline: another replica may lead now
      q_.forget(key);
      q_.add_after(key, std::chrono::milliseconds(500));
      q_.done(key);
      continue;
    }
    auto t0 = clock_t_::now();
    Outcome out;
    static const char* names[] = {"done", "requeue", "error", "terminal"};
    {
      trace::Trace tr(key);
      tr.attr("queueWaitMs", waited_ms);  // ready in the work queue -> this worker took it
      waited_ms = 0;
      try {
        out = it->second->reconcile(ns, name);
      } catch (const std::exception& e) {
        out = Outcome::transient(e.what());
      }
      if (!out.message.empty()) tr.attr("reason", out.message);
      tr.finish(names[out.kind]);
    }
    double secs = std::chrono::duration<double>(clock_t_::now() - t0).count();
    reconciles_++;
    reconcile_total().inc({{"kind", kind}, {"result", names[out.kind]}});
    reconcile_hist().observe({{"kind", kind}}, secs);
    switch (out.kind) {
      case Outcome::Done:
        q_.forget(key);
        if (out.after.count() > 0) q_.add_after(key, out.after);
        break;
      case Outcome::RequeueAfter:
        q_.forget(key);
        q_.add_after(key, out.after);
        break;
      case Outcome::Transient:
        log_.warn("reconcile failed; backing off",
                  Json::object().set("key", key).set("error", out.message).set("requeues", q_.num_requeues(key)));
        q_.add_rate_limited(key);
        break;
      case Outcome::Terminal:
        log_.warn("reconcile terminal; waiting for a spec change", Json::object().set("key", key).set("reason", out.message));
        q_.forget(key);
        break;
    }
    q_.done(key);
  }
}

}  // namespace gpupool

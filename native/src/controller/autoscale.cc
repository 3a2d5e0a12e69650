// Mi355xPoolAutoscaler — see the class comment in reconciler.h.
#include <algorithm>

#include "gpupool/generated/schema_consts.h"
#include "gpupool/reconciler.h"
#include "job_util.h"

namespace gpupool {

namespace {

using ms = std::chrono::milliseconds;
using namespace detail;

CounterVec& scale_events() {
  static CounterVec& c = Registry::global().counter("gpupool_autoscale_total",
                                                    "Mi355xPool autoscaler spec.replicas changes by direction.");
  return c;
}
GaugeVec& demand_gauge() {
  static GaugeVec& g =
      Registry::global().gauge("gpupool_autoscale_demand_gpus", "GPU demand the autoscaler sees per pool.");
  return g;
}

// Waiting gangs that admission (not capacity) holds back add no demand: more GPUs would not help.
bool admission_blocked(const Json& job) {
  for (const auto& c : job.path("status.conditions").elements())
    if (c["type"].as_string() == gen::kCondScheduled) {
      const std::string r = c["reason"].as_string();
      return r == "QueueClosed" || r == "QueueOverCapacity" || r == "QueueNotFound";
    }
  return false;
}

}  // namespace

Mi355xPoolAutoscaler::Mi355xPoolAutoscaler(KubeClient& client, Informer& pools, Informer& jobs, Informer& pods,
                                           EventRecorder* events, ReconcilerOptions opts)
    : PoolReconcilerBase(client, pools, events, opts, "Mi355xPoolAutoscale", res::mi355xpools()),
      jobs_(jobs),
      pods_(pods) {}

std::vector<std::pair<std::string, std::string>> Mi355xPoolAutoscaler::autoscaled() const {
  std::vector<std::pair<std::string, std::string>> out;
  for (const auto& p : pools_.list())
    if (p.path("spec.autoscale.enabled").as_bool(false))
      out.emplace_back(p.path("metadata.namespace").as_string(), p.path("metadata.name").as_string());
  return out;
}

int64_t Mi355xPoolAutoscaler::demand(const std::vector<Json>& pods, const std::vector<Json>& jobs,
                                     const std::string& ns, const std::string& pool, const std::string& resource) {
  int64_t total = 0;
  for (const auto& p : pods) {
    if (terminal(pod_phase(p)) || !p.path("metadata.deletionTimestamp").as_string().empty()) continue;
    total += pod_request(p, resource);
  }
  for (const auto& j : jobs) {
    const std::string phase = j.path("status.phase").str_or("Pending");
    if (terminal(phase) || phase == "Suspended" || j.path("spec.suspend").as_bool(false)) continue;
    if (!j.path("metadata.deletionTimestamp").as_string().empty()) continue;
    const bool mine = j.path("spec.poolRef").as_string() == pool && j.path("metadata.namespace").as_string() == ns;
    if (!mine && job_resource(j, gen::kDefaultResource) != resource) continue;
    const int64_t g = j.path("spec.gpusPerReplica").as_int(1);
    const Json& placement = j.path("status.placement");
    if (placement.size() == 0) {
      if (!admission_blocked(j)) total += g * j.path("spec.replicas").as_int(1);  // gang still waiting
    } else {
      for (const auto& s : placement.elements())
        if (!s["created"].as_bool(false)) total += g;  // reserved slot, pod not created yet
    }
  }
  return total;
}

Outcome Mi355xPoolAutoscaler::reconcile(const std::string& ns, const std::string& name) {
  auto cached = pools_.get(ns, name);
  if (!cached) return Outcome::done(ms(0));
  const Json& obj = *cached;
  ObjectMeta m = ObjectMeta::from(obj);
  Mi355xPoolSpec spec = Mi355xPoolSpec::from(obj["spec"]);
  if (m.deleting() || !spec.autoscale) {
    std::lock_guard<std::mutex> g(mu_);
    low_since_.erase(m.uid);
    return Outcome::done(ms(0));
  }
  const int64_t d = demand(pods_.list(), jobs_.list(), m.ns, m.name, spec.resource_name);
  const int64_t lo = spec.autoscale_min, hi = std::max(spec.autoscale_min, spec.autoscale_max);
  const int64_t target = std::clamp(d, lo, hi);
  demand_gauge().set({{"pool", m.key()}}, static_cast<double>(d));
  const auto now = std::chrono::steady_clock::now();
  ms wait{0};
  {
    // The delay runs from the first pass that saw demand below spec.replicas (a long-idle steady
    // state must not make a later drop shrink the pool at once); any pass at or above resets it.
    std::lock_guard<std::mutex> g(mu_);
    if (target >= spec.replicas) {
      low_since_.erase(m.uid);
    } else {
      auto it = low_since_.emplace(m.uid, now).first;
      const auto due = it->second + std::chrono::seconds(spec.scale_down_delay_seconds);
      if (now < due) wait = std::chrono::duration_cast<ms>(due - now) + ms(20);
    }
  }
  if (target == spec.replicas) return Outcome::done(opts_.resync);
  if (wait.count() > 0) return Outcome::requeue(wait, "scale-down delay");
  const bool up = target > spec.replicas;
  Json patch = Json::object();
  patch["spec"]["replicas"] = target;
  patch["metadata"]["annotations"][gen::kAnnAutoscaleLast] = rfc3339_now();
  patch["metadata"]["annotations"][gen::kAnnAutoscaleDemand] = std::to_string(d);
  client_.patch_merge(res_, m.ns, m.name, patch);
  const std::string msg = "replicas " + std::to_string(spec.replicas) + " -> " + std::to_string(target) + " (demand " +
                          std::to_string(d) + " " + spec.resource_name + ", bounds [" + std::to_string(lo) + ", " +
                          std::to_string(hi) + "])";
  event_(obj, "Normal", up ? "AutoscaledUp" : "AutoscaledDown", msg);
  scale_events().inc({{"direction", up ? "up" : "down"}});
  log_.info("autoscaled",
            Json::object().set("pool", m.key()).set("from", spec.replicas).set("to", target).set("demand", d));
  {
    std::lock_guard<std::mutex> g(mu_);
    low_since_.erase(m.uid);
  }
  return Outcome::done(opts_.resync);
}

}  // namespace gpupool

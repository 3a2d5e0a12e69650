// Mi355xPoolAutoscaler — see the class comment in reconciler.h.
#include <algorithm>
#include <map>

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
    const std::string ref = j.path("spec.poolRef").as_string();
    const bool mine = ref == pool && j.path("metadata.namespace").as_string() == ns;
    // a gang bound to another pool by poolRef is that pool's demand, never this one's
    if (!mine && (!ref.empty() || job_resource(j, gen::kDefaultResource) != resource)) continue;
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

int64_t Mi355xPoolAutoscaler::pool_demand(const std::vector<Json>& pods, const std::vector<Json>& jobs,
                                           const std::vector<Json>& pools, const std::string& ns,
                                           const std::string& pool, const std::string& resource) {
  // explicit(Q): gangs with poolRef == Q; shared: pods of the resource + gangs without a poolRef
  auto is_job_of = [](const Json& j, const std::string& qns, const std::string& qname) {
    return j.path("spec.poolRef").as_string() == qname && j.path("metadata.namespace").as_string() == qns;
  };
  auto explicit_of = [&](const std::string& qns, const std::string& qname) {
    std::vector<Json> mine;
    for (const auto& j : jobs)
      if (is_job_of(j, qns, qname)) mine.push_back(j);
    return demand({}, mine, qns, qname, resource);
  };
  std::vector<Json> unbound;
  for (const auto& j : jobs)
    if (j.path("spec.poolRef").as_string().empty()) unbound.push_back(j);
  // A pod already running on a pool's GPUs (status.devices[].pods, from the agents' PodResources
  // view) is that pool's demand: attributing it to whichever pool comes first in the split would
  // grow an idle pool while the one it runs on looks over-provisioned and drains it.
  std::map<std::string, std::string> pod_pool;  // "ns/pod" -> "ns/pool"
  for (const auto& q : pools) {
    if (q.path("spec.resourceName").str_or(gen::kDefaultResource) != resource) continue;
    const std::string qkey = q.path("metadata.namespace").as_string() + "/" + q.path("metadata.name").as_string();
    for (const auto& d : q.path("status.devices").elements())
      for (const auto& pk : d["pods"].elements()) pod_pool[pk.as_string()] = qkey;
  }
  std::map<std::string, int64_t> bound;  // "ns/pool" -> GPUs its running pods use
  std::vector<Json> pending;
  for (const auto& p : pods) {
    auto it = pod_pool.find(p.path("metadata.namespace").as_string() + "/" + p.path("metadata.name").as_string());
    if (it == pod_pool.end()) {
      pending.push_back(p);
    } else if (!terminal(pod_phase(p)) && p.path("metadata.deletionTimestamp").as_string().empty()) {
      bound[it->second] += pod_request(p, resource);
    }
  }
  int64_t remaining = demand(pending, unbound, "", "", resource);
  // fixed-size pools of the same resource serve shared demand first (whatever their own gangs
  // leave free); what is left is split over the autoscaled pools in (namespace, name) order up to
  // each one's maxReplicas, so two autoscaled pools never both grow for the same pods
  struct Auto {
    std::string ns, name;
    int64_t cap, expl;
  };
  std::vector<Auto> autos;
  for (const auto& q : pools) {
    if (q.path("spec.resourceName").str_or(gen::kDefaultResource) != resource) continue;
    if (!q.path("metadata.deletionTimestamp").as_string().empty()) continue;
    const std::string qns = q.path("metadata.namespace").as_string(), qname = q.path("metadata.name").as_string();
    const int64_t expl = explicit_of(qns, qname) + bound[qns + "/" + qname];
    // capacities in devices of the resource: a shared GPU offers sharing.replicasPerGPU of them
    const int64_t k = std::max<int64_t>(1, q.path("spec.sharing.replicasPerGPU").as_int(1));
    if (q.path("spec.autoscale.enabled").as_bool(false)) {
      const int64_t hi = std::max(q.path("spec.autoscale.minReplicas").as_int(0), q.path("spec.autoscale.maxReplicas").as_int(0));
      autos.push_back({qns, qname, std::max<int64_t>(0, hi * k - expl), expl});
    } else {
      remaining -= std::max<int64_t>(0, q.path("spec.replicas").as_int(0) * k - expl);
    }
  }
  remaining = std::max<int64_t>(0, remaining);
  std::sort(autos.begin(), autos.end(),
            [](const Auto& a, const Auto& b) { return a.ns != b.ns ? a.ns < b.ns : a.name < b.name; });
  for (size_t i = 0; i < autos.size(); ++i) {
    const Auto& a = autos[i];
    // the last pool in order takes all that is left (its own maxReplicas clamps it later), so a
    // single pool's demand is exactly demand() and the overflow stays visible
    const int64_t share = i + 1 == autos.size() ? remaining : std::min(remaining, a.cap);
    remaining -= share;
    if (a.ns == ns && a.name == pool) return a.expl + share;
  }
  return explicit_of(ns, pool) + bound[ns + "/" + pool];  // not (yet) in the pool list
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
  const int64_t d = pool_demand(pods_.list(), jobs_.list(), pools_.list(), m.ns, m.name, spec.resource_name);
  const int64_t lo = spec.autoscale_min, hi = std::max(spec.autoscale_min, spec.autoscale_max);
  // demand is in devices of the resource; a shared GPU (sharing.replicasPerGPU = K) serves K of them
  const int64_t k = std::max<int32_t>(1, spec.sharing_replicas);
  const int64_t target = std::clamp((d + k - 1) / k, lo, hi);
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

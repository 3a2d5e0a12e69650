// Mi355xJobReconciler — gang-scheduled distributed training jobs on pool-advertised MI355X GPUs.
//
// Reference behaviour being replaced: a Volcano Job
// (GPU调度平台搭建.md:643-672: `minAvailable`, `schedulerName: volcano`, `queue: default`,
// `restartPolicy: OnFailure`, `nvidia.com/gpu: 1`) run through the Kubeflow Training Operator
// (:300-306) whose PET_* env the workload inspects to pick single vs distributed mode (:623-630).
// Here one controller does gang placement, rendezvous wiring and gang restarts; see the class
// comment in reconciler.h for the contract.
#include <algorithm>
#include <cstdlib>
#include <set>
#include <tuple>

#include "gpupool/generated/schema_consts.h"
#include "gpupool/reconciler.h"
#include "job_util.h"

namespace gpupool {

namespace {

using ms = std::chrono::milliseconds;

CounterVec& job_events() {
  static CounterVec& c = Registry::global().counter("gpupool_job_transitions_total",
                                                    "Mi355xJob lifecycle transitions by kind.");
  return c;
}
GaugeVec& queue_jobs_gauge() {
  static GaugeVec& g = Registry::global().gauge("gpupool_queue_jobs", "Mi355xJobs per queue and phase.");
  return g;
}
GaugeVec& queue_alloc_gauge() {
  static GaugeVec& g = Registry::global().gauge("gpupool_queue_allocated_gpus",
                                                "GPUs held by a queue's placed jobs, per extended resource.");
  return g;
}
HistogramVec& gang_wait_hist() {
  static HistogramVec& h = Registry::global().histogram(
      "gpupool_job_gang_wait_seconds", "From job creation (or gang restart) to its gang placement.",
      exponential_buckets(0.001, 2, 20));
  return h;
}

using namespace detail;

std::string pod_name(const std::string& job, int index) { return job + "-worker-" + std::to_string(index); }

int label_int(const Json& pod, const char* key, int def) {
  const std::string& v = pod.path("metadata.labels")[key].as_string();
  return v.empty() ? def : std::atoi(v.c_str());
}

bool selector_matches(const std::map<std::string, std::string>& sel, const Json& node) {
  const Json& labels = node.path("metadata.labels");
  for (const auto& kv : sel)
    if (labels[kv.first].as_string() != kv.second) return false;
  return true;
}

bool node_schedulable(const Json& node) {
  if (node.path("spec.unschedulable").as_bool(false)) return false;
  for (const auto& c : node.path("status.conditions").elements())
    if (c["type"].as_string() == "Ready" && c["status"].as_string() == "False") return false;
  return true;
}

}  // namespace

Mi355xJobReconciler::Mi355xJobReconciler(KubeClient& client, Informer& jobs, Informer& nodes, EventRecorder* events,
                                         ReconcilerOptions opts, PodIndex* pods)
    : PoolReconcilerBase(client, jobs, events, opts, "Mi355xJob",
                         ResourceRef{gen::kGroup, gen::kVersion, gen::kPluralMi355xJob, true, "Mi355xJob"}),
      nodes_(nodes), pods_idx_(pods) {
  finalizer_ = gen::kJobFinalizer;
}

namespace {
// resourceVersions are opaque to clients, but every apiserver backend in use (etcd, the sim)
// issues increasing integers: compare them as such, and treat anything else as "not newer"
bool rv_newer(const std::string& a, const std::string& b) {
  char* ea = nullptr;
  char* eb = nullptr;
  const long long x = std::strtoll(a.c_str(), &ea, 10), y = std::strtoll(b.c_str(), &eb, 10);
  return !a.empty() && !b.empty() && *ea == 0 && *eb == 0 && x > y;
}

CounterVec& sched_reads() {
  static CounterVec& c = Registry::global().counter(
      "gpupool_job_scheduler_reads_total", "Object reads of the gang scheduler by source (cache or apiserver LIST).");
  return c;
}
}  // namespace

void Mi355xJobReconciler::wake_blocked_by_(const std::string& key) {
  std::vector<std::string> wake;
  {
    std::lock_guard<std::mutex> g(blocked_mu_);
    for (auto it = blocked_by_.begin(); it != blocked_by_.end();) {
      if (it->second == key) {
        wake.push_back(it->first);
        it = blocked_by_.erase(it);
      } else {
        ++it;
      }
    }
  }
  if (!waker_) return;
  for (const auto& w : wake) {
    const auto slash = w.find('/');
    waker_(w.substr(0, slash), w.substr(slash + 1));
  }
}

void Mi355xJobReconciler::on_status_written_(const Json& written) {
  if (!pods_idx_) return;
  std::lock_guard<std::mutex> g(written_mu_);
  written_[written.path("metadata.uid").as_string()] = written;
}

std::vector<Json> Mi355xJobReconciler::jobs_view_() {
  if (!pods_idx_) {
    sched_reads().inc({{"what", "jobs"}, {"source", "list"}});
    Json lst = client_.list(res_, "");
    return std::vector<Json>(lst["items"].elements().begin(), lst["items"].elements().end());
  }
  sched_reads().inc({{"what", "jobs"}, {"source", "cache"}});
  std::vector<Json> out = pools_.list();
  std::lock_guard<std::mutex> g(written_mu_);
  std::set<std::string> seen;
  for (auto& j : out) {
    const std::string uid = j.path("metadata.uid").as_string();
    seen.insert(uid);
    auto w = written_.find(uid);
    if (w == written_.end()) continue;
    if (rv_newer(w->second.path("metadata.resourceVersion").as_string(), j.path("metadata.resourceVersion").as_string()))
      j = w->second;  // the watch has not delivered our write yet
    else
      written_.erase(w);  // the cache caught up (or moved past it)
  }
  for (auto it = written_.begin(); it != written_.end();)  // deleted jobs
    it = seen.count(it->first) ? std::next(it) : written_.erase(it);
  return out;
}

std::vector<Json> Mi355xJobReconciler::node_objects_() {
  if (!pods_idx_) {
    sched_reads().inc({{"what", "nodes"}, {"source", "list"}});
    Json lst = client_.list(res::nodes());
    return std::vector<Json>(lst["items"].elements().begin(), lst["items"].elements().end());
  }
  sched_reads().inc({{"what", "nodes"}, {"source", "cache"}});
  return nodes_.list();
}

std::map<std::string, int64_t> Mi355xJobReconciler::pod_usage_(const std::string& resource) {
  if (pods_idx_) {
    sched_reads().inc({{"what", "pods"}, {"source", "cache"}});
    return pods_idx_->requested_by_node(resource);
  }
  sched_reads().inc({{"what", "pods"}, {"source", "list"}});
  std::map<std::string, int64_t> used;
  Json pods = client_.list(res::pods(), "");
  for (const auto& p : pods["items"].elements()) {
    const std::string node = p.path("spec.nodeName").as_string();
    if (node.empty() || terminal(pod_phase(p))) continue;
    used[node] += pod_request(p, resource);
  }
  return used;
}

std::vector<std::pair<std::string, std::string>> Mi355xJobReconciler::pending() const {
  std::vector<std::pair<std::string, std::string>> out;
  for (const auto& j : pools_.list()) {
    const std::string phase = j.path("status.phase").str_or("Pending");
    if (phase == "Pending" || phase == "Restarting")
      out.emplace_back(j.path("metadata.namespace").as_string(), j.path("metadata.name").as_string());
  }
  return out;
}

std::vector<Mi355xJobReconciler::Slot> Mi355xJobReconciler::place(
    const std::vector<std::pair<std::string, int64_t>>& free, int replicas, int64_t gpus) {
  std::vector<Slot> out;
  if (free.empty() || replicas <= 0) return out;
  if (gpus <= 0) {  // CPU-only workers: no capacity to account, keep them together on the first node
    for (int i = 0; i < replicas; ++i) out.push_back({i, free.front().first});
    return out;
  }
  const int64_t need = gpus * replicas;
  // Whole gang on one node (xGMI between every pair of its GPUs): the tightest node that fits.
  const std::pair<std::string, int64_t>* best = nullptr;
  for (const auto& f : free)
    if (f.second >= need && (!best || f.second < best->second)) best = &f;
  if (best) {
    for (int i = 0; i < replicas; ++i) out.push_back({i, best->first});
    return out;
  }
  // Otherwise the fewest nodes: fill the roomiest first. Rank 0 lands on the first node.
  std::vector<std::pair<std::string, int64_t>> order(free.begin(), free.end());
  std::stable_sort(order.begin(), order.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
  int i = 0;
  for (auto& f : order) {
    while (i < replicas && f.second >= gpus) {
      out.push_back({i++, f.first});
      f.second -= gpus;
    }
    if (i == replicas) return out;
  }
  return {};
}

std::vector<Json> Mi355xJobReconciler::list_pods_(const ObjectMeta& m, const Json& placement) {
  std::vector<Json> out;
  std::vector<Json> items;
  bool use_list = !pods_idx_;
  if (pods_idx_) {
    items = pods_idx_->job_pods(m.ns, m.name);
    // a pod the job's (fresh) status says was created but the cache does not show yet (or any
    // more): ask the apiserver before concluding it is lost — a stale cache must never restart
    // a gang
    std::set<int> cached;
    for (const auto& p : items) cached.insert(label_int(p, gen::kLabelJobIndex, -1));
    for (const auto& sl : placement.elements())
      use_list = use_list || (sl["created"].as_bool(false) && !cached.count(static_cast<int>(sl["index"].as_int(-1))));
  }
  sched_reads().inc({{"what", "job-pods"}, {"source", use_list ? "list" : "cache"}});
  if (use_list) {
    Json lst = client_.list(res::pods(), m.ns, std::string(gen::kLabelJob) + "=" + m.name);
    items.assign(lst["items"].elements().begin(), lst["items"].elements().end());
  }
  for (const auto& p : items) {
    bool owned = false;
    for (const auto& o : p.path("metadata.ownerReferences").elements())
      owned = owned || o["uid"].as_string() == m.uid;
    if (owned) out.push_back(p);
  }
  return out;
}

bool Mi355xJobReconciler::resolve_pool_(const ObjectMeta& m, const Mi355xJobSpec& spec, std::string* resource,
                                        std::string* node, std::string* why,
                                        std::map<std::string, int64_t>* pool_cap) {
  *resource = spec.resource_name.empty() ? gen::kDefaultResource : spec.resource_name;
  if (spec.pool_ref.empty()) return true;
  Json pool;
  try {
    pool = client_.get(res::mi355xpools(), m.ns, spec.pool_ref);
  } catch (const KubeError& e) {
    if (!e.not_found()) throw;
    *why = "Mi355xPool " + m.ns + "/" + spec.pool_ref + " not found";
    return false;
  }
  if (spec.resource_name.empty()) *resource = pool.path("spec.resourceName").str_or(gen::kDefaultResource);
  // a pool spanning nodes (spec.maxNodes > 1) lists them all: the gang may use any of them
  *node = pool.path("status.nodeName").as_string();
  std::vector<std::string> span;
  for (const auto& n : pool.path("status.nodes").elements()) span.push_back(n.as_string());
  if (!span.empty()) {
    node->clear();
    for (const auto& n : span) *node += (node->empty() ? "" : ",") + n;
  }
  if (node->empty()) {
    *why = "Mi355xPool " + spec.pool_ref + " has no GPUs placed yet";
    return false;
  }
  if (pool_cap) {
    const int64_t slots = std::max<int64_t>(1, pool.path("spec.sharing.replicasPerGPU").as_int(1));
    for (const auto& n : span.empty() ? std::vector<std::string>{*node} : span) (*pool_cap)[n] = 0;
    for (const auto& d : pool.path("status.devices").elements())
      if (d["health"].as_string() == "Healthy" && d["advertised"].as_bool(false))
        (*pool_cap)[d["node"].as_string()] += slots;
  }
  return true;
}

std::vector<Mi355xJobReconciler::Slot> Mi355xJobReconciler::schedule_(const ObjectMeta& m, const Mi355xJobSpec& spec,
                                                                      const std::string& resource,
                                                                      const std::string& pool_node,
                                                                      const std::map<std::string, int64_t>& pool_cap,
                                                                      std::string* reason, std::string* why,
                                                                      std::vector<Json>* victims) {
  trace::Span span("schedule");
  // 1. queue order: jobs of the same queue that still wait for a placement and sort ahead of us
  //    (priority desc, creation asc) block us, unless they could never fit the whole cluster.
  const std::vector<Json> jobs = jobs_view_();
  const std::vector<Json> nodes = node_objects_();
  int64_t cluster_total = 0;
  for (const auto& n : nodes) cluster_total += qty(n.path("status.allocatable")[resource]);
  auto key_of = [](const Json& j) {
    return std::make_tuple(-j.path("spec.priority").as_int(0), j.path("metadata.creationTimestamp").as_string(),
                           j.path("metadata.namespace").as_string() + "/" + j.path("metadata.name").as_string());
  };
  Json self;
  for (const auto& j : jobs)
    if (j.path("metadata.uid").as_string() == m.uid) self = j;
  if (self.is_null()) return {};
  auto my_key = key_of(self);
  // 0. the job's Mi355xQueue: must exist (the "default" queue is implicit), be Open, and have
  //    capability left for the whole gang
  auto get_queue = [&](const std::string& qname) {
    try {
      return client_.get(res::mi355xqueues(), "", qname);
    } catch (const KubeError& e) {
      if (!e.not_found()) throw;
      return Json();
    }
  };
  const Json queue = get_queue(spec.queue);
  // elastic gangs (minAvailable): any size in [min_r, max_r] workers; max_r may shrink below
  const int min_r = spec.min_workers();
  int max_r = spec.replicas;
  const int64_t need_total = static_cast<int64_t>(min_r) * spec.gpus_per_replica;
  int64_t cap = -1;  // -1 = unlimited
  if (queue.is_null() && spec.queue != "default") {
    *reason = "QueueNotFound";
    *why = "Mi355xQueue " + spec.queue + " does not exist";
    return {};
  }
  if (!queue.is_null()) {
    if (queue.path("spec.state").str_or("Open") == "Closed") {
      *reason = "QueueClosed";
      *why = "Mi355xQueue " + spec.queue + " is Closed";
      return {};
    }
    const Json& c = queue.path("spec.capability")[resource];
    if (!c.is_null()) cap = qty(c);
  }
  if (cap >= 0) {
    int64_t used = 0;
    for (const auto& j : jobs) {
      if (j.path("metadata.uid").as_string() == m.uid || terminal(j.path("status.phase").as_string())) continue;
      if (job_queue(j) == spec.queue && job_resource(j, resource) == resource) used += job_held(j);
    }
    if (used + need_total > cap) {
      *reason = "QueueOverCapacity";
      *why = "queue " + spec.queue + ": " + std::to_string(used) + " " + resource + " held + " +
             std::to_string(need_total) + " needed > capability " + std::to_string(cap);
      return {};
    }
    if (spec.gpus_per_replica > 0)
      max_r = static_cast<int>(std::min<int64_t>(max_r, (cap - used) / spec.gpus_per_replica));
  }
  Json blocker;
  for (const auto& j : jobs) {
    if (j.path("metadata.uid").as_string() == m.uid || !j.path("metadata.deletionTimestamp").as_string().empty()) continue;
    if (j.path("spec.queue").str_or("default") != spec.queue) continue;
    const std::string phase = j.path("status.phase").str_or("Pending");
    if (phase != "Pending" && phase != "Restarting") continue;
    if (!j.path("status.placement").elements().empty()) continue;  // already placed
    const std::string jres = job_resource(j, resource);
    const int64_t jrep = j.path("spec.replicas").as_int(1), jmin = j.path("spec.minAvailable").as_int(jrep);
    int64_t jneed = std::min(jrep, std::max<int64_t>(1, jmin)) * j.path("spec.gpusPerReplica").as_int(1);
    // can never run (bigger than the cluster or than the queue's capability): must not block it
    if (jres == resource && (jneed > cluster_total || (cap >= 0 && jneed > cap))) continue;
    // the nearest job ahead in queue order is the one to wait for: once it is placed, nothing
    // further ahead is still waiting (it could only be placed after them)
    if (key_of(j) < my_key && (blocker.is_null() || key_of(blocker) < key_of(j))) blocker = j;
  }
  if (!blocker.is_null()) {
    const std::string bkey = blocker.path("metadata.namespace").as_string() + "/" + blocker.path("metadata.name").as_string();
    *reason = "QueuedBehind";
    *why = "queue " + spec.queue + ": waiting behind " + bkey;
    std::lock_guard<std::mutex> g(blocked_mu_);
    blocked_by_[m.ns + "/" + m.name] = bkey;
    return {};
  }
  // 2. free GPUs per candidate node = allocatable - live pod requests - other jobs' reservations
  std::map<std::string, int64_t> free;
  std::vector<std::string> order;
  for (const auto& n : nodes) {
    const std::string name = n.path("metadata.name").as_string();
    if (!node_schedulable(n) || !selector_matches(spec.node_selector, n)) continue;
    if (!pool_node.empty() && ("," + pool_node + ",").find("," + name + ",") == std::string::npos) continue;
    free[name] = qty(n.path("status.allocatable")[resource]);
    auto pc = pool_cap.find(name);
    // the pool's own ready slots bound it: the kubelet lowers allocatable only after it heard
    // of a drained GPU, the pool's status already says so
    if (pc != pool_cap.end()) free[name] = std::min(free[name], pc->second);
    order.push_back(name);
  }
  if (spec.gpus_per_replica > 0) {
    for (const auto& kv : pod_usage_(resource))
      if (free.count(kv.first)) free[kv.first] -= kv.second;
    for (const auto& j : jobs) {
      if (j.path("metadata.uid").as_string() == m.uid || terminal(j.path("status.phase").as_string())) continue;
      if (job_resource(j, resource) != resource) continue;
      int64_t g = j.path("spec.gpusPerReplica").as_int(1);
      for (const auto& s : j.path("status.placement").elements())
        if (!s["created"].as_bool(false) && free.count(s["node"].as_string())) free[s["node"].as_string()] -= g;
    }
  }
  // the largest gang in [min_r, max_r] that fits ``f`` (a rigid gang has min_r == max_r)
  auto fit = [&](const std::map<std::string, int64_t>& f) {
    std::vector<std::pair<std::string, int64_t>> cands;
    for (const auto& n : order) cands.emplace_back(n, std::max<int64_t>(0, f.at(n)));
    for (int r = max_r; r >= min_r; --r) {
      auto s = place(cands, r, spec.gpus_per_replica);
      if (!s.empty()) return s;
    }
    return std::vector<Slot>{};
  };
  auto slots = fit(free);
  if (slots.empty() && spec.preemption_policy == "PreemptLowerPriority" && spec.gpus_per_replica > 0 && !order.empty()) {
    // 3. preemption: running (placed) jobs of strictly lower priority on our candidate nodes, the
    //    lowest priority and then the most recently started first; add their GPUs back until the
    //    gang fits, then drop every victim the placement does not need.
    struct Cand {
      Json job;
      std::map<std::string, int64_t> held;
    };
    std::vector<Cand> pool;
    for (const auto& j : jobs) {
      if (j.path("metadata.uid").as_string() == m.uid || !j.path("metadata.deletionTimestamp").as_string().empty())
        continue;
      const std::string ph = j.path("status.phase").str_or("Pending");
      if (terminal(ph) || ph == "Suspended" || j.path("spec.suspend").as_bool(false)) continue;
      if (j.path("spec.priority").as_int(0) >= spec.priority) continue;
      if (job_resource(j, resource) != resource) continue;
      if (job_queue(j) != spec.queue) {  // cross-queue reclaim only from reclaimable queues
        const Json q = get_queue(job_queue(j));
        if (!q.is_null() && !q.path("spec.reclaimable").as_bool(true)) continue;
      }
      Cand c{j, {}};
      const int64_t g = j.path("spec.gpusPerReplica").as_int(1);
      for (const auto& sl : j.path("status.placement").elements())
        if (free.count(sl["node"].as_string())) c.held[sl["node"].as_string()] += g;
      if (!c.held.empty()) pool.push_back(std::move(c));
    }
    std::stable_sort(pool.begin(), pool.end(), [](const Cand& a, const Cand& b) {
      const int64_t pa = a.job.path("spec.priority").as_int(0), pb = b.job.path("spec.priority").as_int(0);
      if (pa != pb) return pa < pb;
      return a.job.path("status.startTime").as_string() > b.job.path("status.startTime").as_string();
    });
    std::map<std::string, int64_t> f2 = free;
    std::vector<size_t> chosen;
    for (size_t i = 0; i < pool.size() && slots.empty(); ++i) {
      for (const auto& kv : pool[i].held) f2[kv.first] += kv.second;
      chosen.push_back(i);
      slots = fit(f2);
    }
    if (!slots.empty()) {
      // minimise: the cheapest victims were added first, so try to spare the later (costlier) ones
      for (size_t k = chosen.size(); k-- > 0;) {
        std::map<std::string, int64_t> f3 = f2;
        for (const auto& kv : pool[chosen[k]].held) f3[kv.first] -= kv.second;
        auto s3 = fit(f3);
        if (!s3.empty()) {
          f2 = std::move(f3);
          slots = std::move(s3);
          chosen.erase(chosen.begin() + static_cast<std::ptrdiff_t>(k));
        }
      }
      for (size_t i : chosen) victims->push_back(pool[i].job);
    }
  }
  if (slots.empty()) {
    int64_t total_free = 0;
    for (const auto& n : order) total_free += std::max<int64_t>(0, free[n]);
    *reason = "Unschedulable";
    *why = "gang of " + (min_r < spec.replicas ? std::to_string(min_r) + ".." : std::string()) +
           std::to_string(spec.replicas) + " x " + std::to_string(spec.gpus_per_replica) + " " +
           resource + " does not fit: " + std::to_string(total_free) + " free on " + std::to_string(order.size()) +
           " candidate node(s)";
  }
  return slots;
}

bool Mi355xJobReconciler::capacity_free_(const Mi355xJobSpec& spec, const std::string& resource,
                                         const Json& placement) {
  std::map<std::string, int64_t> need;
  for (const auto& sl : placement.elements())
    if (!sl["created"].as_bool(false)) need[sl["node"].as_string()] += spec.gpus_per_replica;
  if (need.empty() || spec.gpus_per_replica <= 0) return true;
  std::map<std::string, int64_t> free;
  for (const auto& n : node_objects_()) {
    const std::string name = n.path("metadata.name").as_string();
    if (need.count(name)) free[name] = qty(n.path("status.allocatable")[resource]);
  }
  for (const auto& kv : pod_usage_(resource))
    if (free.count(kv.first)) free[kv.first] -= kv.second;
  for (const auto& kv : need)
    if (free[kv.first] < kv.second) return false;
  return true;
}

Json Mi355xJobReconciler::build_pod_(const Json& job, const ObjectMeta& m, const Mi355xJobSpec& spec,
                                     const std::string& resource, int attempt, int world, const Slot& slot,
                                     const std::string& master_addr) {
  Json pod = Json::object();
  pod["apiVersion"] = "v1";
  pod["kind"] = "Pod";
  Json md = spec.tmpl["metadata"].is_object() ? spec.tmpl["metadata"] : Json::object();
  Json out_md = Json::object();
  out_md["name"] = pod_name(m.name, slot.index);
  out_md["namespace"] = m.ns;
  Json labels = md["labels"].is_object() ? md["labels"] : Json::object();
  labels[gen::kLabelJob] = m.name;
  labels[gen::kLabelJobIndex] = std::to_string(slot.index);
  labels[gen::kLabelJobAttempt] = std::to_string(attempt);
  out_md["labels"] = labels;
  if (md["annotations"].is_object()) out_md["annotations"] = md["annotations"];
  Json owner = Json::object();
  owner["apiVersion"] = job["apiVersion"].str_or(gen::kApiVersion);
  owner["kind"] = "Mi355xJob";
  owner["name"] = m.name;
  owner["uid"] = m.uid;
  owner["controller"] = true;
  owner["blockOwnerDeletion"] = true;
  out_md["ownerReferences"] = Json::array({owner});
  pod["metadata"] = out_md;

  Json ps = spec.tmpl["spec"].is_object() ? spec.tmpl["spec"] : Json::object();
  ps["nodeName"] = slot.node;       // gang placement binds every pod up front
  ps["restartPolicy"] = "Never";    // restarts are gang-wide, by this controller
  if (!ps["containers"].is_array() || ps["containers"].size() == 0) {
    Json c = Json::object();
    c["name"] = "main";
    ps["containers"] = Json::array({c});
  }
  const int nnodes = world, nproc = std::max(1, spec.gpus_per_replica);
  std::vector<std::pair<std::string, std::string>> env = {
      {"MASTER_ADDR", master_addr},
      {"MASTER_PORT", std::to_string(spec.master_port)},
      {"PET_MASTER_ADDR", master_addr},
      {"PET_MASTER_PORT", std::to_string(spec.master_port)},
      {"PET_NNODES", std::to_string(nnodes)},
      {"PET_NPROC_PER_NODE", std::to_string(nproc)},
      {"PET_NODE_RANK", std::to_string(slot.index)},
      {"NODE_RANK", std::to_string(slot.index)},
      {"GPUPOOL_JOB_NAME", m.name},
      {"GPUPOOL_JOB_ATTEMPT", std::to_string(attempt)},
      {"GPUPOOL_REPLICA_INDEX", std::to_string(slot.index)},
  };
  if (!spec.checkpoint_dir.empty()) env.push_back({"GPUPOOL_CHECKPOINT_DIR", spec.checkpoint_dir});
  if (nproc == 1) {  // one process per pod: the pod IS the rank (no torchrun needed)
    env.push_back({"WORLD_SIZE", std::to_string(nnodes)});
    env.push_back({"RANK", std::to_string(slot.index)});
    env.push_back({"LOCAL_RANK", "0"});
    env.push_back({"LOCAL_WORLD_SIZE", "1"});
  }
  Json containers = Json::array();
  for (size_t ci = 0; ci < ps["containers"].size(); ++ci) {
    Json c = static_cast<const Json&>(ps)["containers"][ci];
    Json cenv = Json::array();
    std::set<std::string> ours;
    for (const auto& kv : env) ours.insert(kv.first);
    for (const auto& e : c["env"].elements())
      if (!ours.count(e["name"].as_string())) cenv.push_back(e);  // controller-owned names win
    for (const auto& kv : env) cenv.push_back(Json::object().set("name", kv.first).set("value", kv.second));
    c["env"] = cenv;
    if (ci == 0 && spec.gpus_per_replica > 0) {  // the GPU request sits on the first container
      c["resources"]["limits"][resource] = std::to_string(spec.gpus_per_replica);
      c["resources"]["requests"][resource] = std::to_string(spec.gpus_per_replica);
    }
    containers.push_back(c);
  }
  ps["containers"] = containers;
  pod["spec"] = ps;
  return pod;
}

Outcome Mi355xJobReconciler::cleanup_finished_(const Json& obj, const ObjectMeta& m, const Mi355xJobSpec& spec,
                                               const std::vector<Json>& pods) {
  (void)obj;
  (void)m;
  if (spec.clean_pod_policy == "None") return Outcome::done(ms(0));
  int left = 0;
  for (const auto& p : pods) {
    if (!p.path("metadata.deletionTimestamp").as_string().empty()) {
      ++left;
      continue;
    }
    if (spec.clean_pod_policy == "Running" && terminal(pod_phase(p))) continue;
    try {
      client_.del(res::pods(), m.ns, p.path("metadata.name").as_string());
      ++left;
    } catch (const KubeError& e) {
      if (!e.not_found()) throw;
    }
  }
  return left ? Outcome::requeue(opts_.progress_poll, "cleaning up pods") : Outcome::done(ms(0));
}

Outcome Mi355xJobReconciler::finish_(const Json& obj, const ObjectMeta& m, const Mi355xJobSpec& spec, Json st,
                                     const std::string& phase, const std::string& reason, const std::string& msg,
                                     const std::vector<Json>& pods) {
  const std::string now = rfc3339_now();
  const Json& cst = st;
  Json conds = cst["conditions"].is_array() ? cst["conditions"] : Json::array();
  st["phase"] = phase;
  st["completionTime"] = now;
  st["active"] = 0;
  st["placement"] = Json::array();
  set_condition(conds, gen::kCondRunning, "False", phase == "Succeeded" ? "JobSucceeded" : reason, msg, m.generation,
                now);
  set_condition(conds, gen::kCondRestarting, "False", "Finished", "", m.generation, now);
  set_condition(conds, phase == "Succeeded" ? gen::kCondSucceeded : gen::kCondFailed, "True", reason, msg, m.generation,
                now);
  st["conditions"] = conds;
  write_status_(obj, st);
  event_(obj, phase == "Succeeded" ? "Normal" : "Warning", phase == "Succeeded" ? "JobSucceeded" : "JobFailed", msg);
  job_events().inc({{"transition", phase}});
  log_.info("job finished", Json::object().set("job", m.key()).set("phase", phase).set("reason", reason));
  cleanup_finished_(obj, m, spec, pods);
  return Outcome::requeue(opts_.progress_poll, "finished");
}

Outcome Mi355xJobReconciler::reconcile(const std::string& ns, const std::string& name) {
  Json obj;
  try {
    obj = client_.get(res_, ns, name);  // fresh: the state machine keys off our own status writes
  } catch (const KubeError& e) {
    if (e.not_found()) return Outcome::done(ms(0));
    throw;
  }
  ObjectMeta m = ObjectMeta::from(obj);
  const std::string now = rfc3339_now();
  auto now_tp = std::chrono::system_clock::now();
  Json st = obj["status"].is_object() ? obj["status"] : Json::object();
  const Json& cst = st;  // reads: a non-const operator[] would insert nulls the schema rejects
  Json conds = cst["conditions"].is_array() ? cst["conditions"] : Json::array();
  auto errs = validate_job(obj);
  if (!errs.empty()) {
    std::string msg;
    for (const auto& e : errs) msg += (msg.empty() ? "" : "; ") + e;
    st["phase"] = "Failed";
    st["observedGeneration"] = m.generation;
    set_condition(conds, gen::kCondFailed, "True", "InvalidSpec", msg, m.generation, now);
    st["conditions"] = conds;
    write_status_(obj, st);
    return Outcome::terminal("invalid spec: " + msg);
  }
  Mi355xJobSpec spec = Mi355xJobSpec::from(obj["spec"]);
  std::vector<Json> pods = list_pods_(m, obj.path("status.placement"));

  if (m.deleting()) {  // finalizer: no pod of a deleted job keeps a GPU
    int left = 0;
    for (const auto& p : pods) {
      ++left;
      if (!p.path("metadata.deletionTimestamp").as_string().empty()) continue;
      try {
        client_.del(res::pods(), m.ns, p.path("metadata.name").as_string());
      } catch (const KubeError& e) {
        if (!e.not_found()) throw;
      }
    }
    if (left) return Outcome::requeue(opts_.progress_poll, "deleting job pods");
    if (m.has_finalizer(finalizer_)) remove_finalizer_(obj);
    return Outcome::done(ms(0));
  }
  if (!m.has_finalizer(finalizer_)) {
    obj = ensure_finalizer_(obj);
    m = ObjectMeta::from(obj);
  }
  st["observedGeneration"] = m.generation;
  st["replicas"] = spec.replicas;
  std::string phase = cst["phase"].str_or("Pending");

  // ---- finished: pod cleanup and TTL
  if (terminal(phase)) {
    Outcome o = cleanup_finished_(obj, m, spec, pods);
    if (spec.ttl_seconds_after_finished >= 0) {
      std::chrono::system_clock::time_point done_at;
      if (parse_rfc3339(cst["completionTime"].as_string(), &done_at)) {
        auto expire = done_at + std::chrono::seconds(spec.ttl_seconds_after_finished);
        if (now_tp >= expire) {
          client_.del(res_, m.ns, m.name);
          event_(obj, "Normal", "TTLExpired", "deleted " + std::to_string(spec.ttl_seconds_after_finished) +
                                                  "s after it finished");
          return Outcome::requeue(opts_.progress_poll, "ttl delete");
        }
        auto left = std::chrono::duration_cast<ms>(expire - now_tp) + ms(5);
        if (o.kind == Outcome::Done || left < o.after) return Outcome::requeue(left, "ttl");
      }
    }
    return o;
  }

  Json placement = cst["placement"].is_array() ? cst["placement"] : Json::array();
  auto stop_pods = [&]() {
    int left = 0;
    for (const auto& p : pods) {
      ++left;
      if (!p.path("metadata.deletionTimestamp").as_string().empty()) continue;
      try {
        client_.del(res::pods(), m.ns, p.path("metadata.name").as_string(), terminal(pod_phase(p)) ? 0 : -1);
      } catch (const KubeError& e) {
        if (!e.not_found()) throw;
      }
    }
    return left;
  };

  // ---- preempted by a higher-priority gang (annotation written by its reconciler): stop the gang
  //      and go back to the queue; not a failure, so backoffLimit is untouched
  const std::string preempted_by = obj.path("metadata.annotations")[gen::kAnnJobPreemptedBy].as_string();
  if (!preempted_by.empty() && preempted_by != cst["lastPreemption"].as_string()) {
    st["lastPreemption"] = preempted_by;
    if (phase != "Suspended" && (placement.size() > 0 || !pods.empty())) {
      const std::string by = preempted_by.substr(0, preempted_by.find('@'));
      stop_pods();
      st["phase"] = "Restarting";
      st["placement"] = Json::array();
      st["active"] = 0;
      st["preemptions"] = cst["preemptions"].as_int(0) + 1;
      set_condition(conds, gen::kCondRestarting, "True", "Preempted",
                    "preempted by higher-priority job " + by + "; waiting in the queue", m.generation, now);
      set_condition(conds, gen::kCondRunning, "False", "Preempted", "preempted by " + by, m.generation, now);
      st["conditions"] = conds;
      write_status_(obj, st);
      event_(obj, "Warning", "Preempted", "gang stopped for higher-priority job " + by);
      job_events().inc({{"transition", "Preempted"}});
      return Outcome::requeue(opts_.progress_poll, "preempted");
    }
  }

  // ---- suspend / resume (batch/v1 Job semantics: pods deleted, GPUs freed, deadline clock reset)
  if (spec.suspend) {
    const int left = stop_pods();
    if (phase != "Suspended") {
      event_(obj, "Normal", "Suspended", "spec.suspend is true: stopping " + std::to_string(left) + " pod(s)");
      job_events().inc({{"transition", "Suspended"}});
    }
    st["phase"] = "Suspended";
    st["placement"] = Json::array();
    st["preempting"] = Json::array();
    st["active"] = 0;
    st["masterAddr"] = "";
    st.erase("startTime");
    set_condition(conds, gen::kCondSuspended, "True", "JobSuspended",
                  left ? std::to_string(left) + " pod(s) stopping" : "no pods; GPUs released", m.generation, now);
    set_condition(conds, gen::kCondRunning, "False", "Suspended", "spec.suspend is true", m.generation, now);
    st["conditions"] = conds;
    write_status_(obj, st);
    return left ? Outcome::requeue(opts_.progress_poll, "suspending") : Outcome::done(opts_.resync);
  }
  if (phase == "Suspended") {  // resumed: back through the queue for a fresh gang placement
    phase = "Pending";
    st["phase"] = "Pending";
    placement = Json::array();
    set_condition(conds, gen::kCondSuspended, "False", "Resumed", "spec.suspend is false", m.generation, now);
    event_(obj, "Normal", "Resumed", "re-entering queue " + spec.queue);
    job_events().inc({{"transition", "Resumed"}});
  }

  // ---- deadline
  // a running gang is re-checked on its pods' events (the pod index wakes it); the resync is a
  // safety net, never later than the job's deadline
  auto running_resync = pods_idx_ ? opts_.resync * 6 : opts_.resync;
  if (spec.active_deadline_seconds > 0) {
    std::chrono::system_clock::time_point started;
    if (parse_rfc3339(cst["startTime"].as_string(), &started)) {
      const auto end = started + std::chrono::seconds(spec.active_deadline_seconds);
      if (now_tp > end)
        return finish_(obj, m, spec, st, "Failed", "DeadlineExceeded",
                       "ran longer than activeDeadlineSeconds=" + std::to_string(spec.active_deadline_seconds),
                       pods);
      const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(end - now_tp) + ms(50);
      if (left < running_resync) running_resync = left;
    }
  }

  int attempt = static_cast<int>(cst["attempt"].as_int(0));
  for (const auto& p : pods) attempt = std::max(attempt, label_int(p, gen::kLabelJobAttempt, 0));
  st["attempt"] = attempt;
  const int restarts = static_cast<int>(cst["restarts"].as_int(0));  // failure restarts only
  st["restarts"] = restarts;

  // ---- needs a (new) gang placement: first run, or a restart whose old pods are gone
  if (attempt == 0 || phase == "Restarting" || placement.size() == 0) {
    if (!pods.empty()) {  // previous attempt's pods still hold GPUs: delete and wait
      stop_pods();
      st["active"] = 0;
      write_status_(obj, st);
      return Outcome::requeue(opts_.progress_poll, "waiting for previous pods to terminate");
    }
    std::string resource, pool_node, reason, why;
    std::map<std::string, int64_t> pool_cap;
    if (!resolve_pool_(m, spec, &resource, &pool_node, &why, &pool_cap)) {
      st["phase"] = phase == "Restarting" ? "Restarting" : "Pending";
      set_condition(conds, gen::kCondScheduled, "False", "PoolNotReady", why, m.generation, now);
      st["conditions"] = conds;
      write_status_(obj, st);
      return Outcome::requeue(opts_.resync, "pool not ready");
    }
    std::lock_guard<std::mutex> g(sched_mu_);
    std::vector<Json> victims;
    auto slots = schedule_(m, spec, resource, pool_node, pool_cap, &reason, &why, &victims);
    if (slots.empty()) {
      st["phase"] = phase == "Restarting" ? "Restarting" : "Pending";
      const Json& prev = find_condition(conds, gen::kCondScheduled);
      if (prev["reason"].as_string() != reason) event_(obj, "Warning", reason, why);
      set_condition(conds, gen::kCondScheduled, "False", reason, why, m.generation, now);
      st["conditions"] = conds;
      write_status_(obj, st);
      // re-tried when capacity can have changed (a pod or job ended, a node's allocatable or
      // schedulability moved, a queue or pool changed: the handlers' wake_pending); the timer is
      // only a safety net — with the caches, a retry costs no apiserver LIST either way
      return Outcome::requeue(pods_idx_ ? opts_.resync * 6 : opts_.resync, reason);
    }
    // gang wait: from creation, or from the moment the restart began
    const std::string since_s = attempt > 0 ? find_condition(conds, gen::kCondRestarting)["lastTransitionTime"].as_string()
                                            : obj.path("metadata.creationTimestamp").as_string();
    ++attempt;
    placement = Json::array();
    std::map<std::string, int> per_node;
    for (const auto& s : slots) {
      placement.push_back(Json::object().set("index", s.index).set("node", s.node).set("created", false));
      per_node[s.node]++;
    }
    std::string where;
    for (const auto& kv : per_node) where += (where.empty() ? "" : ", ") + kv.first + " x" + std::to_string(kv.second);
    // preemption: mark the victims (their reconcilers stop them); our pods wait for the GPUs
    Json preempting = Json::array();
    for (const auto& v : victims) {
      const std::string vns = v.path("metadata.namespace").as_string(), vname = v.path("metadata.name").as_string();
      Json patch = Json::object();
      patch["metadata"]["annotations"][gen::kAnnJobPreemptedBy] = m.ns + "/" + m.name + "@" + now;
      try {
        client_.patch_merge(res_, vns, vname, patch);
        preempting.push_back(vns + "/" + vname);
      } catch (const KubeError& e) {
        if (!e.not_found()) throw;
      }
    }
    if (preempting.size() > 0) {
      std::string names;
      for (const auto& v : preempting.elements()) names += (names.empty() ? "" : ", ") + v.as_string();
      where += "; preempting " + names;
      event_(obj, "Normal", "Preempting", "lower-priority job(s) stopped for this gang: " + names);
    }
    st["preempting"] = preempting;
    st["resourceName"] = resource;
    st["attempt"] = attempt;
    st["placement"] = placement;
    st["phase"] = "Pending";
    st["masterAddr"] = "";
    set_condition(conds, gen::kCondScheduled, "True", "GangScheduled",
                  std::to_string(slots.size()) + " pod(s) x " + std::to_string(spec.gpus_per_replica) + " " +
                      resource + " placed: " + where,
                  m.generation, now);
    if (attempt > 1) set_condition(conds, gen::kCondRestarting, "False", "Restarted", "attempt " + std::to_string(attempt),
                                   m.generation, now);
    st["conditions"] = conds;
    // The reservation (status.placement) is written before any pod exists and while sched_mu_ is
    // held, so the next placement decision sees it.
    write_status_(obj, st);
    wake_blocked_by_(m.ns + "/" + m.name);
    obj = client_.get(res_, m.ns, m.name);
    std::chrono::system_clock::time_point since;
    if (parse_rfc3339(since_s, &since))
      gang_wait_hist().observe({}, std::chrono::duration<double>(now_tp - since).count());
    event_(obj, "Normal", "GangScheduled", "attempt " + std::to_string(attempt) + ": " + where);
    job_events().inc({{"transition", "Scheduled"}});
    pods.clear();
  }

  // ---- create pods of this attempt: rank 0 first, the rest once rank 0 has a pod IP
  std::string resource = spec.resource_name, pool_node, why;
  if (resource.empty()) resolve_pool_(m, spec, &resource, &pool_node, &why);
  if (resource.empty()) resource = gen::kDefaultResource;
  if (cst["preempting"].size() > 0) {  // the preempted gangs' pods may still hold our GPUs
    if (!capacity_free_(spec, resource, placement)) {
      st["placement"] = placement;
      st["conditions"] = conds;
      write_status_(obj, st);
      return Outcome::requeue(opts_.progress_poll, "waiting for preempted jobs to release GPUs");
    }
    st["preempting"] = Json::array();
  }
  std::map<int, Json> by_index;
  for (const auto& p : pods)
    if (label_int(p, gen::kLabelJobAttempt, 0) == attempt) by_index[label_int(p, gen::kLabelJobIndex, -1)] = p;
  std::string master_ip = by_index.count(0) ? by_index[0].path("status.podIP").as_string() : "";
  bool created_any = false, lost = false;
  std::string lost_msg;
  for (size_t i = 0; i < placement.size(); ++i) {
    Json& s = placement.at(i);
    int idx = static_cast<int>(s["index"].as_int(0));
    if (by_index.count(idx)) {
      s["created"] = true;
      continue;
    }
    if (s["created"].as_bool(false)) {  // existed in this attempt, now gone (evicted / deleted)
      lost = true;
      lost_msg = "pod " + pod_name(m.name, idx) + " disappeared";
      continue;
    }
    if (idx != 0 && master_ip.empty()) continue;
    Slot slot{idx, s["node"].as_string()};
    Json pod = build_pod_(obj, m, spec, resource, attempt, static_cast<int>(placement.size()), slot,
                          idx == 0 ? "localhost" : master_ip);
    try {
      by_index[idx] = client_.create(res::pods(), m.ns, pod);
      s["created"] = true;
      created_any = true;
    } catch (const KubeError& e) {
      if (!e.conflict()) throw;  // 409 AlreadyExists: a pod of an older attempt is still terminating
      return Outcome::requeue(opts_.progress_poll, "pod name still in use");
    }
  }
  if (created_any) event_(obj, "Normal", "PodsCreated", "attempt " + std::to_string(attempt));
  st["placement"] = placement;
  if (!master_ip.empty()) st["masterAddr"] = master_ip;

  // ---- observe pods
  int active = 0, succeeded = 0, failed = 0, running = 0;
  std::string fail_msg;
  Json rs = Json::array();
  for (const auto& kv : by_index) {
    const Json& p = kv.second;
    const std::string ph = pod_phase(p);
    Json r = Json::object();
    r["index"] = kv.first;
    r["pod"] = p.path("metadata.name").as_string();
    r["node"] = p.path("spec.nodeName").as_string();
    r["phase"] = ph;
    if (!p.path("status.podIP").as_string().empty()) r["podIP"] = p.path("status.podIP").as_string();
    const Json& cs = p.path("status.containerStatuses");
    if (cs.size() > 0 && cs[0].path("state.terminated").is_object())
      r["exitCode"] = cs[0].path("state.terminated.exitCode").as_int(0);
    const std::string devs = p.path("metadata.annotations")[gen::kAnnPodDevices].as_string();
    if (!devs.empty()) r["devices"] = devs;
    if (ph == "Failed") {
      ++failed;
      std::string why_pod = p.path("status.message").as_string();
      if (why_pod.empty() && r.contains("exitCode")) why_pod = "exit code " + std::to_string(r["exitCode"].as_int());
      r["message"] = why_pod;
      if (fail_msg.empty()) fail_msg = "pod " + r["pod"].as_string() + " failed: " + why_pod;
    } else if (ph == "Succeeded") {
      ++succeeded;
    } else if (p.path("metadata.deletionTimestamp").as_string().empty()) {
      ++active;
      if (ph == "Running") ++running;
    }
    rs.push_back(r);
  }
  st["replicaStatuses"] = rs;
  st["active"] = active;
  st["succeeded"] = succeeded;
  st["failed"] = failed;

  // ---- transitions
  if (failed > 0 || lost) {
    const std::string msg = !fail_msg.empty() ? fail_msg : lost_msg;
    if (spec.restart_policy == "OnFailure" && restarts < spec.backoff_limit) {
      stop_pods();  // the whole gang restarts
      st["phase"] = "Restarting";
      st["placement"] = Json::array();
      st["active"] = 0;
      st["restarts"] = restarts + 1;
      set_condition(conds, gen::kCondRestarting, "True", lost ? "PodLost" : "PodFailed",
                    msg + "; restarting the gang (restart " + std::to_string(restarts + 1) + "/" +
                        std::to_string(spec.backoff_limit) + ")",
                    m.generation, now);
      set_condition(conds, gen::kCondRunning, "False", "Restarting", msg, m.generation, now);
      st["conditions"] = conds;
      write_status_(obj, st);
      event_(obj, "Warning", "GangRestarting", msg);
      job_events().inc({{"transition", "Restarting"}});
      return Outcome::requeue(opts_.progress_poll, "gang restart");
    }
    st["conditions"] = conds;
    return finish_(obj, m, spec, st, "Failed",
                   spec.restart_policy == "Never" ? "PodFailed" : "BackoffLimitExceeded", msg, pods);
  }
  const int world = static_cast<int>(placement.size());  // workers of this attempt
  st["workers"] = world;
  const bool all_done = world > 0 && succeeded == world;
  const bool rank0_done = by_index.count(0) && pod_phase(by_index[0]) == "Succeeded";
  if (all_done || (spec.success_policy == "Rank0" && rank0_done)) {
    st["conditions"] = conds;
    return finish_(obj, m, spec, st, "Succeeded", "JobSucceeded",
                   std::to_string(succeeded) + "/" + std::to_string(world) + " worker(s) succeeded", pods);
  }
  if (world > 0 && static_cast<int>(by_index.size()) == world && running + succeeded == world) {
    if (phase != "Running") {
      event_(obj, "Normal", "JobRunning", std::to_string(running) + " worker(s) running");
      job_events().inc({{"transition", "Running"}});
    }
    st["phase"] = "Running";
    if (cst["startTime"].as_string().empty()) st["startTime"] = now;
    set_condition(conds, gen::kCondRunning, "True", "AllWorkersRunning",
                  std::to_string(running) + "/" + std::to_string(world) + " worker(s) running", m.generation,
                  now);
    st["conditions"] = conds;
    write_status_(obj, st);
    return Outcome::done(running_resync);
  }
  st["phase"] = phase == "Running" ? "Running" : "Pending";
  st["conditions"] = conds;
  write_status_(obj, st);
  return Outcome::requeue(opts_.progress_poll, "starting workers");
}

Mi355xQueueReconciler::Mi355xQueueReconciler(KubeClient& client, Informer& queues, Informer& jobs,
                                             EventRecorder* events, ReconcilerOptions opts)
    : PoolReconcilerBase(client, queues, events, opts, "Mi355xQueue", res::mi355xqueues()), jobs_(jobs) {}

Outcome Mi355xQueueReconciler::reconcile(const std::string& ns, const std::string& name) {
  (void)ns;
  Json obj;
  try {
    obj = client_.get(res_, "", name);
  } catch (const KubeError& e) {
    if (e.not_found()) return Outcome::done(ms(0));
    throw;
  }
  int pending = 0, running = 0, suspended = 0, completed = 0, failed = 0;
  std::map<std::string, int64_t> alloc;
  for (const auto& j : jobs_.list()) {
    if (job_queue(j) != name) continue;
    const std::string phase = j.path("status.phase").str_or("Pending");
    if (phase == "Running") ++running;
    else if (phase == "Suspended") ++suspended;
    else if (phase == "Succeeded") ++completed;
    else if (phase == "Failed") ++failed;
    else ++pending;
    if (!terminal(phase) && j.path("status.placement").size() > 0)
      alloc[job_resource(j, gen::kDefaultResource)] += job_held(j);
  }
  const Json& cur = obj["status"];
  Json st = cur.is_object() ? cur : Json::object();
  st["observedGeneration"] = obj.path("metadata.generation").as_int(0);
  st["state"] = obj.path("spec.state").str_or("Open");
  st["pending"] = pending;
  st["running"] = running;
  st["suspended"] = suspended;
  st["completed"] = completed;
  st["failed"] = failed;
  Json a = Json::object();
  for (const auto& kv : alloc) {
    a[kv.first] = kv.second;
    queue_alloc_gauge().set({{"queue", name}, {"resource", kv.first}}, static_cast<double>(kv.second));
  }
  for (const auto& kv : cur["allocated"].members())  // resources no longer held go to zero
    if (!alloc.count(kv.first)) queue_alloc_gauge().set({{"queue", name}, {"resource", kv.first}}, 0);
  const std::pair<const char*, int> phases[] = {{"Pending", pending}, {"Running", running}, {"Suspended", suspended},
                                                {"Succeeded", completed}, {"Failed", failed}};
  for (const auto& ph : phases) queue_jobs_gauge().set({{"queue", name}, {"phase", ph.first}}, ph.second);
  st["allocated"] = a;
  write_status_(obj, st);
  return Outcome::done(opts_.resync);
}

}  // namespace gpupool

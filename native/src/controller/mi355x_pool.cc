// Mi355xPool: claim, probe, advertise and drain MI355X GPUs through the node agents
// (RocmProvider), quota reservations, spanning pools, the orphan sweep.
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

namespace {
// GPUs (by uuid) grouped by the node that holds them (spanning pools act per node).
template <class Obs>
std::map<std::string, std::vector<std::string>> by_node(const Obs& o, const std::vector<std::string>& uuids) {
  std::map<std::string, std::vector<std::string>> out;
  for (const auto& u : uuids)
    for (const auto& d : o.mine)
      if (d.uuid == u) out[d.node.empty() ? o.node : d.node].push_back(u);
  return out;
}

// o.nodes = every node holding GPUs of the pool; for a spanning pool also the primary o.node (the
// node holding most of it, ties by name) and its free count.
template <class Obs>
void index_nodes(Obs& o, bool primary) {
  std::map<std::string, int> per_node;
  for (const auto& d : o.mine) ++per_node[d.node.empty() ? o.node : d.node];
  o.nodes.clear();
  for (const auto& kv : per_node) o.nodes.push_back(kv.first);
  if (!primary) return;
  o.node.clear();
  int best = 0;
  for (const auto& kv : per_node)
    if (kv.second > best) {
      best = kv.second;
      o.node = kv.first;
    }
  o.free_healthy = o.node.empty() || !o.free_by_node.count(o.node) ? 0 : o.free_by_node.at(o.node);
}
}  // namespace

// ================================================================== Mi355xPool
Mi355xPoolReconciler::Mi355xPoolReconciler(KubeClient& client, Informer& pools, DeviceProvider& provider,
                                           EventRecorder* events, ReconcilerOptions opts)
    : PoolReconcilerBase(client, pools, events, opts, "Mi355xPool", res::mi355xpools()), provider_(provider) {}

ClaimResult Mi355xPoolReconciler::claim_(const std::string& node, const ClaimRequest& req) {
  try {
    return provider_.claim(node, req);
  } catch (const ProviderError& e) {
    if (e.code == "AgentUnreachable") {  // sent, but no reply: the agent may have committed it
      std::lock_guard<std::mutex> g(mu_);
      suspect_[req.pool_uid].insert(node);
    }
    throw;
  }
}

// A claim whose reply was lost (the agent died or the connection reset after it committed) leaves
// GPUs of a single-node pool on a node its status may never name: invisible to every later pass
// and no orphan either (the pool lives). Each such node is asked once it answers: its GPUs become
// the pool's when the pool holds none elsewhere, else they are released (never acknowledged, so
// no pod can use them); a node without any is forgotten.
void Mi355xPoolReconciler::resolve_suspects_(const ObjectMeta& m, Observed& o) {
  std::set<std::string> sus;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = suspect_.find(m.uid);
    if (it == suspect_.end()) return;
    sus = it->second;
  }
  auto drop = [&](const std::string& n) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = suspect_.find(m.uid);
    if (it == suspect_.end()) return;
    it->second.erase(n);
    if (it->second.empty()) suspect_.erase(it);
  };
  for (const auto& n : sus) {
    if (!o.reachable) return;  // the pool's own node did not answer: nothing can be decided yet
    if (n == o.node) {         // observed as the pool's node this pass: nothing hidden there
      drop(n);
      continue;
    }
    NodeView nv = provider_.observe_pool(n, m.uid);
    if (!nv.reachable) continue;  // still unknown: ask again next pass
    std::vector<DeviceView> got;
    for (auto& d : nv.devices)
      if (d.pool_uid == m.uid) got.push_back(std::move(d));
    if (!got.empty() && o.mine.empty()) {
      log_.warn("adopting GPUs of a claim whose reply was lost",
                Json::object().set("pool", m.key()).set("node", n).set("count", static_cast<long long>(got.size())));
      o.node = n;
      o.mine = std::move(got);
      o.free_healthy = nv.free_healthy >= 0 ? nv.free_healthy : 0;
    } else if (!got.empty()) {
      std::vector<std::string> uuids;
      for (const auto& d : got) uuids.push_back(d.uuid);
      log_.warn("releasing GPUs of a claim whose reply was lost",
                Json::object().set("pool", m.key()).set("node", n).set("count", static_cast<long long>(uuids.size())));
      provider_.release(n, m.uid, uuids);
    }
    drop(n);
  }
}

Mi355xPoolReconciler::Observed Mi355xPoolReconciler::observe_(const ObjectMeta& m, const Mi355xPoolSpec& spec,
                                                              const Json& status) {
  trace::Span span("observe");
  Observed o;
  const bool span_nodes = spans_(spec);
  std::set<std::string> hinted;
  std::string hint = status["nodeName"].as_string();
  if (!hint.empty()) hinted.insert(hint);
  for (const auto& n : status["nodes"].elements()) hinted.insert(n.as_string());
  // The informer may still hold a copy from before this manager's own last status write (a pass
  // queued by that write's own watch event often runs first): where that write put the pool counts
  // too. Without it a pass on the older copy (no nodeName yet) skips the pool's node when its agent
  // is down — and concludes the pool holds nothing (scale-up elsewhere, or a finalizer removed).
  const std::vector<std::string> wrote = written_placement_(m.uid);
  if (hint.empty() && !wrote.empty()) hint = wrote[0];
  for (const auto& n : wrote)
    if (!n.empty()) hinted.insert(n);
  std::vector<std::string> nodes;
  if (span_nodes) {
    nodes = provider_.node_names();  // a spanning pool may hold GPUs on any agent: see them all
  } else {
    if (!hint.empty()) nodes.push_back(hint);
    if (!spec.node_name.empty() && spec.node_name != hint) nodes.push_back(spec.node_name);
    if (nodes.empty()) nodes = provider_.node_names();
  }
  std::vector<std::string> unreachable_hinted;
  std::set<std::string> answered;  // nodes observed this pass (a spanning pool's suspects among them are resolved)
  for (const auto& n : nodes) {
    NodeView nv = provider_.observe_pool(n, m.uid);
    if (nv.reachable) answered.insert(n);
    if (!nv.reachable) {
      if (hinted.count(n) || n == spec.node_name) {
        o.reachable = false;
        o.error = nv.error;
        o.node = n;
        if (hinted.count(n)) unreachable_hinted.push_back(n);
      } else {
        o.unknown.push_back(n);
      }
      continue;
    }
    std::vector<DeviceView> mine;
    int64_t free_healthy = 0;
    for (auto& d : nv.devices) {
      if (d.pool_uid == m.uid) mine.push_back(d);
      else if (d.state == "Free" && d.healthy) ++free_healthy;
    }
    if (nv.free_healthy >= 0) free_healthy = nv.free_healthy;  // pool-scoped view
    if (!provider_.node_schedulable(n)) free_healthy = 0;  // cordoned: no capacity for new claims
    o.free_by_node[n] = free_healthy;
    if (span_nodes) {
      for (auto& d : mine) o.mine.push_back(std::move(d));
      continue;
    }
    if (!mine.empty() || n == hint || (o.node.empty() && n == spec.node_name)) {
      o.node = n;
      o.reachable = true;
      o.error.clear();
      o.mine = std::move(mine);
      o.free_healthy = free_healthy;
      if (!o.mine.empty()) break;
    }
  }
  if (!span_nodes) {
    resolve_suspects_(m, o);
  } else {
    // A spanning pool observes every node: whatever a lost claim reply left on a node that answered
    // this pass is in o.mine already (kept or released by this pass's plan), so that node is no
    // longer a suspect. Without this a spanning pool could never be finalized after a lost reply.
    std::lock_guard<std::mutex> g(mu_);
    auto it = suspect_.find(m.uid);
    if (it != suspect_.end()) {
      for (const auto& n : answered) it->second.erase(n);
      if (it->second.empty()) suspect_.erase(it);
    }
  }
  std::sort(o.mine.begin(), o.mine.end(), [](const DeviceView& a, const DeviceView& b) {
    return a.node != b.node ? a.node < b.node : a.index < b.index;
  });
  index_nodes(o, span_nodes && o.reachable);
  // A node that held GPUs of the pool and is unreachable now keeps its place in status.nodes: its
  // GPUs (and their pods) are still held, so it must stay hinted — and block scale-up (the pass
  // returns early while !reachable) — until it answers again.
  for (const auto& n : unreachable_hinted)
    if (std::find(o.nodes.begin(), o.nodes.end(), n) == o.nodes.end()) o.nodes.push_back(n);
  std::sort(o.nodes.begin(), o.nodes.end());
  o.unreachable = unreachable_hinted;
  return o;
}

std::vector<std::string> Mi355xPoolReconciler::choose_nodes_(const Mi355xPoolSpec& spec, int need) {
  if (!spec.node_name.empty()) return {spec.node_name};
  struct Cand {
    std::string name;
    int64_t free;
  };
  std::vector<Cand> fit;
  for (const auto& n : provider_.node_names()) {
    Json labels = provider_.node_labels(n);
    bool match = true;
    for (const auto& kv : spec.node_selector)
      if (labels[kv.first].as_string() != kv.second) match = false;
    if (!match || !provider_.node_schedulable(n)) continue;  // cordoned nodes get no new claims
    // an estimate (the agents' last full views less claims made or in flight since): placing 256
    // pools on 64 nodes at once asked every agent for its full view on every pass, and every
    // worker raced for the same tightest node (scripts/scale_bench.py, profiles/r5n_*)
    const int64_t free = provider_.free_capacity(n);
    if (free >= need) fit.push_back({n, free});
  }
  // Tightest fit first (bin-packing keeps whole nodes free for big pools); the caller falls
  // through the list when a concurrent claim took the capacity meanwhile.
  std::sort(fit.begin(), fit.end(), [](const Cand& a, const Cand& b) {
    return a.free != b.free ? a.free < b.free : a.name < b.name;
  });
  std::vector<std::string> out;
  for (const auto& c : fit) out.push_back(c.name);
  return out;
}

std::vector<std::pair<std::string, int>> Mi355xPoolReconciler::plan_span_(const Mi355xPoolSpec& spec, int need,
                                                                          const Observed& o) {
  struct Cand {
    std::string name;
    int64_t free;
    bool mine;
  };
  std::vector<Cand> cands;
  for (const auto& kv : o.free_by_node) {
    if (kv.second <= 0) continue;
    bool mine = std::find(o.nodes.begin(), o.nodes.end(), kv.first) != o.nodes.end();
    if (!mine) {
      Json labels = provider_.node_labels(kv.first);
      bool match = true;
      for (const auto& sel : spec.node_selector)
        if (labels[sel.first].as_string() != sel.second) match = false;
      if (!match) continue;
    }
    cands.push_back({kv.first, kv.second, mine});
  }
  // nodes already holding the pool first (locality), then most free first (fewest nodes)
  std::sort(cands.begin(), cands.end(), [](const Cand& a, const Cand& b) {
    if (a.mine != b.mine) return a.mine;
    return a.free != b.free ? a.free > b.free : a.name < b.name;
  });
  const int allowed_new = spec.max_nodes - static_cast<int>(o.nodes.size());
  std::vector<std::pair<std::string, int>> plan;
  int left = need;
  for (const auto& c : cands)  // 1. grow where the pool already is
    if (c.mine && left > 0) {
      int k = static_cast<int>(std::min<int64_t>(c.free, left));
      plan.emplace_back(c.name, k);
      left -= k;
    }
  if (left == 0) return plan;
  if (allowed_new < 1) return {};
  // 2. the rest on ONE new node if any fits it (the tightest such fit keeps big nodes whole)
  const Cand* single = nullptr;
  for (const auto& c : cands)
    if (!c.mine && c.free >= left && (!single || c.free < single->free)) single = &c;
  if (single) {
    plan.emplace_back(single->name, left);
    return plan;
  }
  // 3. else split over the fewest new nodes (most free first), within spec.maxNodes
  int new_nodes = 0;
  for (const auto& c : cands) {
    if (c.mine || left <= 0 || new_nodes >= allowed_new) continue;
    int k = static_cast<int>(std::min<int64_t>(c.free, left));
    plan.emplace_back(c.name, k);
    left -= k;
    ++new_nodes;
  }
  if (left > 0) return {};
  return plan;
}

int Mi355xPoolReconciler::drain_(const Json& obj, const std::string& node, const ObjectMeta& m,
                                 const Mi355xPoolSpec& spec, std::vector<DeviceView>& mine) {
  trace::Span span("drain");
  int still = 0;
  std::map<std::string, std::vector<std::string>> release;  // node -> drained GPUs
  auto now = std::chrono::system_clock::now();
  for (auto& d : mine) {
    if (d.state != "Draining") continue;
    if (d.pods.size() == 0) {
      release[d.node.empty() ? node : d.node].push_back(d.uuid);
      continue;
    }
    ++still;
    bool timed_out = false;
    std::chrono::system_clock::time_point started;
    if (parse_rfc3339(d.drain_started_at, &started))
      timed_out = now - started > std::chrono::seconds(spec.drain_timeout_seconds);
    for (const auto& p : d.pods.elements()) {
      std::string pns = p["namespace"].as_string(), pname = p["name"].as_string();
      if (p.is_string()) {
        auto slash = p.as_string().find('/');
        pns = p.as_string().substr(0, slash);
        pname = p.as_string().substr(slash + 1);
      }
      std::string key = pns + "/" + pname;
      try {
        if (timed_out) {
          client_.del(res::pods(), pns, pname, 0);
          event_(obj, "Warning", "DrainTimeout", "force-deleted pod " + key + " on " + short_id(d) +
                                                     " after " + std::to_string(spec.drain_timeout_seconds) + "s");
        } else if (spec.drain_evict) {
          bool done;
          {
            std::lock_guard<std::mutex> g(mu_);
            done = evicted_[m.uid].count(key) > 0;
          }
          if (!done) {
            // marked evicted only once the API accepted it: a PodDisruptionBudget refusal (429)
            // is retried on the next pass until drain.timeoutSeconds forces the delete
            client_.evict(pns, pname, static_cast<int>(spec.drain_grace_seconds));
            {
              std::lock_guard<std::mutex> g(mu_);
              evicted_[m.uid].insert(key);
              eviction_blocked_[m.uid].erase(key);
            }
            event_(obj, "Normal", "PodEvicted", "evicted pod " + key + " from " + short_id(d) + " (draining)");
          }
        }
      } catch (const KubeError& e) {
        if (e.code == 429) {
          bool first;
          {
            std::lock_guard<std::mutex> g(mu_);
            first = eviction_blocked_[m.uid].insert(key).second;
          }
          if (first)
            event_(obj, "Warning", "EvictionBlocked", "pod " + key + " on " + short_id(d) + ": " + e.what() +
                                                          " (retrying; forced after " +
                                                          std::to_string(spec.drain_timeout_seconds) + "s)");
        } else if (!e.not_found()) {
          log_.warn("drain action failed", Json::object().set("pod", key).set("error", e.what()));
        }
      }
    }
  }
  for (const auto& kv : release) {
    try {
      provider_.release(kv.first, m.uid, kv.second);
    } catch (const ProviderError& e) {
      // The agent re-checks the kubelet before releasing: a pod our view did not show yet (it
      // started after the view was taken) keeps its GPU. Not a failure: the release RPC
      // invalidated the view cache, so the next pass observes the pod and evicts it.
      if (e.code != "PodsRunning") throw;
      still += static_cast<int>(kv.second.size());
      continue;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      evicted_[m.uid].clear();
      eviction_blocked_[m.uid].clear();
    }
    event_(obj, "Normal", "GPUReleased", "released " + std::to_string(kv.second.size()) + " GPU(s) on " + kv.first +
                                             ": " + join(kv.second, ","));
  }
  return still;
}

Json Mi355xPoolReconciler::build_status_(const Json& obj, const ObjectMeta& m, const Mi355xPoolSpec& spec,
                                         const Observed& o, const std::string& progress_reason,
                                         const std::string& progress_msg, const std::string& blocked, bool deleting) {
  const std::string now = rfc3339_now();
  Json st = Json::object();
  st["observedGeneration"] = m.generation;
  int64_t claimed = 0, ready = 0, probing = 0;
  std::vector<std::string> xgmi_bad, xgmi_unknown, ecc_bad, thermal_bad, probe_bad, unhealthy;
  double min_gbps = 1e30, min_tf = 1e30, min_xgmi = 1e30;
  Json devices = Json::array();
  for (const auto& d : o.mine) {
    devices.push_back(d.status_json());
    if (d.state == "Draining") continue;
    ++claimed;
    if (d.state == "Probing" && !d.probe_overdue) {
      ++probing;
      continue;
    }
    if (d.probe_overdue) {
      probe_bad.push_back(short_id(d) + ": ProbeTimeout: still Probing past spec.probe.timeoutSeconds");
      unhealthy.push_back(short_id(d));
      continue;
    }
    auto reasons = [&](const char* prefix) {
      std::vector<std::string> rs;
      for (const auto& r : d.verdict["reasons"].elements())
        if (r.as_string().rfind(prefix, 0) == 0) rs.push_back(r.as_string());
      return short_id(d) + ": " + join(rs, "; ");
    };
    if (!d.verdict["xgmiOk"].as_bool(true)) xgmi_bad.push_back(reasons("XGMI"));
    if (!d.verdict["eccOk"].as_bool(true)) ecc_bad.push_back(reasons("HBM"));
    if (!d.verdict["thermalOk"].as_bool(true)) thermal_bad.push_back(reasons("Thermal"));
    if (d.probe.path("xgmi.GBps").is_number()) min_xgmi = std::min(min_xgmi, d.probe.path("xgmi.GBps").as_double(1e30));
    if (d.probe.path("xgmi.unavailable").as_bool(false))
      xgmi_unknown.push_back(short_id(d) + ": " + d.probe.path("xgmi.error").str_or("peer check could not run"));
    if (!d.probe_passed) {
      const std::string err = d.probe["error"].str_or(d.probe.is_object() ? "probe failed" : "not probed");
      probe_bad.push_back(short_id(d) + ": " + err);
      // the xGMI peer-copy check (spec.probe.xgmiPeerCheck) is link health too
      if (err.rfind("XGMIPeerCheckFailed", 0) == 0) xgmi_bad.push_back(short_id(d) + ": " + err);
    } else {
      min_gbps = std::min(min_gbps, d.probe.path("hbm.GBps").as_double(1e30));
      min_tf = std::min(min_tf, d.probe.path("mfma.tflops").as_double(1e30));
    }
    if (!d.healthy || !d.probe_passed) unhealthy.push_back(short_id(d));
    if (d.state == "Claimed" && d.healthy && d.probe_passed && d.advertised) ++ready;
  }
  // An agent that does not answer (restarting, node network down) says nothing about its GPUs:
  // they are still held, with whatever pods run on them. Its devices stay in status as last
  // observed (health "Unknown") and count in replicas — never erased by a transient failure
  // (the reference returns without touching status on a list error, README.md:189-193). They do
  // not count as ready: with the agent its device plugin is gone too, so no new pod can be given
  // them until it answers and they are verified again (Ready=Unknown, reason AgentUnreachable).
  int64_t retained = 0;
  if (!o.reachable) {
    std::set<std::string> gone(o.unreachable.begin(), o.unreachable.end());
    if (!o.node.empty()) {
      bool seen = false;
      for (const auto& d : o.mine) seen = seen || (d.node.empty() ? o.node : d.node) == o.node;
      if (!seen) gone.insert(o.node);
    }
    for (const auto& d : obj.path("status.devices").elements()) {
      if (!gone.count(d["node"].str_or(obj.path("status.nodeName").as_string()))) continue;
      Json kept = d;
      if (kept["health"].as_string() != "Draining") {
        kept["health"] = "Unknown";
        ++retained;
      }
      devices.push_back(kept);
    }
  }
  st["replicas"] = claimed + retained;
  st["readyReplicas"] = ready;
  st["allocatable"] = ready * static_cast<int64_t>(spec.sharing_replicas);  // slots of resourceName
  if (!o.node.empty()) st["nodeName"] = o.node;
  if (o.nodes.size() > 1 || spans_(spec)) {
    Json ns = Json::array();
    for (const auto& n : o.nodes) ns.push_back(n);
    st["nodes"] = ns;
  }
  st["devices"] = devices;
  Json conds = obj.path("status.conditions").is_array() ? obj.path("status.conditions") : Json::array();
  const int64_t gen = m.generation;
  auto health_cond = [&](const char* type, const std::vector<std::string>& bad, const char* bad_reason,
                         const char* ok_reason, const char* ok_msg) {
    if (!bad.empty()) set_condition(conds, type, "False", bad_reason, join(bad, " | "), gen, now);
    else set_condition(conds, type, "True", claimed ? ok_reason : "NoDevices",
                       claimed ? std::to_string(claimed) + " GPU(s): " + ok_msg : "no GPUs claimed", gen, now);
  };
  std::string xgmi_ok_msg = "xGMI links up";
  if (min_xgmi < 1e29) {
    char buf[96];
    std::snprintf(buf, sizeof buf, "; peer-copy ring min %.0f GB/s", min_xgmi);
    xgmi_ok_msg += buf;
  }
  if (!o.reachable && retained > 0) {
    // the health of the unanswered node's GPUs is unknown: their conditions keep the last verdict
  } else if (xgmi_bad.empty() && !xgmi_unknown.empty()) {
    // the peer-copy check could not run (no peer access / HIP error): the links are unverified,
    // not faulty — Unknown, and no GPU is replaced for it
    set_condition(conds, gen::kCondXGMILinksHealthy, "Unknown", "XGMIPeerCheckUnavailable", join(xgmi_unknown, " | "),
                  gen, now);
  } else {
    health_cond(gen::kCondXGMILinksHealthy, xgmi_bad, "XGMILinkDown", "AllLinksUp", xgmi_ok_msg.c_str());
  }
  if (o.reachable || retained == 0) {
    health_cond(gen::kCondHBMECCHealthy, ecc_bad, "HBMECCErrors", "NoNewECCErrors", "no new HBM ECC errors since claim");
    health_cond(gen::kCondThermalHealthy, thermal_bad, "ThermalLimit", "WithinThermalLimits",
                "temperatures below device limits");
  }
  if (!o.reachable && retained > 0) {
    // DeviceProbePassed keeps its last verdict too
  } else if (probing) {
    set_condition(conds, gen::kCondDeviceProbePassed, "Unknown", "Probing", std::to_string(probing) + " GPU(s) probing", gen, now);
  } else if (!probe_bad.empty()) {
    // the isolation outcomes name themselves (ProbeCrashed / ProbeTimeout / ProbeInterrupted /
    // ProbeUnavailable: the probe helper died, missed its deadline, or a restarted agent found the
    // GPU mid-probe); any other failure is ProbeFailed
    std::string why = "ProbeFailed";
    for (const char* k : {"ProbeCrashed", "ProbeTimeout", "ProbeInterrupted", "ProbeUnavailable"}) {
      bool all = true;
      for (const auto& b : probe_bad) all = all && b.find(std::string(": ") + k + ":") != std::string::npos;
      if (all) why = k;
    }
    set_condition(conds, gen::kCondDeviceProbePassed, "False", why, join(probe_bad, " | "), gen, now);
  } else if (claimed) {
    char msg[200];
    std::snprintf(msg, sizeof msg, "%lld GPU(s) passed HBM+MFMA probe (min HBM %.0f GB/s, min MFMA %.0f TFLOP/s)",
                  static_cast<long long>(claimed), min_gbps > 1e29 ? 0.0 : min_gbps, min_tf > 1e29 ? 0.0 : min_tf);
    set_condition(conds, gen::kCondDeviceProbePassed, "True", "ProbePassed", msg, gen, now);
  } else {
    set_condition(conds, gen::kCondDeviceProbePassed, "True", "NoDevices", "no GPUs claimed", gen, now);
  }
  if (!o.reachable) {
    set_condition(conds, gen::kCondDegraded, "True", "AgentUnreachable", o.error, gen, now);
  } else if (!unhealthy.empty()) {
    set_condition(conds, gen::kCondDegraded, "True", "DeviceUnhealthy", join(unhealthy, ", "), gen, now);
  } else if (!blocked.empty()) {
    set_condition(conds, gen::kCondDegraded, "True", blocked, progress_msg, gen, now);
  } else {
    set_condition(conds, gen::kCondDegraded, "False", "AsExpected", "all claimed GPUs healthy", gen, now);
  }
  if (!blocked.empty()) {
    set_condition(conds, gen::kCondProgressing, "False", blocked, progress_msg, gen, now);
  } else if (!progress_reason.empty()) {
    set_condition(conds, gen::kCondProgressing, "True", progress_reason, progress_msg, gen, now);
  } else {
    set_condition(conds, gen::kCondProgressing, "False", "Stable",
                  std::to_string(ready) + "/" + std::to_string(spec.replicas) + " GPUs ready", gen, now);
  }
  set_condition(conds, gen::kCondDeleting, deleting ? "True" : "False", deleting ? "Finalizing" : "NotDeleting",
                deleting ? "draining and releasing GPUs before removing the finalizer" : "", gen, now);
  bool is_ready = !deleting && o.reachable && ready == spec.replicas && claimed == spec.replicas;
  std::string reason = is_ready ? "AllReplicasReady"
                       : deleting ? "Deleting"
                       : !o.reachable ? "AgentUnreachable"
                       : !blocked.empty() ? blocked
                       : probing ? "Probing"
                       : !progress_reason.empty() ? progress_reason
                       : !unhealthy.empty() ? "DeviceUnhealthy"
                       : "NotReady";
  set_condition(conds, gen::kCondReady, is_ready ? "True" : (!o.reachable && !deleting) ? "Unknown" : "False", reason,
                std::to_string(ready) + "/" + std::to_string(spec.replicas) + " GPUs ready" +
                    (o.nodes.size() > 1 ? " on " + std::to_string(o.nodes.size()) + " nodes"
                     : o.node.empty() ? "" : " on " + o.node),
                gen, now);
  st["conditions"] = conds;
  return st;
}

Outcome Mi355xPoolReconciler::finalize_(const Json& obj, const ObjectMeta& m, const Mi355xPoolSpec& spec) {
  Observed o = observe_(m, spec, obj["status"]);
  if (!o.reachable && !o.node.empty()) {
    const Json cur = fresh_(obj);
    write_status_(cur, build_status_(cur, m, spec, o, "Deleting", "agent unreachable", "", true));
    return Outcome::transient("agent unreachable during finalization: " + o.error);
  }
  // Status names no node (never placed, or a claim whose status write never landed) and some agent
  // did not answer: it may hold GPUs of this pool, with pods on them. The finalizer stays until that
  // agent answers or its node leaves the cluster — "all GPUs released" must be a fact, not a guess.
  if (o.mine.empty() && o.nodes.empty() && !o.unknown.empty()) {
    write_status_(obj, build_status_(obj, m, spec, o, "Deleting",
                                     "waiting for unreachable agent(s) on " + join(o.unknown, ",") +
                                         " to confirm no GPU of this pool is held",
                                     "", true));
    return Outcome::transient("agent(s) unreachable during finalization: " + join(o.unknown, ","));
  }
  std::string lost;  // nodes of claims whose reply was lost and that have not answered since
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = suspect_.find(m.uid);
    if (it != suspect_.end()) lost = join(std::vector<std::string>(it->second.begin(), it->second.end()), ",");
  }
  if (!lost.empty()) {
    write_status_(obj, build_status_(obj, m, spec, o, "Deleting",
                                     "waiting for agent(s) on " + lost + " (a claim reply was lost)", "", true));
    return Outcome::transient("claim outcome unknown on " + lost);
  }
  std::vector<std::string> cordon;
  for (const auto& d : o.mine)
    if (d.state != "Draining") cordon.push_back(d.uuid);
  if (!cordon.empty()) {
    for (const auto& kv : by_node(o, cordon)) provider_.cordon(kv.first, m.uid, kv.second);
    event_(obj, "Normal", "DrainStarted", "pool deleting: draining " + std::to_string(cordon.size()) + " GPU(s)");
    o = observe_(m, spec, obj["status"]);
  }
  int still = drain_(obj, o.node, m, spec, o.mine);
  if (!o.mine.empty()) o = observe_(m, spec, obj["status"]);
  if (still > 0 || !o.mine.empty()) {
    write_status_(obj, build_status_(obj, m, spec, o, "Draining", std::to_string(still) + " GPU(s) still have pods",
                                     "", true));
    return Outcome::requeue(opts_.progress_poll, "draining");
  }
  if (m.has_finalizer(gen::kFinalizer)) {
    remove_finalizer_(obj);
    event_(obj, "Normal", "Finalized", "all GPUs released; finalizer removed");
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    evicted_.erase(m.uid);
    eviction_blocked_.erase(m.uid);
    policy_sent_.erase(m.uid);
    span_backoff_.erase(m.uid);
    suspect_.erase(m.uid);
  }
  {
    std::lock_guard<std::mutex> g(quota_mu_);
    quota_holds_.erase(m.uid);
  }
  forget_(m.uid);
  ready_gauge().erase({{"kind", kind_}, {"pool", m.key()}});
  desired_gauge().erase({{"kind", kind_}, {"pool", m.key()}});
  erase_util_gauges({{"kind", kind_}, {"pool", m.key()}});
  return Outcome::done(ms(0));
}

PoolPlan plan_pool(const Mi355xPoolSpec& spec, const std::vector<DeviceView>& mine) {
  PoolPlan plan;
  std::vector<const DeviceView*> keep;
  for (const auto& d : mine) {
    if (d.state == "Draining") continue;  // already on its way out
    const bool bad = d.probe_overdue || (d.state != "Probing" && (!d.healthy || !d.probe_passed));
    if (bad && spec.replace_policy == "Replace") plan.replace.push_back(d.uuid);
    else keep.push_back(&d);
  }
  auto n = static_cast<int64_t>(keep.size());
  if (n > spec.replicas) {
    // Deterministic victims (fixes README.md:214's arbitrary existingVMs[:n]): unhealthy first,
    // then GPUs without pods, then the smallest node of a spanning pool, then the highest index.
    std::map<std::string, int> on_node;
    for (const DeviceView* d : keep) ++on_node[d->node];
    std::sort(keep.begin(), keep.end(), [&on_node](const DeviceView* a, const DeviceView* b) {
      bool ua = !a->healthy || !a->probe_passed, ub = !b->healthy || !b->probe_passed;
      if (ua != ub) return ua;
      bool pa = a->pods.size() > 0, pb = b->pods.size() > 0;
      if (pa != pb) return !pa;
      if (on_node[a->node] != on_node[b->node]) return on_node[a->node] < on_node[b->node];
      if (a->node != b->node) return a->node > b->node;
      return a->index > b->index;
    });
    for (int64_t i = 0; i < n - spec.replicas; ++i) plan.victims.push_back(keep[static_cast<size_t>(i)]->uuid);
    n = spec.replicas;
  }
  plan.keep = n;
  plan.need = std::max<int64_t>(0, spec.replicas - n);
  return plan;
}

Outcome Mi355xPoolReconciler::reconcile(const std::string& ns, const std::string& name) {
  auto cached = pools_.get(ns, name);
  if (!cached) return Outcome::done(ms(0));  // gone (finalizer already removed)
  Json obj = *cached;
  ObjectMeta m = ObjectMeta::from(obj);
  Logger log = log_.with("pool", m.key()).with("generation", m.generation);
  auto errs = validate_mi355x(obj);
  if (!errs.empty()) {
    Json st = obj["status"].is_object() ? obj["status"] : Json::object();
    Json conds = st["conditions"].is_array() ? st["conditions"] : Json::array();
    set_condition(conds, gen::kCondReady, "False", "InvalidSpec", join(errs, "; "), m.generation, rfc3339_now());
    st["conditions"] = conds;
    st["observedGeneration"] = m.generation;
    write_status_(obj, st);
    return Outcome::terminal("invalid spec: " + join(errs, "; "));
  }
  Mi355xPoolSpec spec = Mi355xPoolSpec::from(obj["spec"]);
  note_generation_(m);
  if (m.deleting()) return finalize_(obj, m, spec);
  if (!m.has_finalizer(gen::kFinalizer)) {
    obj = ensure_finalizer_(obj);
    m = ObjectMeta::from(obj);
  }

  Observed o = observe_(m, spec, obj["status"]);
  if (!o.reachable && !o.node.empty()) {
    const Json cur = fresh_(obj);  // the devices it keeps come from the newest status, not a lagging copy
    write_status_(cur, build_status_(cur, m, spec, o, "", "", "", false));
    ready_gauge().set({{"kind", kind_}, {"pool", m.key()}}, 0);
    return Outcome::transient("agent on " + o.node + " unreachable: " + o.error);
  }
  // Push the (possibly edited) health policy to the agent owning our GPUs — only when the policy
  // itself changed (a replicas-only edit bumps the generation but not the policy).
  const std::string policy_key = spec.policy_json().dump() + "|" + spec.resource_name;
  if (!o.mine.empty()) {
    bool push;
    {
      std::lock_guard<std::mutex> g(mu_);
      push = policy_sent_[m.uid] != policy_key;
    }
    if (push) {
      for (const auto& n : o.nodes) provider_.update_policy(n, m.uid, spec.policy_json(), spec.resource_name);
      std::lock_guard<std::mutex> g(mu_);
      policy_sent_[m.uid] = policy_key;
    }
  }

  std::string progress_reason, progress_msg;
  std::string blocked;  // reason scale-up is blocked (InsufficientDevices | QuotaExceeded)
  bool acted = false;
  bool claimed_only = false;  // the only action was a successful claim
  std::vector<DeviceView> claimed;
  std::string claimed_node;
  const PoolPlan plan = plan_pool(spec, o.mine);
  std::vector<std::string> cordon = plan.replace;
  for (const auto& u : plan.replace) {
    const DeviceView* d = nullptr;
    for (const auto& x : o.mine)
      if (x.uuid == u) d = &x;
    std::vector<std::string> r;
    for (const auto& x : d->verdict["reasons"].elements()) r.push_back(x.as_string());
    if (d->probe_overdue) r.push_back("ProbeTimeout: still probing past spec.probe.timeoutSeconds");
    else if (!d->probe_passed) r.push_back("ProbeFailed: " + d->probe["error"].str_or("probe failed"));
    event_(obj, "Warning", "HealthDegraded", short_id(*d) + " unhealthy (" + join(r, "; ") + "): replacing");
    progress_reason = "ReplacingUnhealthy";
    progress_msg = "replacing " + short_id(*d);
  }
  if (!plan.victims.empty()) {
    cordon.insert(cordon.end(), plan.victims.begin(), plan.victims.end());
    progress_reason = "ScalingDown";
    progress_msg = "draining " + std::to_string(plan.victims.size()) + " GPU(s): " + join(plan.victims, ",");
    event_(obj, "Normal", "DrainStarted", progress_msg);
  }
  int64_t n_active = plan.keep;
  if (!cordon.empty()) {
    for (const auto& kv : by_node(o, cordon)) provider_.cordon(kv.first, m.uid, kv.second);
    acted = true;
  }
  std::string quota_msg, quota_reason;
  bool over_quota = n_active < spec.replicas &&
                    !quota_reserve_(m, spec, static_cast<int>(spec.replicas - n_active), &quota_msg, &quota_reason);
  if (over_quota) {
    blocked = quota_reason;
    progress_msg = quota_msg;
    event_(obj, "Warning", quota_reason, quota_msg);
  } else if (n_active < spec.replicas && spans_(spec)) {
    // spec.maxNodes > 1: the delta may be split over nodes; all-or-nothing per pass (a claim that
    // fails part-way hands back what this pass already claimed on the other nodes).
    int need = static_cast<int>(spec.replicas - n_active);
    bool backing_off;
    {
      std::lock_guard<std::mutex> g(mu_);
      backing_off = span_backoff_.count(m.uid) && clock_t_::now() < span_backoff_[m.uid];
    }
    auto plan = backing_off ? std::vector<std::pair<std::string, int>>{} : plan_span_(spec, need, o);
    if (backing_off) {
      blocked = "InsufficientDevices";
      progress_msg = "a spanning claim of " + std::to_string(need) + " GPU(s) was rolled back; retrying shortly";
    } else if (plan.empty()) {
      blocked = "InsufficientDevices";
      progress_msg = "need " + std::to_string(need) + " free healthy GPU(s) on at most " +
                     std::to_string(spec.max_nodes) + " node(s)";
      event_(obj, "Warning", "InsufficientDevices", progress_msg);
    } else {
      std::vector<std::pair<std::string, std::vector<std::string>>> made;
      std::vector<DeviceView> got;
      std::string fail_reason, fail_msg;
      for (const auto& step : plan) {
        ClaimRequest req;
        req.pool_uid = m.uid;
        req.pool = m.key();
        req.count = step.second;
        req.topology_policy = spec.topology_policy;
        req.resource_name = spec.resource_name;
        req.policy = spec.policy_json();
        req.probe = spec.probe_json();
        ClaimResult cr = claim_(step.first, req);
        if (!cr.ok) {
          fail_reason = cr.reason.empty() ? "InsufficientDevices" : cr.reason;
          fail_msg = step.first + ": " + cr.message;
          break;
        }
        std::vector<std::string> uuids;
        for (auto& d : cr.devices) {
          uuids.push_back(d.uuid);
          got.push_back(std::move(d));
        }
        made.emplace_back(step.first, std::move(uuids));
      }
      acted = true;
      if (!fail_reason.empty()) {
        for (const auto& kv : made) provider_.release(kv.first, m.uid, kv.second);
        {
          std::lock_guard<std::mutex> g(mu_);
          span_backoff_[m.uid] = clock_t_::now() + ms(5000);
        }
        blocked = fail_reason;
        progress_msg = fail_reason + ": " + fail_msg + (made.empty() ? "" : " (this pass's other claims released)");
        event_(obj, "Warning", fail_reason, progress_msg);
      } else {
        if (progress_reason.empty()) progress_reason = "ScalingUp";
        std::vector<std::string> where;
        for (const auto& kv : made) where.push_back(std::to_string(kv.second.size()) + " on " + kv.first);
        progress_msg = "claimed " + std::to_string(got.size()) + " GPU(s): " + join(where, ", ");
        event_(obj, "Normal", "GPUClaimed", progress_msg);
        {
          std::lock_guard<std::mutex> g(mu_);
          policy_sent_[m.uid] = policy_key;
        }
        log.info("claimed", Json::object().set("nodes", static_cast<long long>(made.size())).set("count", need));
        {
          std::lock_guard<std::mutex> g(mu_);
          span_backoff_.erase(m.uid);
        }
        claimed_only = cordon.empty();
        claimed = std::move(got);
        claimed_node = made.front().first;
      }
    }
  } else if (n_active < spec.replicas) {
    int need = static_cast<int>(spec.replicas - n_active);
    // A pool lives on one node: extend where it already is, else try the fitting nodes in order.
    std::vector<std::string> candidates = o.mine.empty() ? choose_nodes_(spec, need) : std::vector<std::string>{o.node};
    const bool cordoned = !o.mine.empty() && !provider_.node_schedulable(o.node);
    if (cordoned) candidates.clear();  // a cordoned node keeps its GPUs but takes no new claims
    if (candidates.empty()) {
      blocked = "InsufficientDevices";
      progress_msg = cordoned ? "node " + o.node + " is cordoned (spec.unschedulable): no new GPUs claimed there"
                              : "no eligible node has " + std::to_string(need) + " free healthy GPU(s)";
      event_(obj, "Warning", "InsufficientDevices", progress_msg);
    }
    for (size_t ci = 0; ci < candidates.size(); ++ci) {
      const std::string& node = candidates[ci];
      ClaimRequest req;
      req.pool_uid = m.uid;
      req.pool = m.key();
      req.count = need;
      req.topology_policy = spec.topology_policy;
      req.resource_name = spec.resource_name;
      req.policy = spec.policy_json();
      req.probe = spec.probe_json();
      auto t = clock_t_::now();
      ClaimResult cr = claim_(node, req);
      double claim_ms = std::chrono::duration<double, std::milli>(clock_t_::now() - t).count();
      if (!cr.ok) {
        const std::string reason = cr.reason.empty() ? "InsufficientDevices" : cr.reason;
        // raced with another pool for this node's capacity: try the next candidate
        if (reason == "InsufficientDevices" && ci + 1 < candidates.size()) continue;
        blocked = reason;
        progress_msg = reason + ": " + cr.message;
        event_(obj, "Warning", reason, cr.message);
        acted = true;
        break;
      } else {
        std::vector<std::string> ids;
        for (const auto& d : cr.devices) ids.push_back(short_id(d));
        if (progress_reason.empty()) progress_reason = "ScalingUp";
        progress_msg = "claimed " + std::to_string(cr.devices.size()) + " GPU(s) on " + node;
        event_(obj, "Normal", "GPUClaimed", progress_msg + ": " + join(ids, ", "));
        {
          std::lock_guard<std::mutex> g(mu_);
          policy_sent_[m.uid] = policy_key;
        }
        log.info("claimed", Json::object().set("node", node).set("count", need).set("claimMs", claim_ms));
        claimed_only = !acted;
        claimed = std::move(cr.devices);
        claimed_node = node;
        acted = true;
        break;
      }
    }
  }
  if (claimed_only) {
    // The claim RPC returns the agent's post-claim ground truth for the new GPUs (probed and,
    // with a device plugin, already advertised); the rest of o.mine was observed this pass and
    // nothing else changed, so merging replaces a second GET /v1/node (A1 still holds).
    if (o.node.empty() || !spans_(spec)) o.node = claimed_node;
    o.reachable = true;
    for (auto& d : claimed) {
      if (o.free_by_node.count(d.node)) o.free_by_node[d.node] = std::max<int64_t>(0, o.free_by_node[d.node] - 1);
      o.mine.push_back(std::move(d));
    }
    o.free_healthy = std::max<int64_t>(0, o.free_healthy - static_cast<int64_t>(claimed.size()));
    std::sort(o.mine.begin(), o.mine.end(), [](const DeviceView& a, const DeviceView& b) {
      return a.node != b.node ? a.node < b.node : a.index < b.index;
    });
    index_nodes(o, spans_(spec));
  } else if (acted) {
    o = observe_(m, spec, obj["status"]);
  }
  int still = drain_(obj, o.node, m, spec, o.mine);
  bool released = false;
  for (const auto& d : o.mine)
    if (d.state == "Draining" && d.pods.size() == 0) released = true;
  if (released) o = observe_(m, spec, obj["status"]);  // A1: status from ground truth after acting
  if (still > 0 && progress_reason.empty()) {
    progress_reason = "Draining";
    progress_msg = std::to_string(still) + " GPU(s) waiting for pods to terminate";
  }
  {
    // Converged within this pass (claimed, probed, advertised, nothing draining): report Stable now
    // instead of leaving Progressing=True until the next resync.
    int64_t ready_now = 0, active_now = 0;
    bool inflight = false;
    for (const auto& d : o.mine) {
      if (d.state == "Draining" || d.state == "Probing") inflight = true;
      else ++active_now;
      if (d.state == "Claimed" && d.healthy && d.probe_passed && d.advertised) ++ready_now;
    }
    if (!inflight && blocked.empty() && ready_now == spec.replicas && active_now == spec.replicas) progress_reason.clear();
  }
  Json status = build_status_(obj, m, spec, o, progress_reason, progress_msg, blocked, false);
  write_status_(obj, status);
  quota_settle_(m, spec, static_cast<int64_t>(o.mine.size()));  // draining GPUs are still held
  int64_t ready = status["readyReplicas"].as_int(0);
  ready_gauge().set({{"kind", kind_}, {"pool", m.key()}}, static_cast<double>(ready));
  set_util_gauges({{"kind", kind_}, {"pool", m.key()}}, o.mine);
  bool is_ready = condition_true(status["conditions"], gen::kCondReady);
  observe_ready_(m, is_ready, spec.replicas);
  if (!blocked.empty()) return Outcome::requeue(ms(5000), blocked);
  bool draining = false;
  for (const auto& d : o.mine) draining = draining || d.state == "Draining" || d.state == "Probing";
  if (draining || !is_ready) return Outcome::requeue(opts_.progress_poll, progress_reason);
  return Outcome::done(opts_.resync);
}

// Per-namespace GPU quota (the reference's ResourceQuota practice,
// GPU调度平台搭建.md:802): a ResourceQuota with spec.hard["<resourceName>"] or
// spec.hard["requests.<resourceName>"] caps the devices of that resource all pools in the namespace
// may offer, in the resource's own units like the pods' requests it also bounds: a GPU counts once,
// a shared GPU (spec.sharing.replicasPerGPU = K) K times.
//
// Admission is a reservation, not a read: the workers reconcile pools in parallel and the informer
// copy of another pool's status lags its claim (and even our own last write lags the watch), so
// "sum status.replicas from the cache, then claim" let three concurrent replicas=2 pools all pass a
// quota of 3. Under quota_mu_ the usage of every pool of the namespace+resource is
// max(informer status.replicas x K, units this manager last wrote for it) + units reserved by
// passes whose claim is still in flight; a pass that fits reserves its delta before the claim RPC.
// The lock is never held across an RPC (only across the quota LIST when no informer is synced).
bool Mi355xPoolReconciler::quota_reserve_(const ObjectMeta& m, const Mi355xPoolSpec& spec, int delta,
                                          std::string* why, std::string* reason) {
  trace::Span span("quota");
  std::lock_guard<std::mutex> g(quota_mu_);
  std::vector<Json> items;
  if (quotas_ && quotas_->synced()) {
    for (auto& q : quotas_->list())
      if (q.path("metadata.namespace").as_string() == m.ns) items.push_back(std::move(q));
  } else {
    try {
      Json quotas = client_.list(res::resourcequotas(), m.ns);
      items = quotas["items"].elements();
    } catch (const std::exception& e) {
      // Quotas unreadable: the namespace's limit is unknown, so a scale-up could exceed it. Fail
      // closed (the tenancy promise of a quota, GPU调度平台搭建.md:802) and retry; clusters that use
      // no quotas run with --quota-fail-open.
      if (opts_.quota_fail_open) return true;
      *reason = "QuotaUnknown";
      *why = "ResourceQuotas of namespace " + m.ns + " cannot be read (" + e.what() +
             "): scale-up blocked until they can (--quota-fail-open admits it)";
      return false;
    }
  }
  int64_t hard = -1;
  std::string qname;
  for (const auto& q : items) {
    for (const std::string& key : {spec.resource_name, "requests." + spec.resource_name}) {
      const Json& h = q.path("spec.hard")[key];
      if (h.is_null()) continue;
      int64_t v = h.is_number() ? h.as_int() : std::atoll(h.as_string().c_str());
      if (hard < 0 || v < hard) {
        hard = v;
        qname = q.path("metadata.name").as_string();
      }
    }
  }
  if (hard < 0) return true;
  std::map<std::string, int64_t> per_pool;  // uid -> units
  std::set<std::string> live{m.uid};
  for (const auto& p : pools_.list()) {
    live.insert(p.path("metadata.uid").as_string());
    if (p.path("metadata.namespace").as_string() != m.ns) continue;
    if (p.path("spec.resourceName").str_or(gen::kDefaultResource) != spec.resource_name) continue;
    per_pool[p.path("metadata.uid").as_string()] =
        p.path("status.replicas").as_int(0) * std::max<int64_t>(1, p.path("spec.sharing.replicasPerGPU").as_int(1));
  }
  int64_t used = 0;
  for (auto it = quota_holds_.begin(); it != quota_holds_.end();) {
    // A pool that left the cache without a finalizer pass (finalizer force-removed) holds nothing:
    // its hold goes with it, or its namespace's quota stays consumed until a manager restart.
    if (!live.count(it->first)) {
      it = quota_holds_.erase(it);
      continue;
    }
    const auto& [uid, h] = *it++;
    if (h.ns != m.ns || h.resource != spec.resource_name) continue;
    int64_t& u = per_pool[uid];
    u = std::max(u, h.written) + (uid == m.uid ? 0 : h.reserved);
  }
  for (const auto& kv : per_pool) used += kv.second;
  const int64_t more = static_cast<int64_t>(delta) * spec.sharing_replicas;
  quota_gauge().set({{"namespace", m.ns}, {"resource", spec.resource_name}, {"quota", qname}, {"type", "hard"}},
                    static_cast<double>(hard));
  quota_gauge().set({{"namespace", m.ns}, {"resource", spec.resource_name}, {"quota", qname}, {"type", "used"}},
                    static_cast<double>(used));
  if (used + more <= hard) {
    QuotaHold& h = quota_holds_[m.uid];
    h.ns = m.ns;
    h.resource = spec.resource_name;
    h.reserved = more;
    quota_gauge().set({{"namespace", m.ns}, {"resource", spec.resource_name}, {"quota", qname}, {"type", "used"}},
                      static_cast<double>(used + more));
    return true;
  }
  *reason = "QuotaExceeded";
  *why = "ResourceQuota " + m.ns + "/" + qname + " allows " + std::to_string(hard) + " " + spec.resource_name +
         "; " + std::to_string(used) + " in use or reserved, " + std::to_string(more) + " more requested";
  return false;
}

void Mi355xPoolReconciler::quota_settle_(const ObjectMeta& m, const Mi355xPoolSpec& spec, int64_t replicas) {
  std::lock_guard<std::mutex> g(quota_mu_);
  QuotaHold& h = quota_holds_[m.uid];
  h.ns = m.ns;
  h.resource = spec.resource_name;
  h.written = replicas * spec.sharing_replicas;
  h.reserved = 0;
}

std::vector<std::pair<std::string, std::string>> Mi355xPoolReconciler::sweep_orphans() {
  std::set<std::string> live;
  // single-node pools by uid -> (namespace, name, the node their status names)
  std::map<std::string, std::array<std::string, 3>> single;
  for (const auto& p : pools_.list()) {
    const std::string uid = p.path("metadata.uid").as_string();
    live.insert(uid);
    const Mi355xPoolSpec spec = Mi355xPoolSpec::from(p["spec"]);
    const std::string node = p.path("status.nodeName").as_string();
    if (!spans_(spec) && !node.empty())
      single[uid] = {p.path("metadata.namespace").as_string(), p.path("metadata.name").as_string(), node};
  }
  std::vector<std::pair<std::string, std::string>> wake;
  for (const auto& n : provider_.node_names()) {
    NodeView nv = provider_.observe(n);
    if (!nv.reachable) continue;
    std::map<std::string, std::vector<std::string>> orphans;
    std::set<std::string> misplaced;
    for (const auto& d : nv.devices) {
      if (!d.pool_uid.empty() && !live.count(d.pool_uid) && d.pods.size() == 0) orphans[d.pool_uid].push_back(d.uuid);
      auto it = single.find(d.pool_uid);
      if (it != single.end() && it->second[2] != n) misplaced.insert(d.pool_uid);
    }
    // GPUs of a live single-node pool on a node its status does not name: a claim whose reply was
    // lost before a manager restart (the in-memory record of it went with the old process). The
    // pool's own pass decides — adopt or release — serialised with its other passes.
    for (const auto& uid : misplaced) {
      {
        std::lock_guard<std::mutex> g(mu_);
        suspect_[uid].insert(n);
      }
      log_.warn("GPUs of a pool on a node its status does not name",
                Json::object().set("node", n).set("poolUID", uid).set("pool", single[uid][0] + "/" + single[uid][1]));
      wake.emplace_back(single[uid][0], single[uid][1]);
    }
    for (const auto& kv : orphans) {
      log_.warn("releasing orphaned claims", Json::object().set("node", n).set("poolUID", kv.first).set("count", static_cast<long long>(kv.second.size())));
      try {
        provider_.release(n, kv.first, kv.second);
      } catch (const std::exception& e) {
        log_.warn("orphan release failed", Json::object().set("error", e.what()));
      }
    }
  }
  return wake;
}

}  // namespace gpupool

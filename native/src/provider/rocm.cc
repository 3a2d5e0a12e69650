// RocmProvider: the MI355X provider. Where the reference called the Azure Go SDK over HTTPS
// (README.md:179-221), this talks to the node agent that owns the node's GPUs (claim ledger,
// libmi355x_dev telemetry, HIP probe, device plugin) over HTTP/1.1 JSON — a unix socket on the
// same host, or TCP across nodes. In a cluster an agent is found through its own Pod (the IP the
// kubelet/CNI gave the agent Pod bound to that node, AgentAccess "pod"); local setups name it in
// the Node's gpupool.amd.com/agent-endpoint annotation. Every request carries a per-request
// Ed25519 signature bound to the node (agentauth.h), so no endpoint ever receives a credential it
// could replay against another agent — least privilege, as README.md:43-57 scopes its SP.
#include "gpupool/generated/schema_consts.h"
#include "gpupool/informer.h"
#include "gpupool/metrics.h"
#include "gpupool/provider.h"
#include "gpupool/leader.h"
#include "gpupool/trace.h"

#include <cstdlib>
#include <fstream>
#include <thread>
#include <tuple>

namespace gpupool {

DeviceView DeviceView::from(const Json& j) {
  DeviceView d;
  d.uuid = j["uuid"].as_string();
  d.hip_uuid = j["hipUUID"].as_string();
  d.bdf = j["bdf"].as_string();
  d.render_node = j["renderNode"].as_string();
  d.node = j["node"].as_string();
  d.index = j["index"].as_int(-1);
  d.kfd_node = j["kfdNode"].as_int(-1);
  d.state = j["state"].str_or("Free");
  d.pool_uid = j["poolUID"].as_string();
  d.pool = j["pool"].as_string();
  d.healthy = j["healthy"].as_bool(false);
  d.advertised = j["advertised"].as_bool(false);
  d.probe_passed = j.path("probe.passed").as_bool(false);
  d.probe_overdue = d.state == "Probing" && j["probeOverdue"].as_bool(false);
  d.verdict = j["verdict"];
  d.probe = j["probe"];
  d.pods = j["pods"].is_array() ? j["pods"] : Json::array();
  d.claimed_at = j["claimedAt"].as_string();
  d.partition = j["partition"];
  d.drain_started_at = j["drainStartedAt"].as_string();
  d.hbm_sweep = j["hbmSweep"];
  d.xgmi_pairs = j["xgmiPairs"];
  d.sharing = j["sharing"];
  d.telemetry = j["telemetry"];
  return d;
}

Json DeviceView::status_json() const {
  Json s = Json::object();
  s["uuid"] = uuid;
  if (!hip_uuid.empty()) s["hipUUID"] = hip_uuid;
  if (!bdf.empty()) s["bdf"] = bdf;
  s["index"] = index;
  s["node"] = node;
  if (!render_node.empty()) s["renderNode"] = render_node;
  if (kfd_node >= 0) s["kfdNode"] = kfd_node;
  std::string h = state == "Draining" ? "Draining" : state == "Probing" ? "Probing" : healthy && probe_passed ? "Healthy" : "Unhealthy";
  s["health"] = h;
  Json reasons = Json::array();
  for (const auto& r : verdict["reasons"].elements()) reasons.push_back(r);
  if (probe.is_object() && !probe_passed && state != "Probing") {
    std::string msg = probe["error"].str_or(probe["message"].str_or("probe failed"));
    reasons.push_back("ProbeFailed: " + msg);
  }
  if (probe_overdue) reasons.push_back("ProbeTimeout: still probing past spec.probe.timeoutSeconds");
  s["reasons"] = reasons;
  s["advertised"] = advertised;
  Json pods_out = Json::array();
  for (const auto& p : pods.elements()) pods_out.push_back(p.is_string() ? p : Json(p["namespace"].as_string() + "/" + p["name"].as_string()));
  s["pods"] = pods_out;
  if (!claimed_at.empty()) s["claimedAt"] = claimed_at;
  if (partition.is_object() && partition.size()) s["partition"] = partition;
  if (probe.is_object()) {
    Json p = Json::object();
    p["passed"] = probe_passed;
    if (probe.path("hbm.GBps").is_number()) p["hbmGBps"] = probe.path("hbm.GBps");
    if (probe.path("mfma.tflops").is_number()) p["mfmaTflops"] = probe.path("mfma.tflops");
    if (probe.path("xgmi.GBps").is_number()) p["xgmiGBps"] = probe.path("xgmi.GBps");
    if (probe["ms"].is_number()) p["ms"] = probe["ms"];
    if (probe["backend"].is_string()) p["backend"] = probe["backend"];
    if (probe["error"].is_string()) p["message"] = probe["error"];
    if (probe.path("cus.mfmaVerified").is_number()) {
      p["cusVerified"] = probe.path("cus.mfmaVerified");
      p["cusExpected"] = probe.path("cus.expected");
    }
    s["probe"] = p;
  }
  if (sharing.is_object() && sharing.size()) s["sharing"] = sharing;  // slot isolation (agent slots.py)
  if (hbm_sweep.is_object()) {  // HBM scrubber coverage of this GPU (agent's rotating sweep)
    Json c = Json::object();
    for (const char* k : {"passes", "fraction", "span", "cursor", "lastFullSweepAt", "lastBadBits"})
      if (!hbm_sweep[k].is_null()) c[k] = hbm_sweep[k];
    s["hbmCoverage"] = c;
  }
  if (xgmi_pairs.is_object() || probe.path("xgmi.unavailable").as_bool(false)) {
    // xGMI link coverage of this GPU: pairs with the node's other GPUs the agent's peer-copy
    // rings (claims + idle rechecks, rotating order) have checked, and which peers failed
    Json x = Json::object();
    for (const char* k : {"pairsCovered", "pairsTotal", "failedPeers", "unavailablePeers", "lastCheckedAt"})
      if (!xgmi_pairs[k].is_null()) x[k] = xgmi_pairs[k];
    if (probe.path("xgmi.unavailable").as_bool(false)) x["peerCheckUnavailable"] = true;
    s["xgmi"] = x;
  }
  return s;
}

RocmProvider::RocmProvider(Informer& nodes, int timeout_ms, AgentAccess access)
    : nodes_(nodes), timeout_ms_(timeout_ms), access_(std::move(access)) {
  if (access_.discovery == "pod" && !access_.pods)
    throw std::invalid_argument("agent discovery \"pod\" needs an agent pods informer");
  // the handler first, then the informer's current contents: an update in between is applied by
  // the handler and then again (same or newer state) by the seed
  nodes_.add_handler([this](const std::string& type, const Json& obj) { note_node_(type, obj); });
  for (const auto& n : nodes_.list()) note_node_("ADDED", n);
  if (access_.pods) {
    access_.pods->add_handler([this](const std::string& type, const Json& obj) { note_agent_pod_(type, obj); });
    for (const auto& p : access_.pods->list()) note_agent_pod_("ADDED", p);
  }
}

void RocmProvider::note_node_(const std::string& type, const Json& obj) {
  const std::string name = obj.path("metadata.name").as_string();
  if (name.empty()) return;
  std::lock_guard<std::mutex> g(facts_mu_);
  if (type == "DELETED") {
    facts_.erase(name);
    return;
  }
  NodeFacts& f = facts_[name];
  f.labels = obj.path("metadata.labels").is_object() ? obj.path("metadata.labels") : Json::object();
  f.schedulable = !obj.path("spec.unschedulable").as_bool(false);
  f.annotation = obj.path("metadata.annotations")[gen::kAnnAgentEndpoint].str_or("");
  f.kx = obj.path("metadata.annotations")[gen::kAnnAgentKx].str_or("");
  derive_endpoint_(name, f);
}

void RocmProvider::note_agent_pod_(const std::string& type, const Json& pod) {
  const std::string node = pod.path("spec.nodeName").as_string();
  const std::string key = Informer::key_of(pod);
  const std::string ip = pod.path("status.podIP").as_string();
  const bool live = type != "DELETED" && !ip.empty() && pod.path("status.phase").as_string() == "Running" &&
                    !pod.path("metadata.deletionTimestamp").is_string();
  std::lock_guard<std::mutex> g(facts_mu_);
  // a pod's node never changes, but a DELETED event may carry it: drop the key everywhere
  for (auto it = agent_pods_.begin(); it != agent_pods_.end();) {
    it->second.erase(key);
    it = it->second.empty() ? agent_pods_.erase(it) : std::next(it);
  }
  if (live && !node.empty()) {
    bool ready = false;
    for (const auto& c : pod.path("status.conditions").elements())
      if (c["type"].str_or("") == "Ready") ready = c["status"].str_or("") == "True";
    agent_pods_[node][key] = AgentPod{ip, ready, pod.path("metadata.creationTimestamp").str_or("")};
  }
  if (!node.empty()) {
    auto f = facts_.find(node);
    if (f != facts_.end()) derive_endpoint_(node, f->second);
  }
}

void RocmProvider::derive_endpoint_(const std::string& node, NodeFacts& f) {
  if (access_.discovery != "pod") {
    f.endpoint = f.annotation;
    return;
  }
  auto it = agent_pods_.find(node);
  if (it == agent_pods_.end() || it->second.empty()) {
    f.endpoint.clear();  // no running agent pod on the node: nothing to call
    return;
  }
  // a DaemonSet runs one per node, but a surge rollout briefly runs two: the Ready one, then the
  // newer one (the old pod is about to go)
  const AgentPod* best = nullptr;
  for (const auto& kv : it->second)
    if (!best || std::tie(kv.second.ready, kv.second.created) > std::tie(best->ready, best->created))
      best = &kv.second;
  const std::string& ip = best->ip;
  const std::string host = ip.find(':') != std::string::npos ? "[" + ip + "]" : ip;
  f.endpoint = access_.scheme + "://" + host + ":" + std::to_string(access_.port);
  if (!f.annotation.empty() && f.annotation != f.endpoint) {
    // honoured only when it names the agent Pod's own address (another port or scheme)
    bool same_host = false;
    try {
      Url u = Url::parse(f.annotation);
      same_host = u.scheme != "unix" && (u.host == ip || u.host == host);
    } catch (const std::exception&) {
    }
    if (same_host) {
      f.endpoint = f.annotation;
    } else {
      endpoints_rejected_.fetch_add(1);
      static CounterVec& rej = Registry::global().counter(
          "gpupool_agent_endpoint_rejected_total",
          "Node agent-endpoint annotations ignored: the host is not the node's agent Pod IP.");
      rej.inc({{"node", node}});
    }
  }
}

std::unique_ptr<HttpClient> RocmProvider::new_client(const std::string& node, const std::string& endpoint,
                                                     int timeout_ms) {
  std::unique_ptr<HttpClient> c;
  if (access_.signer) {
    // signatures replace the bearer: the endpoint gets nothing it could replay elsewhere
    c = std::make_unique<HttpClient>(Url::parse(endpoint), std::shared_ptr<TokenSource>(), timeout_ms, access_.tls);
    std::shared_ptr<AgentSigner> signer = access_.signer;
    // v2 (a MAC keyed per node) once the agent has published its key-exchange key, else v1
    c->set_signer([this, signer, node](const std::string& m, const std::string& target, const std::string& body) {
      return signer->header(m, target, node, body, agent_kx_(node));
    });
  } else {
    c = std::make_unique<HttpClient>(Url::parse(endpoint), access_.token, timeout_ms, access_.tls);
  }
  return c;
}

std::string RocmProvider::agent_kx_(const std::string& node) {
  std::lock_guard<std::mutex> g(facts_mu_);
  auto it = facts_.find(node);
  if (it == facts_.end()) return "";
  auto bad = bad_kx_.find(node);
  return bad != bad_kx_.end() && bad->second == it->second.kx ? std::string() : it->second.kx;
}

void RocmProvider::distrust_kx(const std::string& node) {
  std::lock_guard<std::mutex> g(facts_mu_);
  mark_kx_bad_locked_(node);
}

// one count per (node, key) refused, whichever path saw the 401 first (an RPC or the long-poll feed)
bool RocmProvider::mark_kx_bad_locked_(const std::string& node) {
  auto it = facts_.find(node);
  if (it == facts_.end() || it->second.kx.empty() || bad_kx_[node] == it->second.kx) return false;
  bad_kx_[node] = it->second.kx;
  static CounterVec& c = Registry::global().counter(
      "gpupool_agent_kx_refused_total", "Agent RPCs refused for a stale key-exchange key (re-sent with Ed25519).");
  c.inc({{"node", node}});
  return true;
}

bool RocmProvider::stale_kx_(const std::string& node, const HttpResponse& r) {
  if (r.status != 401) return false;
  auto j = Json::try_parse(r.body);
  const std::string why = j ? (*j)["reason"].str_or("") : "";
  if (why != "StaleAgentKey" && why != "NoAgentKey") return false;
  std::lock_guard<std::mutex> g(facts_mu_);
  if (mark_kx_bad_locked_(node)) return true;
  // another path (the feed) marked this key first: the request went out MACed before that, so
  // re-send it signed — it was refused before its body was read
  auto it = facts_.find(node);
  return it != facts_.end() && !it->second.kx.empty();
}

std::vector<std::string> RocmProvider::node_names() {
  std::vector<std::string> out;
  std::lock_guard<std::mutex> g(facts_mu_);
  for (const auto& kv : facts_)
    if (!kv.second.endpoint.empty()) out.push_back(kv.first);
  return out;
}

Json RocmProvider::node_labels(const std::string& node) {
  std::lock_guard<std::mutex> g(facts_mu_);
  auto it = facts_.find(node);
  return it == facts_.end() ? Json::object() : it->second.labels;
}

bool RocmProvider::node_schedulable(const std::string& node) {
  std::lock_guard<std::mutex> g(facts_mu_);
  auto it = facts_.find(node);
  return it == facts_.end() || it->second.schedulable;
}

std::string RocmProvider::endpoint_of(const std::string& node) {
  std::lock_guard<std::mutex> g(facts_mu_);
  auto it = facts_.find(node);
  return it == facts_.end() ? "" : it->second.endpoint;
}

std::shared_ptr<HttpClient> RocmProvider::client_for(const std::string& node) {
  std::string ep = endpoint_of(node);
  if (ep.empty()) throw ProviderError("AgentNotFound", "no gpupool agent registered on node " + node);
  std::lock_guard<std::mutex> g(mu_);
  auto& slot = clients_[node];
  if (!slot.second || slot.first != ep) {
    slot.first = ep;
    slot.second = std::shared_ptr<HttpClient>(new_client(node, ep, timeout_ms_));
  }
  return slot.second;
}

Json RocmProvider::post_(const std::string& node, const std::string& path, const Json& body) {
  {
    std::lock_guard<std::mutex> g(cache_mu_);
    ++inflight_[node];
  }
  struct Done {
    RocmProvider* p;
    const std::string& node;
    ~Done() {
      std::lock_guard<std::mutex> g(p->cache_mu_);
      if (--p->inflight_[node] == 0) p->cache_cv_.notify_all();
    }
  } done{this, node};
  if (!leader_fence_ok())  // a paused leader must not claim or release after another took over
    throw ProviderError("NotLeader", "agent on " + node + ": " + path + " not sent: leadership not renewed in time");
  // The check above is local: a leader paused right after it would still send. The fencing token
  // makes the agent the judge — it refuses an epoch older than one it has seen (StaleLeader).
  std::string fence;
  if (const LeaderToken tok = leader_token(); tok.epoch >= 0)
    fence = "X-Gpupool-Leader: " + tok.identity + "\r\nX-Gpupool-Leader-Epoch: " + std::to_string(tok.epoch) +
            "\r\nX-Gpupool-Leader-Lease: " + tok.lease_created + " " + tok.lease_uid + "\r\n";
  test_pause_after_fence_(path);
  invalidate_(node);  // every POST mutates the agent: the next observe must ask it
  trace::Span span("agent:POST " + path);
  std::shared_ptr<HttpClient> c = client_for(node);
  HttpResponse r;
  try {
    r = c->request("POST", path, body.dump(), "application/json", "application/json", -1, fence);
    // refused before its body was read (nothing executed): once more, signed with Ed25519
    if (stale_kx_(node, r)) r = c->request("POST", path, body.dump(), "application/json", "application/json", -1, fence);
  } catch (const std::exception& e) {
    throw ProviderError("AgentUnreachable", "agent on " + node + ": " + e.what());
  }
  {
    std::lock_guard<std::mutex> g(cache_mu_);
    ++answered_[node];
  }
  auto j = Json::try_parse(r.body);
  if (r.status >= 400) {
    std::string msg = j ? (*j)["message"].str_or(r.body) : r.body;
    std::string code = j ? (*j)["reason"].str_or("AgentError") : "AgentError";
    throw ProviderError(code, "agent on " + node + " " + path + ": HTTP " + std::to_string(r.status) + ": " + msg,
                        r.status >= 500);
  }
  return j ? *j : Json::object();
}

// Test hook (chaos tests only): with $GPUPOOL_TEST_FENCE_HOLD_DIR set, a mutating RPC whose path
// has a file "<dir>/hold<path with / as _>" waits — after its fence check and token, before the
// send — until that file is removed: the "leader paused between check and act" the fencing token
// is for. Unset in production: one getenv per RPC.
void RocmProvider::test_pause_after_fence_(const std::string& path) {
  static const char* dir = std::getenv("GPUPOOL_TEST_FENCE_HOLD_DIR");
  if (!dir || !*dir) return;
  std::string tag;
  for (char ch : path) tag.push_back(ch == '/' ? '_' : ch);
  const std::string f = std::string(dir) + "/hold" + tag;
  bool marked = false;
  for (int i = 0; i < 6000; ++i) {  // at most 60 s
    std::ifstream in(f);
    if (!in.good()) return;
    std::string who;  // the file names the identity to hold (empty: any)
    std::getline(in, who);
    if (!who.empty() && who != leader_token().identity) return;
    if (!marked) {  // tell the test the send is being held
      std::ofstream(std::string(dir) + "/held" + tag) << leader_token().epoch << "\n";
      marked = true;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
}

NodeView RocmProvider::observe(const std::string& node) {
  NodeView nv = observe_pool(node, "");
  if (nv.reachable) {
    std::lock_guard<std::mutex> g(cache_mu_);
    note_capacity_(node, nv);
  }
  return nv;
}

void RocmProvider::note_capacity_(const std::string& node, const NodeView& full) {
  Capacity& c = cap_[node];
  c.free = 0;
  for (const auto& d : full.devices)
    if (d.state == "Free" && d.healthy) ++c.free;
  c.taken = 0;  // the view already shows what was claimed before it (pending claims still count)
  c.at = std::chrono::steady_clock::now();
  c.valid = true;
}

int64_t RocmProvider::free_capacity(const std::string& node) {
  {
    std::lock_guard<std::mutex> g(cache_mu_);
    auto it = cap_.find(node);
    if (it != cap_.end() && it->second.valid &&
        std::chrono::steady_clock::now() - it->second.at < std::chrono::milliseconds(view_max_age_ms_)) {
      static CounterVec& hits = Registry::global().counter(
          "gpupool_capacity_estimate_hits_total", "Placement capacity answered without an agent RPC.");
      hits.inc({{"node", node}});
      const Capacity& c = it->second;
      return std::max<int64_t>(0, c.free - c.taken - c.pending);
    }
  }
  NodeView nv = observe(node);  // refreshes cap_
  if (!nv.reachable) return -1;
  std::lock_guard<std::mutex> g(cache_mu_);
  const Capacity& c = cap_[node];
  return std::max<int64_t>(0, c.free - c.taken - c.pending);
}

uint64_t RocmProvider::answered(const std::string& node) {
  std::lock_guard<std::mutex> g(cache_mu_);
  auto it = answered_.find(node);
  return it == answered_.end() ? 0 : it->second;
}

void RocmProvider::note_gen(const std::string& node, int64_t gen) {
  std::lock_guard<std::mutex> g(cache_mu_);
  latest_gen_[node] = gen;
}

void RocmProvider::invalidate_(const std::string& node) {
  std::lock_guard<std::mutex> g(cache_mu_);
  cache_[node].valid = false;
  ++epoch_[node];
}

void RocmProvider::prefetch(const std::string& node, int max_wait_ms) {
  uint64_t epoch;
  {
    std::unique_lock<std::mutex> g(cache_mu_);
    // system_clock deadline: libstdc++ then waits with pthread_cond_timedwait, which TSan
    // intercepts (a steady_clock wait_for uses pthread_cond_clockwait, which GCC 11's TSan misses)
    if (max_wait_ms > 0)
      cache_cv_.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(max_wait_ms),
                           [&] { return inflight_[node] == 0; });
    // a mutating RPC is in flight: its reply invalidates the cache anyway, and the caller (the
    // node's event-stream thread) must not stall behind it — skip, the next observe asks the agent
    if (inflight_[node] > 0) return;
    epoch = epoch_[node];
  }
  NodeView v = observe_pool(node, "");  // the full view (an RPC: the cache serves pools only)
  if (!v.reachable) return;
  std::lock_guard<std::mutex> g(cache_mu_);
  auto lg = latest_gen_.find(node);
  if (epoch_[node] != epoch || (lg != latest_gen_.end() && v.gen < lg->second)) return;  // raced
  note_capacity_(node, v);
  CachedView& c = cache_[node];
  c.valid = true;
  c.at = std::chrono::steady_clock::now();
  c.view = std::move(v);
}

NodeView RocmProvider::observe_pool(const std::string& node, const std::string& pool_uid) {
  if (!pool_uid.empty()) {
    std::lock_guard<std::mutex> g(cache_mu_);
    auto it = cache_.find(node);
    auto lg = latest_gen_.find(node);
    if (it != cache_.end() && it->second.valid && lg != latest_gen_.end() && it->second.view.gen == lg->second &&
        std::chrono::steady_clock::now() - it->second.at < std::chrono::milliseconds(view_max_age_ms_)) {
      trace::Span span("agent:view-cache");
      const NodeView& full = it->second.view;
      NodeView nv;
      nv.name = full.name;
      nv.endpoint = full.endpoint;
      nv.backend = full.backend;
      nv.reachable = true;
      nv.advertise_required = full.advertise_required;
      nv.gen = full.gen;
      nv.free_healthy = 0;
      for (const auto& d : full.devices) {
        if (d.pool_uid == pool_uid) nv.devices.push_back(d);
        else if (d.state == "Free" && d.healthy) ++nv.free_healthy;
      }
      cache_hits_.fetch_add(1);
      static CounterVec& hits = Registry::global().counter(
          "gpupool_agent_view_cache_hits_total", "Pool observes answered from the agent view cache (no RPC).");
      hits.inc({{"node", node}});
      return nv;
    }
  }
  NodeView nv;
  nv.name = node;
  nv.endpoint = endpoint_of(node);
  trace::Span span("agent:GET /v1/node");
  try {
    std::shared_ptr<HttpClient> c = client_for(node);
    const std::string target = pool_uid.empty() ? "/v1/node" : "/v1/node?pool=" + pool_uid;
    HttpResponse r = c->request("GET", target);
    if (stale_kx_(node, r)) r = c->request("GET", target);
    {
      std::lock_guard<std::mutex> g(cache_mu_);
      ++answered_[node];
    }
    if (r.status >= 400) throw ProviderError("AgentError", "GET /v1/node: HTTP " + std::to_string(r.status));
    Json j = Json::parse(r.body);
    nv.reachable = true;
    nv.backend = j["backend"].as_string();
    nv.gen = j["gen"].as_int(0);
    nv.advertise_required = j["advertiseRequired"].as_bool(true);
    nv.free_healthy = j["freeHealthy"].as_int(-1);
    for (const auto& d : j["devices"].elements()) {
      DeviceView v = DeviceView::from(d);
      if (v.node.empty()) v.node = node;
      nv.devices.push_back(std::move(v));
    }
  } catch (const std::exception& e) {
    nv.reachable = false;
    nv.error = e.what();
  }
  return nv;
}

ClaimResult RocmProvider::claim(const std::string& node, const ClaimRequest& req) {
  Json body = Json::object();
  body["poolUID"] = req.pool_uid;
  body["pool"] = req.pool;
  body["count"] = req.count;
  body["topologyPolicy"] = req.topology_policy;
  body["resourceName"] = req.resource_name;
  body["policy"] = req.policy;
  body["probe"] = req.probe;
  {
    std::lock_guard<std::mutex> g(cache_mu_);
    cap_[node].pending += req.count;
  }
  struct Unpend {
    RocmProvider* p;
    const std::string& node;
    int64_t n;
    ~Unpend() {
      std::lock_guard<std::mutex> g(p->cache_mu_);
      p->cap_[node].pending -= n;
    }
  } unpend{this, node, req.count};
  Json r = post_(node, "/v1/claims", body);
  ClaimResult out;
  out.ok = r["ok"].as_bool(false);
  {
    std::lock_guard<std::mutex> g(cache_mu_);
    Capacity& c = cap_[node];
    if (out.ok)
      c.taken += static_cast<int64_t>(r["devices"].elements().size());
    else
      c.valid = false;  // refused (capacity, sharing limits): ask the agent next time
  }
  out.reason = r["reason"].as_string();
  out.message = r["message"].as_string();
  for (const auto& d : r["devices"].elements()) out.devices.push_back(DeviceView::from(d));
  // the agent's own phase timings (select/commit/probe/advertise) become child spans
  for (const auto& kv : r["timingsMs"].members()) trace::add_span("agent.claim." + kv.first, kv.second.as_double(0));
  return out;
}

static Json uuid_body(const std::string& pool_uid, const std::vector<std::string>& uuids) {
  Json body = Json::object();
  body["poolUID"] = pool_uid;
  Json arr = Json::array();
  for (const auto& u : uuids) arr.push_back(u);
  body["uuids"] = arr;
  return body;
}

void RocmProvider::cordon(const std::string& node, const std::string& pool_uid, const std::vector<std::string>& uuids) {
  post_(node, "/v1/cordon", uuid_body(pool_uid, uuids));
}

void RocmProvider::release(const std::string& node, const std::string& pool_uid, const std::vector<std::string>& uuids) {
  post_(node, "/v1/release", uuid_body(pool_uid, uuids));
  std::lock_guard<std::mutex> g(cache_mu_);
  cap_[node].valid = false;  // GPUs came back (or went to quarantine): count them again
}

void RocmProvider::update_policy(const std::string& node, const std::string& pool_uid, const Json& policy,
                                 const std::string& resource_name) {
  Json body = Json::object();
  body["poolUID"] = pool_uid;
  body["policy"] = policy;
  body["resourceName"] = resource_name;
  post_(node, "/v1/policy", body);
}

}  // namespace gpupool

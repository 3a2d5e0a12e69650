// Provider layer (reference A5: getAzureVMClient/listManagedVMs/createVM/deleteVM,
// README.md:179-221, contract README.md:238-240).
//
// Two provider families:
//  * CloudProvider — the AzureVmPool contract (tag-scoped ownership, full cleanup of NIC + OS
//    disk, idempotent create/delete). FakeCloudProvider implements it in-process (optionally
//    persisted to a JSON file) because there is no Azure access here; provisioning is
//    asynchronous (Creating -> Succeeded after a configurable delay) like ARM long-running ops.
//  * DeviceProvider — the MI355X contract: enumerate physical GPUs per node, claim a delta
//    all-or-nothing (gang-style), cordon/release, with per-device health verdicts.
//    RocmProvider implements it by talking to each node's agent (HTTP over unix socket or TCP);
//    the agent owns the claim ledger, libmi355x_dev and the HIP probe.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gpupool/api.h"
#include "gpupool/agentauth.h"
#include "gpupool/http.h"
#include "gpupool/json.h"

namespace gpupool {

class Informer;

// ============================================================== cloud (AzureVmPool)
struct Credentials {
  std::map<std::string, std::string> values;
};

struct VmRecord {
  std::string name, id, state;  // state: Creating | Succeeded | Deleting | Failed
  std::string resource_group, location, vm_size, nic, os_disk, created_at, message;
  std::map<std::string, std::string> tags;
  Json to_json() const;
};

class ProviderError : public std::runtime_error {
 public:
  ProviderError(std::string code, const std::string& msg, bool transient = true)
      : std::runtime_error(msg), code(std::move(code)), transient(transient) {}
  std::string code;
  bool transient;
};

class CloudProvider {
 public:
  virtual ~CloudProvider() = default;
  // Tag-scoped listing: managed-by=azurevmpool-operator, owner=<ns>-<name> (README.md:238).
  virtual std::vector<VmRecord> list(const Credentials& c, const std::string& rg, const std::string& owner) = 0;
  // Starts an asynchronous create (idempotent on name). Returns the record in Creating state.
  virtual VmRecord create(const Credentials& c, const AzureVmPoolSpec& spec, const std::string& owner,
                          const std::string& name) = 0;
  // Starts an asynchronous delete of VM + NIC + OS disk (README.md:216, :239). Idempotent.
  virtual void destroy(const Credentials& c, const std::string& rg, const std::string& name) = 0;
  // NICs / disks of ``owner`` that no longer belong to a VM, as "nic/<name>" / "disk/<name>"
  // (must end up empty; destroy() accepts these ids). NICs are matched by tag; OS disks (ARM
  // gives implicitly created disks no tags) by the exact name "<vm_prefix><slot>-osdisk" of the
  // pool's deterministic VM names.
  virtual std::vector<std::string> orphans(const Credentials& c, const std::string& rg, const std::string& owner,
                                           const std::string& vm_prefix) = 0;
};

struct FakeCloudOptions {
  std::chrono::milliseconds provision{0};
  std::chrono::milliseconds deprovision{0};
  std::string state_file;     // persist the fake cloud across manager restarts
  int quota_per_rg = 1000;    // create beyond this -> QuotaExceeded (transient)
  std::string faults_file;    // {"failCreates": n, "failDeletes": n} consumed one by one
};

class FakeCloudProvider : public CloudProvider {
 public:
  explicit FakeCloudProvider(FakeCloudOptions opts);
  std::vector<VmRecord> list(const Credentials& c, const std::string& rg, const std::string& owner) override;
  VmRecord create(const Credentials& c, const AzureVmPoolSpec& spec, const std::string& owner,
                  const std::string& name) override;
  void destroy(const Credentials& c, const std::string& rg, const std::string& name) override;
  std::vector<std::string> orphans(const Credentials& c, const std::string& rg, const std::string& owner,
                                   const std::string& vm_prefix) override;
  Json dump();  // whole fake cloud (tests)

 private:
  struct Vm {
    VmRecord rec;
    std::chrono::steady_clock::time_point ready_at, gone_at;
    bool deleting = false;
  };
  void advance_locked_();
  void load_();
  void save_locked_();
  bool take_fault_(const char* key);
  void check_creds_(const Credentials& c);
  FakeCloudOptions opts_;
  std::mutex mu_;
  std::map<std::string, Vm> vms_;                       // key rg/name
  std::map<std::string, std::map<std::string, std::string>> nics_, disks_;  // key rg/name -> tags
  uint64_t seq_ = 0;
};

// ============================================================== devices (Mi355xPool)
struct DeviceView {
  std::string uuid, hip_uuid, bdf, render_node, node;
  int64_t index = -1, kfd_node = -1;
  std::string state;  // Free | Claimed | Draining | Quarantined | Probing
  std::string pool_uid, pool;
  bool healthy = false, advertised = false, probe_passed = false;
  // 'Probing' past spec.probe.timeoutSeconds (+ the agent's grace): the claim that probes it is
  // stuck outside its probe helper's deadline — replaced like a failed probe, never waited on
  bool probe_overdue = false;
  Json verdict, probe, pods, partition, hbm_sweep, xgmi_pairs, sharing;
  Json telemetry;     // agent-sampled utilisation: gfx/umc activity %, power W, VRAM used/total
  std::string claimed_at, drain_started_at;
  static DeviceView from(const Json& j);
  Json status_json() const;
};

struct NodeView {
  std::string name, endpoint, backend, error;
  bool reachable = false;
  bool advertise_required = true;
  std::vector<DeviceView> devices;
  int64_t gen = 0;
  int64_t free_healthy = -1;  // pool-scoped views: the agent's count of free healthy GPUs
};

struct ClaimRequest {
  std::string pool_uid, pool;  // pool = ns/name
  int count = 0;
  std::string topology_policy = "xgmi-packed";
  std::string resource_name = "amd.com/gpu";
  Json policy;  // {"health":{...},"partition":{...}}
  Json probe;   // {"enabled","hbmBytes","mfma"}
};

struct ClaimResult {
  bool ok = false;
  std::string reason, message;
  std::vector<DeviceView> devices;
};

class DeviceProvider {
 public:
  virtual ~DeviceProvider() = default;
  virtual std::vector<std::string> node_names() = 0;
  virtual Json node_labels(const std::string& node) = 0;
  // false while the Node is cordoned (spec.unschedulable): no new GPUs are claimed there; pools
  // already on it keep theirs (like pods on a cordoned node)
  virtual bool node_schedulable(const std::string& /*node*/) { return true; }
  virtual NodeView observe(const std::string& node) = 0;
  // Only ``pool_uid``'s GPUs plus the node's free-healthy count (smaller, cheaper answer for the
  // reconcile path). Default: the full view.
  virtual NodeView observe_pool(const std::string& node, const std::string& /*pool_uid*/) { return observe(node); }
  // Free healthy GPUs of ``node`` for placing a new claim (-1: unreachable). A ranking hint only —
  // the claim itself is authoritative (InsufficientDevices makes the caller try the next node).
  // Default: counted from a full observe.
  virtual int64_t free_capacity(const std::string& node) {
    NodeView nv = observe(node);
    if (!nv.reachable) return -1;
    int64_t free = 0;
    for (const auto& d : nv.devices)
      if (d.state == "Free" && d.healthy) ++free;
    return free;
  }
  virtual ClaimResult claim(const std::string& node, const ClaimRequest& req) = 0;
  virtual void cordon(const std::string& node, const std::string& pool_uid, const std::vector<std::string>& uuids) = 0;
  virtual void release(const std::string& node, const std::string& pool_uid, const std::vector<std::string>& uuids) = 0;
  virtual void update_policy(const std::string& node, const std::string& pool_uid, const Json& policy,
                             const std::string& resource_name) = 0;
};

// How the manager finds and authenticates each node's agent.
struct AgentAccess {
  // "pod": the endpoint is <scheme>://<podIP>:<port> of the agent Pod the scheduler bound to the
  //        node (pods informer, namespace + label selector) — addresses the kubelet/CNI assign,
  //        which no agent can point at another node. A Node annotation is used only if its host
  //        is that Pod's IP (e.g. to name a different port or scheme), else ignored and counted.
  // "annotation": the Node's gpupool.amd.com/agent-endpoint as written (local / dev setups,
  //        unix sockets).
  std::string discovery = "annotation";
  Informer* pods = nullptr;  // required for "pod"
  std::string scheme = "https";
  int port = 9443;
  // credentials: per-request Ed25519 signatures bound to the node (preferred; no bearer is sent
  // then) and/or a shared bearer token from a rotating source
  std::shared_ptr<AgentSigner> signer;
  std::shared_ptr<TokenSource> token;
  TlsOptions tls;  // how https:// agent endpoints are verified
};

// Agents are found per node (AgentAccess::discovery) and called over HTTP/1.1 JSON.
class RocmProvider : public DeviceProvider {
 public:
  RocmProvider(Informer& nodes, int timeout_ms = 30000, AgentAccess access = {});
  // how https:// agent endpoints are verified (CA of the agents' serving certificates)
  const TlsOptions& agent_tls() const { return access_.tls; }
  // A client for ``node``'s agent at ``endpoint`` carrying this manager's credentials for that
  // node (the event feed's long-polls; client_for caches one per node for RPCs).
  std::unique_ptr<HttpClient> new_client(const std::string& node, const std::string& endpoint, int timeout_ms);
  uint64_t endpoints_rejected() const { return endpoints_rejected_.load(); }
  std::vector<std::string> node_names() override;
  Json node_labels(const std::string& node) override;
  bool node_schedulable(const std::string& node) override;
  NodeView observe(const std::string& node) override;
  NodeView observe_pool(const std::string& node, const std::string& pool_uid) override;
  // From the node's last full view (younger than view_max_age) less the GPUs claimed there since
  // and those claims in flight, so concurrent placements spread instead of all racing for the same
  // tightest node; a full view (an RPC) only when there is none. Releases and a claim refused for
  // capacity drop the estimate (the next call asks the agent).
  int64_t free_capacity(const std::string& node) override;
  ClaimResult claim(const std::string& node, const ClaimRequest& req) override;
  void cordon(const std::string& node, const std::string& pool_uid, const std::vector<std::string>& uuids) override;
  void release(const std::string& node, const std::string& pool_uid, const std::vector<std::string>& uuids) override;
  void update_policy(const std::string& node, const std::string& pool_uid, const Json& policy,
                     const std::string& resource_name) override;
  std::string endpoint_of(const std::string& node);
  // Shared so an in-flight RPC keeps its client alive when the node's endpoint changes (agent
  // restarted elsewhere) and another thread swaps the cached client. Throws ProviderError.
  std::shared_ptr<HttpClient> client_for(const std::string& node);

  // Informer-style cache of the agents' node views. The agent's event feed reports its state
  // generation (note_gen); after a change the feed's thread prefetches the full view. A pool's
  // observe is answered from the cache when it is at the newest generation the manager has heard
  // of, younger than ``view_max_age`` (telemetry keeps moving without generation bumps) and no
  // mutating RPC to that node started since it was fetched; otherwise it is an RPC as before.
  void note_gen(const std::string& node, int64_t gen);
  // The node's event feed broke (agent gone): drop its cached view, so the next observe asks.
  void forget_view(const std::string& node) { invalidate_(node); }
  // Skipped while a mutating RPC to the node is in flight (optionally after waiting up to
  // ``max_wait_ms`` for it): a claim bumps the agent's generation several times and its reply
  // invalidates the cache anyway, and the caller — the node's event-stream thread — must never
  // stall behind RPC traffic (pod-exit and capacity events would queue up behind it).
  void prefetch(const std::string& node, int max_wait_ms = 0);
  void set_view_max_age_ms(int ms) { view_max_age_ms_ = ms; }
  uint64_t view_cache_hits() const { return cache_hits_.load(); }
  // RPCs the node's agent has answered so far: the event feed's reconnect loop backs off while
  // the agent is away and retries at once when a reconcile's RPC shows it is back.
  uint64_t answered(const std::string& node);

 private:
  Json post_(const std::string& node, const std::string& path, const Json& body);
  static void test_pause_after_fence_(const std::string& path);
  void invalidate_(const std::string& node);
  Informer& nodes_;
  int timeout_ms_;
  AgentAccess access_;
  std::atomic<uint64_t> endpoints_rejected_{0};
  std::mutex mu_;
  std::map<std::string, std::pair<std::string, std::shared_ptr<HttpClient>>> clients_;
  struct CachedView {
    bool valid = false;
    std::chrono::steady_clock::time_point at;
    NodeView view;
  };
  std::mutex cache_mu_;
  std::map<std::string, CachedView> cache_;
  std::map<std::string, int64_t> latest_gen_;  // newest agent generation heard of, per node
  std::map<std::string, uint64_t> epoch_;      // bumped by every mutating RPC, per node
  std::map<std::string, int> inflight_;        // mutating RPCs in progress, per node
  std::condition_variable cache_cv_;           // signalled when a node's inflight_ drops to 0
  std::map<std::string, uint64_t> answered_;   // RPCs answered (any status), per node
  int view_max_age_ms_ = 5000;
  std::atomic<uint64_t> cache_hits_{0};
  struct Capacity {
    bool valid = false;
    std::chrono::steady_clock::time_point at;  // when the full view it counts was fetched
    int64_t free = 0;                          // free healthy GPUs in that view
    int64_t taken = 0;                         // GPUs claimed there since
    int64_t pending = 0;                       // GPUs of claims in flight there
  };
  std::map<std::string, Capacity> cap_;  // under cache_mu_
  void note_capacity_(const std::string& node, const NodeView& full);  // caller holds cache_mu_
  // What placement reads of each Node, kept current by a handler on the nodes informer: reading
  // them from the informer copied whole Node objects — four per node per pass of an unplaced pool
  // (~10 ms of CPU per pass at 128 nodes).
  struct NodeFacts {
    Json labels = Json::object();
    bool schedulable = true;
    std::string annotation;  // gpupool.amd.com/agent-endpoint as the Node carries it
    std::string endpoint;    // what the manager calls (derived per AgentAccess::discovery)
    std::string kx;          // gpupool.amd.com/agent-kx: the agent's X25519 key (v2 MAC)
  };
  std::string agent_kx_(const std::string& node);

 public:
  // the node's agent refused a request whose reason the caller could not read (a watch stream's
  // 401): stop MACing with the key its Node names until that changes (Ed25519 always works)
  void distrust_kx(const std::string& node);

 private:
  // a 401 StaleAgentKey / NoAgentKey: the agent has another key-exchange key than its Node says
  // (a wiped state dir, a restart racing its re-registration) — stop MACing with that key until
  // the Node shows a different one (Ed25519 meanwhile); true when the request should be re-sent
  bool stale_kx_(const std::string& node, const HttpResponse& r);
  bool mark_kx_bad_locked_(const std::string& node);  // true when newly marked (counted)
  std::map<std::string, std::string> bad_kx_;  // node -> kx the agent refused (under facts_mu_)
  std::mutex facts_mu_;
  std::map<std::string, NodeFacts> facts_;
  // pod discovery: node -> (agent pod "ns/name" -> its address) of Running, undeleted agent pods
  struct AgentPod {
    std::string ip;
    bool ready = false;
    std::string created;  // RFC 3339: orders as a string
  };
  std::map<std::string, std::map<std::string, AgentPod>> agent_pods_;
  void note_node_(const std::string& type, const Json& obj);
  void note_agent_pod_(const std::string& type, const Json& pod);
  void derive_endpoint_(const std::string& node, NodeFacts& f);  // caller holds facts_mu_
};

}  // namespace gpupool

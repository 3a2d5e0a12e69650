// Pool reconcilers — the MI355X-native re-design of AzureVmPoolReconciler.Reconcile
// (README.md:170-235), fixing the reference's defects:
//   A1 readyReplicas comes from a re-observation AFTER acting, counting only ready instances;
//   A2 typed outcomes (RequeueAfter vs backoff) instead of RequeueAfter+err;
//   A3 status written through the status subresource with conflict retry on a fresh GET;
//   A4 deterministic scale-down victims with cordon + drain + eviction;
//   A5 finalizer-guarded release; A6 full Conditions + status.devices/vms.
#pragma once

#include <atomic>
#include <chrono>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "gpupool/api.h"
#include "gpupool/events.h"
#include "gpupool/informer.h"
#include "gpupool/podindex.h"
#include "gpupool/kube.h"
#include "gpupool/log.h"
#include "gpupool/metrics.h"
#include "gpupool/provider.h"
#include "gpupool/trace.h"
#include "gpupool/workqueue.h"

namespace gpupool {

// Typed reconcile outcome (SURVEY.md §5 failure-detection row).
struct Outcome {
  enum Kind { Done, RequeueAfter, Transient, Terminal } kind = Done;
  std::chrono::milliseconds after{0};
  std::string message;
  static Outcome done(std::chrono::milliseconds resync) { return {Done, resync, ""}; }
  static Outcome requeue(std::chrono::milliseconds d, std::string why = "") { return {RequeueAfter, d, std::move(why)}; }
  static Outcome transient(std::string why) { return {Transient, std::chrono::milliseconds(0), std::move(why)}; }
  static Outcome terminal(std::string why) { return {Terminal, std::chrono::milliseconds(0), std::move(why)}; }
};

struct ReconcilerOptions {
  std::chrono::milliseconds resync{10000};        // steady-state health resync
  std::chrono::milliseconds progress_poll{250};   // while scaling/draining
  std::chrono::milliseconds credentials_retry{30000};  // README.md:184's 30 s, now effective
  bool emit_events = true;
  // ResourceQuotas unreadable (no synced informer, LIST failing): admit scale-ups anyway (clusters
  // that use no quotas) instead of blocking them with QuotaUnknown until the quotas can be read
  bool quota_fail_open = false;
};

// Shared base: status writes with conflict retry, finalizer management, metrics.
class PoolReconcilerBase {
 public:
  PoolReconcilerBase(KubeClient& client, Informer& pools, EventRecorder* events, ReconcilerOptions opts,
                     std::string kind, ResourceRef res);
  virtual ~PoolReconcilerBase() = default;
  virtual Outcome reconcile(const std::string& ns, const std::string& name) = 0;
  const std::string& kind() const { return kind_; }
  // True for the watch event of this reconciler's own status write (its resourceVersion is the
  // one the write returned): nothing a pass acts on changed, so it needs no new pass (the
  // GenerationChanged-style predicate controller-runtime operators use, exact to the write).
  bool own_status_write(const Json& obj);

 protected:
  // Writes ``status`` (unless semantically unchanged) with a fresh-GET retry on 409.
  void write_status_(const Json& obj, const Json& status);
  // called with the object a successful status write returned (read-your-writes caches)
  virtual void on_status_written_(const Json& /*written*/) {}
  // Throws a 409 when the pass read a stale copy whose status placement (nodeName/nodes) differs
  // from the stored one, unless ``writing`` (an object carrying the status being written) already
  // agrees with the stored placement.
  static void stale_placement_check_(const Json& seen, const Json& fresh, const Json* writing = nullptr);
  // Adds/removes the finalizer with RV precondition; returns the updated object.
  Json edit_finalizers_(const Json& obj, bool add);
  Json ensure_finalizer_(const Json& obj);
  Json fresh_(const Json& obj);
  Json remove_finalizer_(const Json& obj);
  void event_(const Json& obj, const std::string& type, const std::string& reason, const std::string& msg);
  void note_generation_(const ObjectMeta& m);  // starts the reconcile-to-Ready clock
  void observe_ready_(const ObjectMeta& m, bool ready, int64_t desired);
  void forget_(const std::string& uid);
  // Placement (nodeName first, then nodes) of this manager's last status write for ``uid``.
  std::vector<std::string> written_placement_(const std::string& uid);

  KubeClient& client_;
  Informer& pools_;
  EventRecorder* events_;
  ReconcilerOptions opts_;
  std::string kind_;
  ResourceRef res_;
  std::string finalizer_;  // gen::kFinalizer for pools
  Logger log_;
  std::mutex mu_;
  // reconcile-to-Ready tracking: uid -> (generation, first time that generation was seen)
  std::map<std::string, std::pair<int64_t, std::chrono::steady_clock::time_point>> pending_;
  std::map<std::string, int64_t> ready_gen_;
  std::map<std::string, std::string> own_rv_;  // uid -> resourceVersion of our last status write
  // uid -> status.nodeName + status.nodes of our last status write: where this manager last put the
  // pool, for passes that run on an informer copy from before that write (see observe_)
  std::map<std::string, std::vector<std::string>> own_place_;
};

// The decision a Mi355xPool pass takes on its observed GPUs, before any RPC (pure; the C++
// decision-table test drives it): which unhealthy GPUs to replace, which GPUs a scale-down drains
// (in order), and how many to claim.
struct PoolPlan {
  std::vector<std::string> replace;  // claimed GPUs failing health or their probe (replacePolicy Replace)
  std::vector<std::string> victims;  // scale-down: unhealthy first, then pod-free, smallest node, highest index
  int64_t keep = 0;                  // GPUs active after this pass
  int64_t need = 0;                  // GPUs to claim this pass (replicas - keep, never negative)
};
PoolPlan plan_pool(const Mi355xPoolSpec& spec, const std::vector<DeviceView>& mine);

class Mi355xPoolReconciler : public PoolReconcilerBase {
 public:
  Mi355xPoolReconciler(KubeClient& client, Informer& pools, DeviceProvider& provider, EventRecorder* events,
                       ReconcilerOptions opts = {});
  Outcome reconcile(const std::string& ns, const std::string& name) override;
  // Releases claims whose pool no longer exists (manager restart / force-deleted CR).
  // Returns (namespace, name) of pools to wake: GPUs of theirs sit on a node status does not name.
  std::vector<std::pair<std::string, std::string>> sweep_orphans();
  // ResourceQuota cache; without one (or before it syncs) quota checks LIST from the API.
  void set_quota_informer(Informer* q) { quotas_ = q; }

 private:
  struct Observed {
    std::string node;                              // the pool's (primary) node
    std::vector<std::string> nodes;                // every node holding GPUs of the pool
    bool reachable = true;
    std::string error;
    std::vector<DeviceView> mine;
    int64_t free_healthy = 0;
    std::map<std::string, int64_t> free_by_node;   // free healthy GPUs per observed node
    std::vector<std::string> unknown;              // unreachable nodes status did not name
    std::vector<std::string> unreachable;          // nodes status names whose agent did not answer
  };
  Observed observe_(const ObjectMeta& m, const Mi355xPoolSpec& spec, const Json& status);
  // Nodes (reachable, selector-matching) with >= need free healthy GPUs, tightest fit first.
  std::vector<std::string> choose_nodes_(const Mi355xPoolSpec& spec, int need);
  // spec.maxNodes > 1: split a scale-up of ``need`` GPUs over the pool's nodes first, then the
  // fewest new selector-matching nodes (most free first). Empty when it does not fit.
  std::vector<std::pair<std::string, int>> plan_span_(const Mi355xPoolSpec& spec, int need, const Observed& o);
  static bool spans_(const Mi355xPoolSpec& spec) { return spec.max_nodes > 1 && spec.node_name.empty(); }
  // Quota admission: under quota_mu_, usage = per pool max(informer status.replicas,
  // the replicas this manager last wrote) + reservations of claims in flight; a pass that fits
  // reserves its delta before the claim RPC, so concurrent passes of different pools cannot both
  // fit the same headroom. quota_settle_ (after the pass's status write) turns the reservation
  // into the written count.
  // false: blocked, ``*reason`` QuotaExceeded (the quota is full) or QuotaUnknown (unreadable)
  bool quota_reserve_(const ObjectMeta& m, const Mi355xPoolSpec& spec, int delta, std::string* why,
                      std::string* reason);
  void quota_settle_(const ObjectMeta& m, const Mi355xPoolSpec& spec, int64_t replicas);
  Outcome finalize_(const Json& obj, const ObjectMeta& m, const Mi355xPoolSpec& spec);
  // Evicts pods on draining devices and releases drained ones. Returns #devices still draining.
  int drain_(const Json& obj, const std::string& node, const ObjectMeta& m, const Mi355xPoolSpec& spec,
             std::vector<DeviceView>& mine);
  Json build_status_(const Json& obj, const ObjectMeta& m, const Mi355xPoolSpec& spec, const Observed& o,
                     const std::string& progress_reason, const std::string& progress_msg, const std::string& blocked,
                     bool deleting);

  DeviceProvider& provider_;
  Informer* quotas_ = nullptr;
  std::map<std::string, std::set<std::string>> evicted_;  // pool uid -> pod keys already evicted
  std::map<std::string, std::set<std::string>> eviction_blocked_;  // pool uid -> pods refused by a PDB (evented)
  // pool uid -> the policy (+ resource name) the agents hold: pushed again only when it changes, so
  // a replicas-only edit (new generation, same policy) costs no /v1/policy RPC
  std::map<std::string, std::string> policy_sent_;
  struct QuotaHold {
    std::string ns, resource;
    int64_t written = 0;   // resource units (GPUs x replicasPerGPU) of our last status write
    int64_t reserved = 0;  // units reserved by a pass whose claim is in flight
  };
  std::mutex quota_mu_;
  std::map<std::string, QuotaHold> quota_holds_;  // pool uid -> hold
  // pool uid -> no spanning claim before this time: a rolled-back pass frees GPUs, whose capacity
  // event would otherwise wake the same pool into the same failing claim at once
  std::map<std::string, std::chrono::steady_clock::time_point> span_backoff_;
  // uid -> nodes where a claim RPC failed in transport (reset, timeout): the agent may have
  // committed it before the reply was lost. observe_ resolves them (adopt / release / forget).
  std::map<std::string, std::set<std::string>> suspect_;
  ClaimResult claim_(const std::string& node, const ClaimRequest& req);
  void resolve_suspects_(const ObjectMeta& m, Observed& o);
};

class AzureVmPoolReconciler : public PoolReconcilerBase {
 public:
  AzureVmPoolReconciler(KubeClient& client, Informer& pools, CloudProvider& cloud, EventRecorder* events,
                        ReconcilerOptions opts = {});
  Outcome reconcile(const std::string& ns, const std::string& name) override;

 private:
  bool credentials_(const ObjectMeta& m, const AzureVmPoolSpec& spec, Credentials* out, std::string* why);
  CloudProvider& cloud_;
};

// Mi355xJob: the GoHai platform's training-job path (reference GPU调度平台搭建.md:638-675 Volcano Job
// with minAvailable/queue/restartPolicy, :300-306 Kubeflow PyTorchJob, PET_* env read at :623)
// as one kind. A job is a gang of `replicas` pods, each requesting `gpusPerReplica` GPUs of a
// pool's extended resource:
//   * placement is all-or-nothing (every pod bound to a node up front, or none), per-queue strict
//     (priority desc, creation) order so a big gang is not starved by smaller ones, packed onto
//     the fewest nodes (tightest single node when the gang fits on one);
//   * the rank-0 pod is created first; the others get MASTER_ADDR = its pod IP (+ MASTER_PORT,
//     WORLD_SIZE/RANK for one-GPU workers, PET_NNODES/PET_NPROC_PER_NODE/PET_NODE_RANK for
//     torchrun), so RCCL/gloo rendezvous needs no Service or DNS;
//   * a failed or lost pod restarts the whole gang (restartPolicy OnFailure, backoffLimit), since
//     DDP ranks cannot rejoin alone; activeDeadlineSeconds, successPolicy, cleanPodPolicy,
//     ttlSecondsAfterFinished and suspend follow the batch/v1 Job and Kubeflow meanings;
//   * preemptionPolicy PreemptLowerPriority (Volcano's preempt action, PriorityClass semantics):
//     a gang that does not fit annotates the fewest lower-priority running jobs whose GPUs make it
//     fit; each victim's own reconciler stops its gang and re-queues it (not a failure restart),
//     while the preemptor holds its reservation and creates pods once the GPUs are really free.
// Reservations of placed-but-not-yet-created pods live in status.placement, and every placement
// decision runs under one mutex against fresh LISTs, so two gangs never share a GPU.
class Mi355xJobReconciler : public PoolReconcilerBase {
 public:
  // ``pods``: the manager's pod index (podindex.h). With it, placement reads jobs, nodes and pod
  // usage from the informers' caches — no cluster-wide LIST per pass; without it (unit tests), the
  // apiserver is LISTed as before.
  Mi355xJobReconciler(KubeClient& client, Informer& jobs, Informer& nodes, EventRecorder* events,
                      ReconcilerOptions opts = {}, PodIndex* pods = nullptr);
  Outcome reconcile(const std::string& ns, const std::string& name) override;
  // Jobs still waiting for a gang placement (re-enqueued when capacity may have freed up).
  std::vector<std::pair<std::string, std::string>> pending() const;
  // How to enqueue a job: a gang queued behind another is woken when that one is placed (or
  // ends: wake_blocked_by), not on every queue or job event.
  void set_waker(std::function<void(const std::string& ns, const std::string& name)> w) { waker_ = std::move(w); }
  void wake_blocked_by(const std::string& ns, const std::string& name) { wake_blocked_by_(ns + "/" + name); }

  struct Slot {
    int index = 0;
    std::string node;
  };
  // Pure placement: free GPUs per node (already ordered candidates) -> one node per replica, or
  // empty when the gang does not fit. Exposed for unit tests.
  static std::vector<Slot> place(const std::vector<std::pair<std::string, int64_t>>& free, int replicas,
                                 int64_t gpus_per_replica);

 private:
  Outcome finish_(const Json& obj, const ObjectMeta& m, const Mi355xJobSpec& spec, Json st, const std::string& phase,
                  const std::string& reason, const std::string& msg, const std::vector<Json>& pods);
  Outcome cleanup_finished_(const Json& obj, const ObjectMeta& m, const Mi355xJobSpec& spec,
                            const std::vector<Json>& pods);
  std::vector<Json> list_pods_(const ObjectMeta& m, const Json& placement);
  // Tries to place the gang (under sched_mu_). Returns the placement, or empty with *why set. With
  // preemptionPolicy PreemptLowerPriority a placement may rely on GPUs of lower-priority running
  // jobs, returned in *victims (the smallest set found, lowest priority and newest first).
  // ``pool_cap``: with a poolRef, the pool's ready device slots per node (status.devices Healthy
  // and advertised x replicasPerGPU) — an upper bound on what the gang may take on each node, so a
  // Node allocatable the kubelet has not lowered yet (the pool just shrank) is not trusted.
  std::vector<Slot> schedule_(const ObjectMeta& m, const Mi355xJobSpec& spec, const std::string& resource,
                              const std::string& pool_node, const std::map<std::string, int64_t>& pool_cap,
                              std::string* reason, std::string* why, std::vector<Json>* victims);
  // True when every not-yet-created slot's node has that many GPUs free right now (pods of
  // preempted jobs may still be terminating on it).
  bool capacity_free_(const Mi355xJobSpec& spec, const std::string& resource, const Json& placement);
  Json build_pod_(const Json& job, const ObjectMeta& m, const Mi355xJobSpec& spec, const std::string& resource,
                  int attempt, int world, const Slot& slot, const std::string& master_addr);
  bool resolve_pool_(const ObjectMeta& m, const Mi355xJobSpec& spec, std::string* resource, std::string* node,
                     std::string* why, std::map<std::string, int64_t>* pool_cap = nullptr);
  // Every job as this reconciler last knows it: the jobs informer's cache, except where our own
  // status write (a gang reservation, written under sched_mu_) is newer than what the watch has
  // delivered yet — read-your-writes, so the next placement never double-books GPUs.
  std::vector<Json> jobs_view_();
  std::vector<Json> node_objects_();
  // node -> GPUs of ``resource`` requested by live pods (the pod index, or one LIST without it)
  std::map<std::string, int64_t> pod_usage_(const std::string& resource);
  void on_status_written_(const Json& written) override;

  void wake_blocked_by_(const std::string& key);
  std::function<void(const std::string&, const std::string&)> waker_;
  std::mutex blocked_mu_;
  std::map<std::string, std::string> blocked_by_;  // "ns/job" queued behind -> "ns/job" ahead
  Informer& nodes_;
  PodIndex* pods_idx_;
  std::mutex sched_mu_;
  std::mutex written_mu_;
  std::map<std::string, Json> written_;  // job uid -> the object our last status write returned
};

// Mi355xQueue status (Volcano queue status): job counts per phase and the GPUs its placed jobs
// hold per extended resource. Admission (state, capability, reclaimable) is enforced by the job
// reconciler's scheduling step; this one only reports.
class Mi355xQueueReconciler : public PoolReconcilerBase {
 public:
  Mi355xQueueReconciler(KubeClient& client, Informer& queues, Informer& jobs, EventRecorder* events,
                        ReconcilerOptions opts = {});
  Outcome reconcile(const std::string& ns, const std::string& name) override;

 private:
  Informer& jobs_;
};

// Mi355xPoolAutoscaler: demand-driven spec.replicas for pools with spec.autoscale.enabled — the
// on-prem counterpart of growing and shrinking the reference's AzureVmPool by hand
// (README.md:292-296, roadmap :309-312) and of the cluster-autoscaler a GPU platform runs beside
// Volcano (GPU调度平台搭建.md:275-287). Demand = GPUs of the pool's resourceName asked for by live
// pods (bound or pending) + gangs of Mi355xJobs still waiting for a placement (their poolRef or
// resource) + reserved-but-uncreated job slots, attributed across pools of the same resource
// (pool_demand), clamped to [minReplicas, maxReplicas]. Scale-up
// is immediate; scale-down only after demand has stayed below spec.replicas for
// scaleDownDelaySeconds, and the pool's drain then releases pod-free GPUs first. Writes are JSON
// merge patches of spec.replicas + two annotations, so they never race the pool's status writes.
class Mi355xPoolAutoscaler : public PoolReconcilerBase {
 public:
  Mi355xPoolAutoscaler(KubeClient& client, Informer& pools, Informer& jobs, Informer& pods, EventRecorder* events,
                       ReconcilerOptions opts = {});
  Outcome reconcile(const std::string& ns, const std::string& name) override;
  // Pools with autoscale enabled (re-evaluated whenever pods or jobs change).
  std::vector<std::pair<std::string, std::string>> autoscaled() const;
  // Pure demand computation over cached pods and jobs; exposed for unit tests.
  static int64_t demand(const std::vector<Json>& pods, const std::vector<Json>& jobs, const std::string& ns,
                        const std::string& pool, const std::string& resource);
  // Demand attributed to one pool when several pools serve the same resource: gangs naming the
  // pool (poolRef) are its own; pods and poolRef-less gangs are served first by fixed-size pools of
  // the resource, the rest is split over autoscaled pools in (namespace, name) order up to their
  // maxReplicas. A single pool gets exactly demand().
  static int64_t pool_demand(const std::vector<Json>& pods, const std::vector<Json>& jobs,
                             const std::vector<Json>& pools, const std::string& ns, const std::string& pool,
                             const std::string& resource);

 private:
  Informer& jobs_;
  Informer& pods_;
  // pool uid -> first pass that saw demand below spec.replicas (the scale-down delay runs from
  // there; a restarted manager starts it over, so it never shrinks early)
  std::map<std::string, std::chrono::steady_clock::time_point> low_since_;
};

// Controller: a shared work queue + N workers dispatching "Kind/ns/name" keys to reconcilers,
// mapping Outcomes onto the queue (Done -> forget + resync; RequeueAfter -> forget + add_after;
// Transient -> rate-limited backoff; Terminal -> forget, wait for the next spec change).
class Controller {
 public:
  explicit Controller(int workers);
  ~Controller();
  void add_reconciler(PoolReconcilerBase* r);
  void enqueue(const std::string& kind, const std::string& ns, const std::string& name);
  void enqueue_after(const std::string& kind, const std::string& ns, const std::string& name,
                     std::chrono::milliseconds d);
  void start();
  void stop();
  WorkQueue& queue() { return q_; }
  uint64_t reconciles() const { return reconciles_.load(); }

 private:
  void worker_();
  int workers_;
  WorkQueue q_;
  std::map<std::string, PoolReconcilerBase*> by_kind_;
  std::vector<std::thread> threads_;
  std::atomic<uint64_t> reconciles_{0};
  Logger log_{"controller"};
};

}  // namespace gpupool

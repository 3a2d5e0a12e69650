// Typed views of the two pool kinds (schema source: gpupool/api/schema.py) plus metav1.Condition
// semantics and validation that mirrors the CRD's OpenAPI checks (defence in depth: the manager
// refuses to act on an object the apiserver should never have admitted).
#pragma once

#include <map>
#include <string>
#include <vector>

#include "gpupool/json.h"

namespace gpupool {

struct ObjectMeta {
  std::string ns, name, uid, resource_version, deletion_timestamp;
  int64_t generation = 0;
  std::vector<std::string> finalizers;
  static ObjectMeta from(const Json& obj);
  bool deleting() const { return !deletion_timestamp.empty(); }
  bool has_finalizer(const std::string& f) const;
  std::string key() const { return ns + "/" + name; }
};

// ---------------------------------------------------------------- AzureVmPool (README.md:92-118)
struct ImageReference {
  std::string publisher, offer, sku, version;
};

struct AzureVmPoolSpec {
  int32_t replicas = 0;
  std::string resource_group, location, vm_size, vnet, subnet, credential_secret;
  ImageReference image;
  static AzureVmPoolSpec from(const Json& spec);
};

// ---------------------------------------------------------------- Mi355xPool
struct HealthPolicy {
  int64_t max_uncorrectable_ecc = 0;
  int64_t max_correctable_ecc = 100000;
  bool require_all_xgmi = true;
  int32_t min_xgmi_up = 7;
  std::string thermal = "belowCritical";
  int32_t thermal_margin_c = 0;
  int64_t max_retired_pages = 64;                 // HBM pages retired by the driver (absolute)
  int64_t max_pending_pages = 0;                  // bad pages awaiting retirement
  int64_t max_lifetime_uncorrectable_ecc = -1;    // -1: unset (only the delta since claim counts)
  Json to_json() const;
};

struct Mi355xPoolSpec {
  int32_t replicas = 0;
  std::string node_name;
  std::map<std::string, std::string> node_selector;
  std::string resource_name = "amd.com/gpu";
  std::string topology_policy = "xgmi-packed";
  std::string partition_compute = "Any", partition_memory = "Any";
  HealthPolicy health;
  int64_t drain_grace_seconds = 30;
  bool drain_evict = true;
  int64_t drain_timeout_seconds = 300;
  bool probe_enabled = true;
  int64_t probe_hbm_bytes = 1LL << 30;
  bool probe_mfma = true;
  double probe_min_hbm_gbps = 0;     // performance floors (0 = off)
  double probe_min_mfma_tflops = 0;
  int64_t probe_recheck_seconds = 0;  // periodic re-probe of idle claimed GPUs (0 = off)
  bool probe_xgmi_peer_check = false;   // ring peer-copy check across the pool's GPUs
  double probe_min_xgmi_gbps = 0;
  double probe_timeout_seconds = 10;  // per-GPU probe deadline (agent's probe helper)
  Json probe_json() const;            // the probe options sent with claims and policy updates
  std::string replace_policy = "Replace";
  int32_t max_nodes = 1;  // nodes the pool may span
  int32_t sharing_replicas = 1;  // time-sliced slots advertised per GPU (spec.sharing.replicasPerGPU)
  int64_t sharing_hbm_bytes = 0;  // per-slot HBM budget (spec.sharing.hbmBytesPerSlot; 0 = none)
  int32_t sharing_cus = 0;        // per-slot CU share (spec.sharing.cuPerSlot; 0 = all CUs)
  std::string sharing_over_budget = "Flag";  // Flag | Evict (agent-enforced)
  bool autoscale = false;  // demand-driven spec.replicas (Mi355xPoolAutoscaler)
  int32_t autoscale_min = 0, autoscale_max = 8;
  int64_t scale_down_delay_seconds = 300;
  static Mi355xPoolSpec from(const Json& spec);
  Json policy_json() const;  // health + partition, as the agent/device library consume it
};

// ---------------------------------------------------------------- Mi355xJob
// Gang-scheduled distributed training job (schema: gpupool/api/schema.py MI355X_JOB_SPEC).
struct Mi355xJobSpec {
  int32_t replicas = 1;
  int32_t min_available = 0;  // 0 = replicas (rigid gang)
  int32_t gpus_per_replica = 1;
  std::string resource_name;  // "" = the poolRef's, else amd.com/gpu
  std::string pool_ref;
  std::map<std::string, std::string> node_selector;
  std::string queue = "default";
  int32_t priority = 0;
  std::string preemption_policy = "Never";  // | PreemptLowerPriority
  bool suspend = false;
  std::string restart_policy = "OnFailure";
  int32_t backoff_limit = 3;
  int64_t active_deadline_seconds = 0;
  int64_t ttl_seconds_after_finished = -1;
  std::string clean_pod_policy = "Running";
  std::string success_policy = "AllWorkers";
  int32_t master_port = 29500;
  std::string checkpoint_dir;  // -> GPUPOOL_CHECKPOINT_DIR
  Json tmpl;  // PodTemplateSpec
  // Smallest gang the job may start with (minAvailable clamped to [1, replicas]).
  int32_t min_workers() const { return min_available > 0 && min_available < replicas ? min_available : replicas; }
  static Mi355xJobSpec from(const Json& spec);
};

// Validation mirroring the CRD schema; returns "field: message" strings.
std::vector<std::string> validate_azure(const Json& obj);
std::vector<std::string> validate_mi355x(const Json& obj);
std::vector<std::string> validate_job(const Json& obj);

// ---------------------------------------------------------------- conditions
// meta.SetStatusCondition semantics: merge by type; lastTransitionTime moves only on a status
// flip. Returns true if anything changed. ``conditions`` must be an array (or null).
bool set_condition(Json& conditions, const std::string& type, const std::string& status,
                   const std::string& reason, const std::string& message, int64_t generation,
                   const std::string& now);
const Json& find_condition(const Json& conditions, const std::string& type);
bool condition_true(const Json& conditions, const std::string& type);

}  // namespace gpupool

#include "gpupool/api.h"

#include <algorithm>
#include <regex>

namespace gpupool {

ObjectMeta ObjectMeta::from(const Json& obj) {
  ObjectMeta m;
  const Json& md = obj["metadata"];
  m.ns = md["namespace"].as_string();
  m.name = md["name"].as_string();
  m.uid = md["uid"].as_string();
  m.resource_version = md["resourceVersion"].as_string();
  m.deletion_timestamp = md["deletionTimestamp"].as_string();
  m.generation = md["generation"].as_int(0);
  for (const auto& f : md["finalizers"].elements()) m.finalizers.push_back(f.as_string());
  return m;
}

bool ObjectMeta::has_finalizer(const std::string& f) const {
  return std::find(finalizers.begin(), finalizers.end(), f) != finalizers.end();
}

AzureVmPoolSpec AzureVmPoolSpec::from(const Json& s) {
  AzureVmPoolSpec a;
  a.replicas = static_cast<int32_t>(s["replicas"].as_int(0));
  a.resource_group = s["resourceGroupName"].as_string();
  a.location = s["location"].as_string();
  a.vm_size = s["vmSize"].as_string();
  a.vnet = s["vnetName"].as_string();
  a.subnet = s["subnetName"].as_string();
  a.credential_secret = s["azureCredentialSecret"].as_string();
  const Json& img = s["imageReference"];
  a.image = {img["publisher"].as_string(), img["offer"].as_string(), img["sku"].as_string(),
             img["version"].as_string()};
  return a;
}

Json HealthPolicy::to_json() const {
  Json j = Json::object();
  j["maxUncorrectableECC"] = max_uncorrectable_ecc;
  j["maxCorrectableECC"] = max_correctable_ecc;
  j["requireAllXGMILinks"] = require_all_xgmi;
  j["minXGMILinksUp"] = min_xgmi_up;
  j["thermal"] = thermal;
  j["thermalMarginC"] = thermal_margin_c;
  j["maxRetiredPages"] = max_retired_pages;
  j["maxPendingPages"] = max_pending_pages;
  if (max_lifetime_uncorrectable_ecc >= 0) j["maxLifetimeUncorrectableECC"] = max_lifetime_uncorrectable_ecc;
  return j;
}

Mi355xPoolSpec Mi355xPoolSpec::from(const Json& s) {
  Mi355xPoolSpec p;
  p.replicas = static_cast<int32_t>(s["replicas"].as_int(0));
  p.node_name = s["nodeName"].as_string();
  for (const auto& kv : s["nodeSelector"].members()) p.node_selector[kv.first] = kv.second.as_string();
  p.resource_name = s["resourceName"].str_or("amd.com/gpu");
  p.topology_policy = s["topologyPolicy"].str_or("xgmi-packed");
  p.partition_compute = s.path("partition.compute").str_or("Any");
  p.partition_memory = s.path("partition.memory").str_or("Any");
  const Json& h = s["health"];
  p.health.max_uncorrectable_ecc = h["maxUncorrectableECC"].as_int(0);
  p.health.max_correctable_ecc = h["maxCorrectableECC"].as_int(100000);
  p.health.require_all_xgmi = h["requireAllXGMILinks"].as_bool(true);
  p.health.min_xgmi_up = static_cast<int32_t>(h["minXGMILinksUp"].as_int(7));
  p.health.thermal = h["thermal"].str_or("belowCritical");
  p.health.thermal_margin_c = static_cast<int32_t>(h["thermalMarginC"].as_int(0));
  p.health.max_retired_pages = h["maxRetiredPages"].as_int(64);
  p.health.max_pending_pages = h["maxPendingPages"].as_int(0);
  p.health.max_lifetime_uncorrectable_ecc =
      h.contains("maxLifetimeUncorrectableECC") ? h["maxLifetimeUncorrectableECC"].as_int(-1) : -1;
  const Json& d = s["drain"];
  p.drain_grace_seconds = d["gracePeriodSeconds"].as_int(30);
  p.drain_evict = d["evict"].as_bool(true);
  p.drain_timeout_seconds = d["timeoutSeconds"].as_int(300);
  const Json& pr = s["probe"];
  p.probe_enabled = pr["enabled"].as_bool(true);
  p.probe_hbm_bytes = pr["hbmBytes"].as_int(1LL << 30);
  p.probe_mfma = pr["mfma"].as_bool(true);
  p.probe_min_hbm_gbps = pr["minHbmGBps"].as_double(0);
  p.probe_min_mfma_tflops = pr["minMfmaTflops"].as_double(0);
  p.probe_recheck_seconds = pr["recheckSeconds"].as_int(0);
  p.probe_xgmi_peer_check = pr["xgmiPeerCheck"].as_bool(false);
  p.probe_min_xgmi_gbps = pr["minXgmiGBps"].as_double(0);
  p.probe_timeout_seconds = pr["timeoutSeconds"].as_double(10);
  p.replace_policy = s["replacePolicy"].str_or("Replace");
  p.max_nodes = static_cast<int32_t>(s["maxNodes"].as_int(1));
  p.sharing_replicas = static_cast<int32_t>(std::max<int64_t>(1, s.path("sharing.replicasPerGPU").as_int(1)));
  p.sharing_hbm_bytes = std::max<int64_t>(0, s.path("sharing.hbmBytesPerSlot").as_int(0));
  p.sharing_cus = static_cast<int32_t>(std::max<int64_t>(0, s.path("sharing.cuPerSlot").as_int(0)));
  p.sharing_over_budget = s.path("sharing.overBudgetAction").str_or("Flag");
  const Json& a = s["autoscale"];
  p.autoscale = a["enabled"].as_bool(false);
  p.autoscale_min = static_cast<int32_t>(a["minReplicas"].as_int(0));
  p.autoscale_max = static_cast<int32_t>(a["maxReplicas"].as_int(8));
  p.scale_down_delay_seconds = a["scaleDownDelaySeconds"].as_int(300);
  return p;
}

Json Mi355xPoolSpec::probe_json() const {
  Json j = Json::object();
  j["enabled"] = probe_enabled;
  j["hbmBytes"] = probe_hbm_bytes;
  j["mfma"] = probe_mfma;
  j["minHbmGBps"] = probe_min_hbm_gbps;
  j["minMfmaTflops"] = probe_min_mfma_tflops;
  j["recheckSeconds"] = probe_recheck_seconds;
  j["xgmiPeerCheck"] = probe_xgmi_peer_check;
  j["minXgmiGBps"] = probe_min_xgmi_gbps;
  j["timeoutSeconds"] = probe_timeout_seconds;
  return j;
}

Json Mi355xPoolSpec::policy_json() const {
  Json j = Json::object();
  j["health"] = health.to_json();
  j["partition"]["compute"] = partition_compute;
  j["partition"]["memory"] = partition_memory;
  j["probe"] = probe_json();  // re-probe settings live with the claim (agent-side recheck)
  if (sharing_replicas > 1) j["sharing"]["replicasPerGPU"] = sharing_replicas;  // device-plugin slots
  // isolation of the slots (the agent's Allocate loads libgpupool_share.so into the pod)
  if (sharing_hbm_bytes > 0) j["sharing"]["hbmBytesPerSlot"] = sharing_hbm_bytes;
  if (sharing_cus > 0) j["sharing"]["cuPerSlot"] = sharing_cus;
  if (sharing_over_budget != "Flag") j["sharing"]["overBudgetAction"] = sharing_over_budget;
  return j;
}

namespace {

void require_string(const Json& s, const char* field, std::vector<std::string>& errs) {
  if (!s.contains(field)) {
    errs.push_back(std::string("spec.") + field + ": Required value");
  } else if (!s[field].is_string()) {
    errs.push_back(std::string("spec.") + field + ": must be of type string");
  }
}

bool in(const std::string& v, std::initializer_list<const char*> xs) {
  for (const char* x : xs)
    if (v == x) return true;
  return false;
}

}  // namespace

std::vector<std::string> validate_azure(const Json& obj) {
  std::vector<std::string> errs;
  const Json& s = obj["spec"];
  if (!s.is_object()) return {"spec: Required value"};
  if (!s["replicas"].is_int()) {
    errs.push_back("spec.replicas: Required value (integer)");
  } else if (s["replicas"].as_int() < 0) {
    errs.push_back("spec.replicas: Invalid value: " + std::to_string(s["replicas"].as_int()) +
                   ": should be greater than or equal to 0");
  }
  for (const char* f : {"resourceGroupName", "location", "vmSize", "vnetName", "subnetName", "azureCredentialSecret"})
    require_string(s, f, errs);
  const Json& img = s["imageReference"];
  if (!img.is_object()) {
    errs.push_back("spec.imageReference: Required value");
  } else {
    for (const char* f : {"publisher", "offer", "sku", "version"})
      if (!img[f].is_string()) errs.push_back(std::string("spec.imageReference.") + f + ": Required value");
  }
  return errs;
}

Mi355xJobSpec Mi355xJobSpec::from(const Json& s) {
  Mi355xJobSpec j;
  j.replicas = static_cast<int32_t>(s["replicas"].as_int(1));
  j.min_available = static_cast<int32_t>(s["minAvailable"].as_int(0));
  j.gpus_per_replica = static_cast<int32_t>(s["gpusPerReplica"].as_int(1));
  j.resource_name = s["resourceName"].as_string();
  j.pool_ref = s["poolRef"].as_string();
  for (const auto& kv : s["nodeSelector"].members()) j.node_selector[kv.first] = kv.second.as_string();
  j.queue = s["queue"].str_or("default");
  j.priority = static_cast<int32_t>(s["priority"].as_int(0));
  j.preemption_policy = s["preemptionPolicy"].str_or("Never");
  j.suspend = s["suspend"].as_bool(false);
  j.restart_policy = s["restartPolicy"].str_or("OnFailure");
  j.backoff_limit = static_cast<int32_t>(s["backoffLimit"].as_int(3));
  j.active_deadline_seconds = s["activeDeadlineSeconds"].as_int(0);
  j.ttl_seconds_after_finished = s["ttlSecondsAfterFinished"].as_int(-1);
  j.clean_pod_policy = s["cleanPodPolicy"].str_or("Running");
  j.success_policy = s["successPolicy"].str_or("AllWorkers");
  j.master_port = static_cast<int32_t>(s["masterPort"].as_int(29500));
  j.checkpoint_dir = s["checkpointDir"].as_string();
  j.tmpl = s["template"].is_object() ? s["template"] : Json::object();
  return j;
}

std::vector<std::string> validate_job(const Json& obj) {
  std::vector<std::string> errs;
  const Json& s = obj["spec"];
  if (!s.is_object()) return {"spec: Required value"};
  auto int_range = [&](const char* k, int64_t lo, int64_t hi, bool required) {
    if (!s.contains(k)) {
      if (required) errs.push_back(std::string("spec.") + k + ": Required value (integer)");
      return;
    }
    if (!s[k].is_int()) {
      errs.push_back(std::string("spec.") + k + ": must be of type integer");
      return;
    }
    int64_t v = s[k].as_int();
    if (v < lo || v > hi)
      errs.push_back(std::string("spec.") + k + ": Invalid value: " + std::to_string(v) + ": must be within [" +
                     std::to_string(lo) + ", " + std::to_string(hi) + "]");
  };
  int_range("replicas", 1, 1024, true);
  int_range("gpusPerReplica", 0, 64, false);
  int_range("minAvailable", 1, 1024, false);
  int_range("backoffLimit", 0, INT32_MAX, false);
  int_range("activeDeadlineSeconds", 0, INT64_MAX, false);
  int_range("ttlSecondsAfterFinished", -1, INT64_MAX, false);
  int_range("masterPort", 1, 65535, false);
  if (s["minAvailable"].is_int() && s["replicas"].is_int() &&
      s["minAvailable"].as_int() > s["replicas"].as_int())
    errs.push_back("spec: minAvailable must not exceed replicas");
  if (s.contains("resourceName")) {
    static const std::regex re("^[a-z0-9.-]+/[a-z0-9.-]+$");
    if (!s["resourceName"].is_string() || !std::regex_match(s["resourceName"].as_string(), re))
      errs.push_back("spec.resourceName: Invalid value: should match '^[a-z0-9.-]+/[a-z0-9.-]+$'");
  }
  if (s.contains("restartPolicy") && !in(s["restartPolicy"].as_string(), {"OnFailure", "Never"}))
    errs.push_back("spec.restartPolicy: Unsupported value");
  if (s.contains("cleanPodPolicy") && !in(s["cleanPodPolicy"].as_string(), {"Running", "All", "None"}))
    errs.push_back("spec.cleanPodPolicy: Unsupported value");
  if (s.contains("preemptionPolicy") && !in(s["preemptionPolicy"].as_string(), {"Never", "PreemptLowerPriority"}))
    errs.push_back("spec.preemptionPolicy: Unsupported value");
  if (s.contains("suspend") && !s["suspend"].is_bool()) errs.push_back("spec.suspend: must be of type boolean");
  if (s.contains("successPolicy") && !in(s["successPolicy"].as_string(), {"AllWorkers", "Rank0"}))
    errs.push_back("spec.successPolicy: Unsupported value");
  if (!s["template"].is_object()) errs.push_back("spec.template: Required value");
  return errs;
}

std::vector<std::string> validate_mi355x(const Json& obj) {
  std::vector<std::string> errs;
  const Json& s = obj["spec"];
  if (!s.is_object()) return {"spec: Required value"};
  if (!s["replicas"].is_int()) {
    errs.push_back("spec.replicas: Required value (integer)");
  } else {
    int64_t r = s["replicas"].as_int();
    if (r < 0) errs.push_back("spec.replicas: Invalid value: " + std::to_string(r) + ": should be greater than or equal to 0");
    if (r > 1024) errs.push_back("spec.replicas: Invalid value: " + std::to_string(r) + ": should be less than or equal to 1024");
  }
  if (s.contains("resourceName")) {
    static const std::regex re("^[a-z0-9.-]+/[a-z0-9.-]+$");
    if (!s["resourceName"].is_string() || !std::regex_match(s["resourceName"].as_string(), re))
      errs.push_back("spec.resourceName: Invalid value: should match '^[a-z0-9.-]+/[a-z0-9.-]+$'");
  }
  if (s.contains("topologyPolicy") && !in(s["topologyPolicy"].as_string(), {"xgmi-packed", "any"}))
    errs.push_back("spec.topologyPolicy: Unsupported value");
  if (s.contains("replacePolicy") && !in(s["replacePolicy"].as_string(), {"Replace", "Keep"}))
    errs.push_back("spec.replacePolicy: Unsupported value");
  if (s.contains("maxNodes")) {
    int64_t v = s["maxNodes"].as_int(0);
    if (!s["maxNodes"].is_int() || v < 1 || v > 64) errs.push_back("spec.maxNodes: must be within [1, 64]");
  }
  if (s.path("sharing").contains("overBudgetAction") &&
      !in(s.path("sharing.overBudgetAction").as_string(), {"Flag", "Evict"}))
    errs.push_back("spec.sharing.overBudgetAction: Unsupported value");
  if (s.path("sharing").contains("replicasPerGPU")) {
    const Json& r = s.path("sharing.replicasPerGPU");
    if (!r.is_int() || r.as_int(0) < 1 || r.as_int(0) > 64)
      errs.push_back("spec.sharing.replicasPerGPU: must be within [1, 64]");
  }
  {
    // disjoint CU shares: the slots of one GPU must fit its 256 CUs (MI355X, SPX)
    const int64_t k = s.path("sharing.replicasPerGPU").as_int(1), cu = s.path("sharing.cuPerSlot").as_int(0);
    if (cu < 0 || cu > 256) errs.push_back("spec.sharing.cuPerSlot: must be within [0, 256]");
    else if (cu > 0 && cu * k > 256)
      errs.push_back("spec.sharing.cuPerSlot: cuPerSlot x replicasPerGPU must not exceed the GPU's 256 CUs");
    else if (cu > 0) {
      // a queue's workgroups are dealt to every XCD of the (partition of the) GPU, and a CU mask
      // that leaves an XCD empty is not applied at all (profiles/r4b_cu_mask_layouts.json): a
      // slot needs at least one CU per XCD — 8 on SPX (the "Any" default may land there)
      const std::string part = s.path("partition.compute").str_or("Any");
      const int64_t xcds = part == "CPX" ? 1 : part == "QPX" ? 2 : part == "DPX" ? 4 : 8;
      if (cu < xcds)
        errs.push_back("spec.sharing.cuPerSlot: must be at least " + std::to_string(xcds) +
                       " (one CU per XCD of a " + (part == "Any" ? std::string("SPX") : part) +
                       " GPU), or 0");
    }
    if (s.path("sharing.hbmBytesPerSlot").as_int(0) < 0)
      errs.push_back("spec.sharing.hbmBytesPerSlot: should be greater than or equal to 0");
  }
  const Json& h = s["health"];
  if (h.contains("thermal") && !in(h["thermal"].as_string(), {"belowCritical", "belowEmergency", "ignore"}))
    errs.push_back("spec.health.thermal: Unsupported value");
  if (h.contains("maxUncorrectableECC") && h["maxUncorrectableECC"].as_int(0) < 0)
    errs.push_back("spec.health.maxUncorrectableECC: should be greater than or equal to 0");
  if (h.contains("minXGMILinksUp")) {
    int64_t v = h["minXGMILinksUp"].as_int(0);
    if (v < 0 || v > 8) errs.push_back("spec.health.minXGMILinksUp: must be within [0, 8]");
  }
  const Json& pr = s["probe"];
  if (pr.contains("hbmBytes")) {
    int64_t b = pr["hbmBytes"].as_int(0);
    if (b < (1LL << 20) || b > (64LL << 30)) errs.push_back("spec.probe.hbmBytes: must be within [1MiB, 64GiB]");
  }
  if (pr.contains("recheckSeconds") && (!pr["recheckSeconds"].is_int() || pr["recheckSeconds"].as_int(0) < 0))
    errs.push_back("spec.probe.recheckSeconds: should be greater than or equal to 0");
  if (pr.contains("xgmiPeerCheck") && !pr["xgmiPeerCheck"].is_bool())
    errs.push_back("spec.probe.xgmiPeerCheck: must be of type boolean");
  if (pr.contains("timeoutSeconds") &&
      (!pr["timeoutSeconds"].is_number() || pr["timeoutSeconds"].as_double(0) < 0.1 ||
       pr["timeoutSeconds"].as_double(0) > 600))
    errs.push_back("spec.probe.timeoutSeconds: must be within [0.1, 600]");
  for (const char* k : {"minHbmGBps", "minMfmaTflops", "minXgmiGBps"})
    if (pr.contains(k) && (!pr[k].is_number() || pr[k].as_double(0) < 0))
      errs.push_back(std::string("spec.probe.") + k + ": should be greater than or equal to 0");
  const Json& part = s["partition"];
  if (part.contains("compute") && !in(part["compute"].as_string(), {"Any", "SPX", "DPX", "QPX", "CPX"}))
    errs.push_back("spec.partition.compute: Unsupported value");
  if (part.contains("memory") && !in(part["memory"].as_string(), {"Any", "NPS1", "NPS2", "NPS4", "NPS8"}))
    errs.push_back("spec.partition.memory: Unsupported value");
  const Json& as = s["autoscale"];
  if (as.contains("enabled") && !as["enabled"].is_bool()) errs.push_back("spec.autoscale.enabled: must be of type boolean");
  for (const char* k : {"minReplicas", "maxReplicas"})
    if (as.contains(k) && (!as[k].is_int() || as[k].as_int(0) < 0 || as[k].as_int(0) > 1024))
      errs.push_back(std::string("spec.autoscale.") + k + ": must be within [0, 1024]");
  if (as.contains("scaleDownDelaySeconds") &&
      (!as["scaleDownDelaySeconds"].is_int() || as["scaleDownDelaySeconds"].as_int(0) < 0))
    errs.push_back("spec.autoscale.scaleDownDelaySeconds: should be greater than or equal to 0");
  // the CRD's x-kubernetes-validations rules, for objects written before the rules existed
  if (as["minReplicas"].is_int() && as["maxReplicas"].is_int() &&
      as["minReplicas"].as_int() > as["maxReplicas"].as_int())
    errs.push_back("spec.autoscale: minReplicas must not exceed maxReplicas");
  return errs;
}

const Json& find_condition(const Json& conditions, const std::string& type) {
  for (const auto& c : conditions.elements())
    if (c["type"].as_string() == type) return c;
  return Json::null_ref();
}

bool condition_true(const Json& conditions, const std::string& type) {
  return find_condition(conditions, type)["status"].as_string() == "True";
}

bool set_condition(Json& conditions, const std::string& type, const std::string& status,
                   const std::string& reason, const std::string& message, int64_t generation,
                   const std::string& now) {
  if (!conditions.is_array()) conditions = Json::array();
  for (auto& c : conditions.elements()) {
    if (c["type"].as_string() != type) continue;
    bool changed = false;
    if (c["status"].as_string() != status) {
      c["status"] = status;
      c["lastTransitionTime"] = now;
      changed = true;
    }
    if (c["reason"].as_string() != reason) {
      c["reason"] = reason;
      changed = true;
    }
    if (c["message"].as_string() != message) {
      c["message"] = message;
      changed = true;
    }
    if (c["observedGeneration"].as_int(-1) != generation) {
      c["observedGeneration"] = generation;
      changed = true;
    }
    return changed;
  }
  Json c = Json::object();
  c["type"] = type;
  c["status"] = status;
  c["observedGeneration"] = generation;
  c["lastTransitionTime"] = now;
  c["reason"] = reason;
  c["message"] = message;
  conditions.push_back(c);
  return true;
}

}  // namespace gpupool

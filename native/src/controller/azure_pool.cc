// AzureVmPool: the reference's operator (README.md:84-235) against a CloudProvider
// (fake cloud or Azure Resource Manager), credentials from a Secret or Workload Identity.
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

// ================================================================== AzureVmPool
AzureVmPoolReconciler::AzureVmPoolReconciler(KubeClient& client, Informer& pools, CloudProvider& cloud,
                                             EventRecorder* events, ReconcilerOptions opts)
    : PoolReconcilerBase(client, pools, events, opts, "AzureVmPool", res::azurevmpools()), cloud_(cloud) {}

static const char* const kWorkloadIdentity = "workload-identity";

bool AzureVmPoolReconciler::credentials_(const ObjectMeta& m, const AzureVmPoolSpec& spec, Credentials* out,
                                         std::string* why) {
  // Workload Identity (README.md:311, the reference's production recommendation): with
  // spec.azureCredentialSecret == "workload-identity" the manager uses ITS OWN federated identity:
  // AZURE_CLIENT_ID / AZURE_TENANT_ID / AZURE_SUBSCRIPTION_ID and the projected ServiceAccount
  // token at AZURE_FEDERATED_TOKEN_FILE (what the AKS webhook injects) - no static secret.
  if (spec.credential_secret == kWorkloadIdentity) {
    std::vector<std::string> missing;
    for (const char* k : {"AZURE_CLIENT_ID", "AZURE_TENANT_ID", "AZURE_SUBSCRIPTION_ID", "AZURE_FEDERATED_TOKEN_FILE"}) {
      const char* v = getenv(k);
      if (!v || !*v) missing.push_back(k);
      else out->values[k] = v;
    }
    if (!missing.empty()) {
      *why = "workload identity: manager environment lacks " + join(missing, ",");
      return false;
    }
    std::ifstream tf(out->values["AZURE_FEDERATED_TOKEN_FILE"]);
    std::string token((std::istreambuf_iterator<char>(tf)), std::istreambuf_iterator<char>());
    if (token.find_first_not_of(" \r\n\t") == std::string::npos) {
      *why = "workload identity: federated token file " + out->values["AZURE_FEDERATED_TOKEN_FILE"] + " is empty or unreadable";
      return false;
    }
    out->values["AZURE_CLIENT_SECRET"] = "";  // a client assertion (the token) replaces the secret
    out->values["AZURE_FEDERATED_TOKEN"] = token;
    return true;
  }
  // README.md:179-185: the client is built from the Secret named by spec.azureCredentialSecret.
  Json secret;
  try {
    secret = client_.get(res::secrets(), m.ns, spec.credential_secret);
  } catch (const KubeError& e) {
    if (e.not_found()) {
      *why = "Secret " + m.ns + "/" + spec.credential_secret + " not found";
      return false;
    }
    throw;
  }
  std::vector<std::string> missing;
  for (const char* k : gen::kAzureCredentialKeys) {
    std::string v = base64_decode(secret["data"][k].as_string());
    if (v.empty()) missing.push_back(k);
    else out->values[k] = v;
  }
  if (!missing.empty()) {
    *why = "Secret " + m.ns + "/" + spec.credential_secret + " lacks keys: " + join(missing, ",");
    return false;
  }
  // optional: the SSH key the VMs' admin account trusts (else the manager's --azure-ssh-public-key-file)
  std::string ssh = base64_decode(secret["data"]["AZURE_SSH_PUBLIC_KEY"].as_string());
  if (!ssh.empty()) out->values["AZURE_SSH_PUBLIC_KEY"] = ssh;
  return true;
}

Outcome AzureVmPoolReconciler::reconcile(const std::string& ns, const std::string& name) {
  auto cached = pools_.get(ns, name);
  if (!cached) return Outcome::done(ms(0));
  Json obj = *cached;
  ObjectMeta m = ObjectMeta::from(obj);
  const std::string now = rfc3339_now();
  Json conds = obj.path("status.conditions").is_array() ? obj.path("status.conditions") : Json::array();
  Json st = Json::object();
  st["observedGeneration"] = m.generation;
  // What the last successful list observed. A pass that cannot observe (invalid spec, missing or
  // refused credentials, an ARM 429/5xx) keeps it: the VMs still exist whether or not this pass
  // could list them (the reference returns without touching status on a list error,
  // README.md:189-193; replacing the whole status with only the error wiped readyReplicas and vms).
  auto keep_observed = [&]() {
    for (const char* k : {"readyReplicas", "replicas", "vms"})
      if (!obj.path("status")[k].is_null()) st[k] = obj.path("status")[k];
  };
  auto errs = validate_azure(obj);
  if (!errs.empty()) {
    set_condition(conds, gen::kCondReady, "False", "InvalidSpec", join(errs, "; "), m.generation, now);
    keep_observed();
    st["conditions"] = conds;
    write_status_(obj, st);
    return Outcome::terminal("invalid spec");
  }
  AzureVmPoolSpec spec = AzureVmPoolSpec::from(obj["spec"]);
  note_generation_(m);
  // README.md:238 tags every resource with its owner. "<ns>-<name>" (the reference's form) is
  // ambiguous — pools a-b/c and a/b-c would share it and could list and delete each other's VMs
  // — so the owner is "<ns>/<name>" ('/' occurs in neither part).
  const std::string owner = m.ns + "/" + m.name;
  // Deterministic VM names "<name>-<uid8>-<slot>": a create whose reply was lost is retried under
  // the same name, so ARM's create-or-update PUT makes the retry idempotent (README.md:240) instead
  // of creating a second VM; the uid part keeps a recreated pool of the same name distinct.
  std::string uid8;
  for (char ch : m.uid)
    if (ch != '-' && uid8.size() < 8) uid8.push_back(ch);
  const std::string vm_prefix = m.name + "-" + uid8 + "-";
  Credentials creds;
  std::string why;
  bool have_creds = credentials_(m, spec, &creds, &why);
  if (!have_creds) {
    set_condition(conds, gen::kCondCredentialsValid, "False", "CredentialsMissing", why, m.generation, now);
    set_condition(conds, gen::kCondReady, "False", "CredentialsMissing", why, m.generation, now);
    set_condition(conds, gen::kCondDegraded, "True", "CredentialsMissing", why, m.generation, now);
    set_condition(conds, gen::kCondDeleting, m.deleting() ? "True" : "False", m.deleting() ? "Finalizing" : "NotDeleting", "",
                  m.generation, now);
    st["readyReplicas"] = obj.path("status.readyReplicas").as_int(0);
    st["replicas"] = obj.path("status.replicas").as_int(0);
    keep_observed();
    st["conditions"] = conds;
    write_status_(obj, st);
    event_(obj, "Warning", "CredentialsMissing", why);
    // README.md:184 intended a 30 s requeue; typed outcome makes that delay real.
    return Outcome::requeue(opts_.credentials_retry, why);
  }
  if (spec.credential_secret == kWorkloadIdentity)
    set_condition(conds, gen::kCondCredentialsValid, "True", "WorkloadIdentity",
                  "federated token for client " + creds.values["AZURE_CLIENT_ID"], m.generation, now);
  else
    set_condition(conds, gen::kCondCredentialsValid, "True", "SecretResolved",
                  "Secret " + m.ns + "/" + spec.credential_secret + " has all four keys", m.generation, now);

  std::vector<VmRecord> vms;
  try {
    vms = cloud_.list(creds, spec.resource_group, owner);
  } catch (const ProviderError& e) {
    const bool refused = e.code == "AuthenticationFailed" || e.code == "AuthorizationFailed";
    if (refused) {  // the cloud refused the credentials: retried like missing ones (Secret may be fixed)
      set_condition(conds, gen::kCondCredentialsValid, "False", e.code, e.what(), m.generation, now);
      set_condition(conds, gen::kCondReady, "False", e.code, e.what(), m.generation, now);
    }
    set_condition(conds, gen::kCondDegraded, "True", e.code, e.what(), m.generation, now);
    keep_observed();
    st["conditions"] = conds;
    write_status_(obj, st);
    if (refused) {
      event_(obj, "Warning", e.code, e.what());
      return Outcome::requeue(opts_.credentials_retry, e.what());
    }
    return e.transient ? Outcome::transient(e.what()) : Outcome::terminal(e.what());
  }

  if (m.deleting()) {
    std::vector<std::string> orphans;
    try {
      for (const auto& vm : vms)
        if (vm.state != "Deleting") cloud_.destroy(creds, spec.resource_group, vm.name);
      vms = cloud_.list(creds, spec.resource_group, owner);
      // NICs / OS disks left by an interrupted create: removed once their VMs are gone
      orphans = cloud_.orphans(creds, spec.resource_group, owner, vm_prefix);
      if (vms.empty())
        for (const auto& o : orphans) cloud_.destroy(creds, spec.resource_group, o);
    } catch (const ProviderError& e) {
      set_condition(conds, gen::kCondDegraded, "True", e.code, e.what(), m.generation, now);
      keep_observed();
      st["conditions"] = conds;
      write_status_(obj, st);
      return Outcome::transient(e.what());
    }
    if (!vms.empty() || !orphans.empty()) {
      set_condition(conds, gen::kCondDeleting, "True", "DeletingVMs",
                    std::to_string(vms.size()) + " VM(s), " + std::to_string(orphans.size()) +
                        " leftover NIC/disk(s) still deleting",
                    m.generation, now);
      set_condition(conds, gen::kCondReady, "False", "Deleting", "pool is being deleted", m.generation, now);
      st["conditions"] = conds;
      st["replicas"] = static_cast<long long>(vms.size());
      st["readyReplicas"] = 0;
      write_status_(obj, st);
      return Outcome::requeue(opts_.progress_poll, "deleting VMs");
    }
    if (m.has_finalizer(gen::kFinalizer)) remove_finalizer_(obj);
    event_(obj, "Normal", "Finalized", "all VMs, NICs and OS disks deleted; finalizer removed");
    forget_(m.uid);
    return Outcome::done(ms(0));
  }
  if (!m.has_finalizer(gen::kFinalizer)) {
    obj = ensure_finalizer_(obj);
    m = ObjectMeta::from(obj);
  }

  std::vector<VmRecord> live;
  for (const auto& vm : vms)
    if (vm.state != "Deleting") live.push_back(vm);
  std::string progress_reason, progress_msg, error_reason, error_msg;
  int64_t desired = spec.replicas;
  auto cur = static_cast<int64_t>(live.size());
  try {
    // replace failed VMs
    for (const auto& vm : live) {
      if (vm.state == "Failed") {
        cloud_.destroy(creds, spec.resource_group, vm.name);
        event_(obj, "Warning", "VMFailed", "VM " + vm.name + " failed provisioning: deleting");
        --cur;
      }
    }
    if (cur < desired) {
      progress_reason = "ScalingUp";
      std::set<std::string> taken;  // every listed VM name, Deleting ones included
      for (const auto& vm : vms) taken.insert(vm.name);
      int64_t slot = 0;
      for (int64_t i = cur; i < desired; ++i) {
        std::string vname;
        do vname = vm_prefix + std::to_string(slot++);  // README.md:204-205 unique name
        while (taken.count(vname));
        taken.insert(vname);
        cloud_.create(creds, spec, owner, vname);
        event_(obj, "Normal", "VMCreating", "creating VM " + vname + " (" + spec.vm_size + ")");
      }
      progress_msg = "creating " + std::to_string(desired - cur) + " VM(s)";
    } else if (cur > desired) {
      std::vector<VmRecord> order;
      for (const auto& vm : live)
        if (vm.state != "Failed") order.push_back(vm);
      std::sort(order.begin(), order.end(), [](const VmRecord& a, const VmRecord& b) {
        bool ca = a.state == "Creating", cb = b.state == "Creating";
        if (ca != cb) return ca;
        if (a.created_at != b.created_at) return a.created_at > b.created_at;
        return a.name > b.name;
      });
      int64_t drop = cur - desired;
      for (int64_t i = 0; i < drop && i < static_cast<int64_t>(order.size()); ++i) {
        cloud_.destroy(creds, spec.resource_group, order[static_cast<size_t>(i)].name);
        event_(obj, "Normal", "VMDeleting", "deleting VM " + order[static_cast<size_t>(i)].name + " with its NIC and OS disk");
      }
      progress_reason = "ScalingDown";
      progress_msg = "deleting " + std::to_string(drop) + " VM(s)";
    }
  } catch (const ProviderError& e) {
    error_reason = e.code;
    error_msg = e.what();
    event_(obj, "Warning", e.code, e.what());
  }
  // Re-observe after acting (fixes README.md:225 which reported the pre-action count).
  try {
    vms = cloud_.list(creds, spec.resource_group, owner);
  } catch (const ProviderError& e) {  // acted, but cannot see the result: keep the last observation
    set_condition(conds, gen::kCondDegraded, "True", e.code, e.what(), m.generation, now);
    keep_observed();
    st["conditions"] = conds;
    write_status_(obj, st);
    return Outcome::transient(e.what());
  }
  int64_t ready = 0, total = 0;
  bool inflight = false;
  Json names = Json::array();
  std::vector<std::string> sorted;
  for (const auto& vm : vms) {
    if (vm.state == "Deleting") {
      inflight = true;
      continue;
    }
    ++total;
    if (vm.state == "Succeeded") ++ready;
    else inflight = true;
    sorted.push_back(vm.name);
  }
  std::sort(sorted.begin(), sorted.end());
  for (const auto& n : sorted) names.push_back(n);
  st["replicas"] = total;
  st["readyReplicas"] = ready;
  st["vms"] = names;
  bool is_ready = ready == desired && total == desired;
  if (!error_reason.empty()) {
    set_condition(conds, gen::kCondDegraded, "True", error_reason, error_msg, m.generation, now);
  } else {
    set_condition(conds, gen::kCondDegraded, "False", "AsExpected", "", m.generation, now);
  }
  if (inflight || !progress_reason.empty()) {
    set_condition(conds, gen::kCondProgressing, "True", progress_reason.empty() ? "Provisioning" : progress_reason,
                  progress_msg.empty() ? "cloud operations in flight" : progress_msg, m.generation, now);
  } else {
    set_condition(conds, gen::kCondProgressing, "False", "Stable",
                  std::to_string(ready) + "/" + std::to_string(desired) + " VMs ready", m.generation, now);
  }
  set_condition(conds, gen::kCondDeleting, "False", "NotDeleting", "", m.generation, now);
  set_condition(conds, gen::kCondReady, is_ready ? "True" : "False",
                is_ready ? "AllReplicasReady" : (!error_reason.empty() ? error_reason : "Provisioning"),
                std::to_string(ready) + "/" + std::to_string(desired) + " VMs ready", m.generation, now);
  st["conditions"] = conds;
  write_status_(obj, st);
  ready_gauge().set({{"kind", kind_}, {"pool", m.key()}}, static_cast<double>(ready));
  observe_ready_(m, is_ready, desired);
  if (!error_reason.empty()) return Outcome::transient(error_msg);
  if (inflight || !is_ready) return Outcome::requeue(opts_.progress_poll, "cloud operations in flight");
  return Outcome::done(opts_.resync);
}

}  // namespace gpupool

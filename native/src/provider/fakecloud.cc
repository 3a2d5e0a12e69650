// FakeCloudProvider: the "no cloud" backend for AzureVmPool (BASELINE config 1). Models the parts
// of Azure the reference relies on: tag-scoped VM listing (README.md:187-189, :238), asynchronous
// create of VM + NIC + OS disk with a unique name (README.md:204-205), delete that also removes
// NIC and OS disk (README.md:216-217, :239), idempotency (README.md:240), credential checks
// (README.md:107-109), and transient failures/quotas for error-path tests.
#include <fstream>
#include <sstream>

#include "gpupool/generated/schema_consts.h"
#include "gpupool/log.h"
#include "gpupool/provider.h"

namespace gpupool {

Json VmRecord::to_json() const {
  Json j = Json::object();
  j["name"] = name;
  j["id"] = id;
  j["state"] = state;
  j["resourceGroup"] = resource_group;
  j["location"] = location;
  j["vmSize"] = vm_size;
  j["nic"] = nic;
  j["osDisk"] = os_disk;
  j["createdAt"] = created_at;
  for (const auto& kv : tags) j["tags"][kv.first] = kv.second;
  return j;
}

FakeCloudProvider::FakeCloudProvider(FakeCloudOptions opts) : opts_(std::move(opts)) { load_(); }

void FakeCloudProvider::check_creds_(const Credentials& c) {
  // ARM accepts either a client secret or a federated client assertion (workload identity)
  auto fed = c.values.find("AZURE_FEDERATED_TOKEN");
  const bool federated = fed != c.values.end() && !fed->second.empty();
  for (const char* k : gen::kAzureCredentialKeys) {
    if (federated && std::string(k) == "AZURE_CLIENT_SECRET") continue;
    auto it = c.values.find(k);
    if (it == c.values.end() || it->second.empty())
      throw ProviderError("CredentialsMissing", std::string("credential key ") + k + " missing", false);
  }
}

bool FakeCloudProvider::take_fault_(const char* key) {
  if (opts_.faults_file.empty()) return false;
  std::ifstream f(opts_.faults_file);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  auto j = Json::try_parse(ss.str());
  if (!j || (*j)[key].as_int(0) <= 0) return false;
  (*j)[key] = (*j)[key].as_int(0) - 1;
  std::ofstream o(opts_.faults_file);
  o << j->dump();
  return true;
}

void FakeCloudProvider::advance_locked_() {
  auto now = std::chrono::steady_clock::now();
  bool changed = false;
  for (auto it = vms_.begin(); it != vms_.end();) {
    Vm& vm = it->second;
    if (vm.deleting && now >= vm.gone_at) {
      nics_[vm.rec.resource_group].erase(vm.rec.nic);
      disks_[vm.rec.resource_group].erase(vm.rec.os_disk);
      it = vms_.erase(it);
      changed = true;
      continue;
    }
    if (!vm.deleting && vm.rec.state == "Creating" && now >= vm.ready_at) {
      vm.rec.state = "Succeeded";
      changed = true;
    }
    ++it;
  }
  if (changed) save_locked_();
}

std::vector<VmRecord> FakeCloudProvider::list(const Credentials& c, const std::string& rg, const std::string& owner) {
  check_creds_(c);
  std::lock_guard<std::mutex> g(mu_);
  advance_locked_();
  std::vector<VmRecord> out;
  for (const auto& kv : vms_) {
    const VmRecord& r = kv.second.rec;
    if (r.resource_group != rg) continue;
    auto m = r.tags.find("managed-by");
    auto o = r.tags.find("owner");
    if (m == r.tags.end() || m->second != "azurevmpool-operator") continue;
    if (o == r.tags.end() || o->second != owner) continue;
    out.push_back(r);
  }
  return out;
}

VmRecord FakeCloudProvider::create(const Credentials& c, const AzureVmPoolSpec& spec, const std::string& owner,
                                   const std::string& name) {
  check_creds_(c);
  std::lock_guard<std::mutex> g(mu_);
  advance_locked_();
  std::string key = spec.resource_group + "/" + name;
  auto it = vms_.find(key);
  if (it != vms_.end()) return it->second.rec;  // idempotent
  int in_rg = 0;
  for (const auto& kv : vms_)
    if (kv.second.rec.resource_group == spec.resource_group) ++in_rg;
  if (in_rg >= opts_.quota_per_rg)
    throw ProviderError("QuotaExceeded", "resource group " + spec.resource_group + " is at its VM quota");
  if (take_fault_("failCreates")) throw ProviderError("InternalServerError", "injected create failure");
  Vm vm;
  vm.rec.name = name;
  vm.rec.id = "/subscriptions/fake/resourceGroups/" + spec.resource_group + "/providers/Microsoft.Compute/virtualMachines/" + name;
  vm.rec.state = opts_.provision.count() > 0 ? "Creating" : "Succeeded";
  vm.rec.resource_group = spec.resource_group;
  vm.rec.location = spec.location;
  vm.rec.vm_size = spec.vm_size;
  vm.rec.nic = name + "-nic";
  vm.rec.os_disk = name + "-osdisk";
  vm.rec.created_at = rfc3339_now();
  vm.rec.tags = {{"managed-by", "azurevmpool-operator"}, {"owner", owner}};
  vm.ready_at = std::chrono::steady_clock::now() + opts_.provision;
  nics_[spec.resource_group][vm.rec.nic] = owner;
  disks_[spec.resource_group][vm.rec.os_disk] = owner;
  vms_[key] = vm;
  save_locked_();
  return vm.rec;
}

void FakeCloudProvider::destroy(const Credentials& c, const std::string& rg, const std::string& name) {
  check_creds_(c);
  std::lock_guard<std::mutex> g(mu_);
  advance_locked_();
  if (name.rfind("nic/", 0) == 0 || name.rfind("disk/", 0) == 0) {  // a leftover from orphans()
    const bool nic = name[0] == 'n';
    (nic ? nics_ : disks_)[rg].erase(name.substr(nic ? 4 : 5));
    return;
  }
  auto it = vms_.find(rg + "/" + name);
  if (it == vms_.end() || it->second.deleting) return;  // idempotent
  if (take_fault_("failDeletes")) throw ProviderError("InternalServerError", "injected delete failure");
  it->second.deleting = true;
  it->second.rec.state = "Deleting";
  it->second.gone_at = std::chrono::steady_clock::now() + opts_.deprovision;
  save_locked_();
  advance_locked_();
}

std::vector<std::string> FakeCloudProvider::orphans(const Credentials& c, const std::string& rg,
                                                    const std::string& owner, const std::string& /*vm_prefix*/) {
  check_creds_(c);
  std::lock_guard<std::mutex> g(mu_);
  advance_locked_();
  std::vector<std::string> out;
  auto owned_by_vm = [&](const std::string& res, bool nic) {
    for (const auto& kv : vms_)
      if (kv.second.rec.resource_group == rg && (nic ? kv.second.rec.nic : kv.second.rec.os_disk) == res) return true;
    return false;
  };
  for (const auto& kv : nics_[rg])
    if (kv.second == owner && !owned_by_vm(kv.first, true)) out.push_back("nic/" + kv.first);
  for (const auto& kv : disks_[rg])
    if (kv.second == owner && !owned_by_vm(kv.first, false)) out.push_back("disk/" + kv.first);
  return out;
}

Json FakeCloudProvider::dump() {
  std::lock_guard<std::mutex> g(mu_);
  advance_locked_();
  Json j = Json::object();
  Json vms = Json::array();
  for (const auto& kv : vms_) vms.push_back(kv.second.rec.to_json());
  j["vms"] = vms;
  Json nics = Json::array(), disks = Json::array();
  for (const auto& rg : nics_)
    for (const auto& kv : rg.second) nics.push_back(rg.first + "/" + kv.first);
  for (const auto& rg : disks_)
    for (const auto& kv : rg.second) disks.push_back(rg.first + "/" + kv.first);
  j["nics"] = nics;
  j["disks"] = disks;
  return j;
}

void FakeCloudProvider::save_locked_() {
  if (opts_.state_file.empty()) return;
  Json j = Json::object();
  Json vms = Json::array();
  for (const auto& kv : vms_) {
    Json v = kv.second.rec.to_json();
    v["deleting"] = kv.second.deleting;
    vms.push_back(v);
  }
  j["vms"] = vms;
  j["seq"] = static_cast<long long>(seq_);
  std::string tmp = opts_.state_file + ".tmp";
  {
    std::ofstream o(tmp);
    o << j.dump(1);
  }
  std::rename(tmp.c_str(), opts_.state_file.c_str());
}

void FakeCloudProvider::load_() {
  if (opts_.state_file.empty()) return;
  std::ifstream f(opts_.state_file);
  if (!f) return;
  std::stringstream ss;
  ss << f.rdbuf();
  auto j = Json::try_parse(ss.str());
  if (!j) return;
  auto now = std::chrono::steady_clock::now();
  for (const auto& v : (*j)["vms"].elements()) {
    Vm vm;
    vm.rec.name = v["name"].as_string();
    vm.rec.id = v["id"].as_string();
    vm.rec.state = v["state"].as_string();
    vm.rec.resource_group = v["resourceGroup"].as_string();
    vm.rec.location = v["location"].as_string();
    vm.rec.vm_size = v["vmSize"].as_string();
    vm.rec.nic = v["nic"].as_string();
    vm.rec.os_disk = v["osDisk"].as_string();
    vm.rec.created_at = v["createdAt"].as_string();
    for (const auto& kv : v["tags"].members()) vm.rec.tags[kv.first] = kv.second.as_string();
    vm.deleting = v["deleting"].as_bool(false);
    vm.ready_at = now;
    vm.gone_at = now;
    nics_[vm.rec.resource_group][vm.rec.nic] = vm.rec.tags["owner"];
    disks_[vm.rec.resource_group][vm.rec.os_disk] = vm.rec.tags["owner"];
    vms_[vm.rec.resource_group + "/" + vm.rec.name] = vm;
  }
  seq_ = static_cast<uint64_t>((*j)["seq"].as_int(0));
}

}  // namespace gpupool

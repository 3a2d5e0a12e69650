// AzureArmProvider: the reference's actual backend (README.md:179-221 — getAzureVMClient,
// listManagedVMs, createVM, deleteVM; contract README.md:238-240) against the Azure Resource
// Manager REST API instead of the Go SDK:
//
//   token   POST {authority}/{tenant}/oauth2/v2.0/token  (client_credentials: client secret, or a
//           federated client assertion = Workload Identity, README.md:59-60/311), cached per client
//           until 5 minutes before expiry, refreshed once on a 401
//   list    GET  .../resourceGroups/{rg}/providers/Microsoft.Compute/virtualMachines (nextLink
//           paging), filtered by the tags managed-by=azurevmpool-operator, owner=<ns>/<name>
//   create  PUT  .../Microsoft.Network/networkInterfaces/{vm}-nic (subnet of spec.vnetName /
//           spec.subnetName), waited for until Succeeded, then PUT .../virtualMachines/{vm} with
//           spec.vmSize, spec.imageReference, an SSH-only Linux profile, and deleteOption=Delete on
//           the NIC and the OS disk so ARM removes both with the VM (README.md:216, :239); a VM PUT
//           that fails removes the NIC it just made
//   destroy DELETE .../virtualMachines/{vm} (async, 202); "nic/<name>" / "disk/<name>" delete a
//           leftover NIC / OS disk
//   orphans unattached NICs tagged for the owner and unattached "<pool>-<uid8>-<slot>-osdisk" disks
//
// Every call is idempotent (PUT by name, DELETE 404 = done). Throttling (429) and 5xx are
// transient ProviderErrors (the reconciler backs off); other 4xx carry ARM's error code.
// Endpoints are options so sovereign clouds — and the in-repo ARM simulator the tests run over
// TLS (gpupool/cloud_sim) — work unchanged.
#include <chrono>
#include <mutex>
#include <set>
#include <thread>

#include "gpupool/azure_arm.h"

namespace gpupool {

namespace {

std::string form(const std::vector<std::pair<std::string, std::string>>& kv) {
  std::string out;
  for (const auto& p : kv) out += (out.empty() ? "" : "&") + url_encode(p.first) + "=" + url_encode(p.second);
  return out;
}

std::string value_of(const Credentials& c, const char* k) {
  auto it = c.values.find(k);
  return it == c.values.end() ? std::string() : it->second;
}

// provisioningState -> the CloudProvider state vocabulary
std::string state_of(const std::string& ps) {
  if (ps == "Succeeded") return "Succeeded";
  if (ps == "Deleting") return "Deleting";
  if (ps == "Failed" || ps == "Canceled") return "Failed";
  return "Creating";  // Creating | Updating | Migrating | (absent)
}

std::string last_segment(const std::string& id) {
  size_t s = id.rfind('/');
  return s == std::string::npos ? id : id.substr(s + 1);
}

}  // namespace

AzureArmProvider::AzureArmProvider(AzureArmOptions o) : opts_(std::move(o)) {
  while (!opts_.arm_endpoint.empty() && opts_.arm_endpoint.back() == '/') opts_.arm_endpoint.pop_back();
  while (!opts_.authority_host.empty() && opts_.authority_host.back() == '/') opts_.authority_host.pop_back();
}

std::string AzureArmProvider::token_(const Credentials& c, bool refresh) {
  const std::string tenant = value_of(c, "AZURE_TENANT_ID"), client = value_of(c, "AZURE_CLIENT_ID");
  const std::string secret = value_of(c, "AZURE_CLIENT_SECRET"), assertion = value_of(c, "AZURE_FEDERATED_TOKEN");
  if (tenant.empty() || client.empty() || (secret.empty() && assertion.empty()))
    throw ProviderError("CredentialsMissing", "Azure credentials need tenant, client id and a secret or federated token",
                        false);
  const std::string key = tenant + "/" + client;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = tokens_.find(key);
    if (!refresh && it != tokens_.end() && std::chrono::steady_clock::now() < it->second.refresh_at)
      return it->second.token;
  }
  std::vector<std::pair<std::string, std::string>> body = {
      {"grant_type", "client_credentials"}, {"client_id", client}, {"scope", opts_.scope}};
  if (!assertion.empty()) {
    body.emplace_back("client_assertion_type", "urn:ietf:params:oauth:client-assertion-type:jwt-bearer");
    body.emplace_back("client_assertion", assertion);
  } else {
    body.emplace_back("client_secret", secret);
  }
  HttpClient auth(Url::parse(opts_.authority_host), "", opts_.timeout_ms, opts_.tls);
  HttpResponse r;
  try {
    r = auth.request("POST", "/" + url_encode(tenant) + "/oauth2/v2.0/token", form(body),
                     "application/x-www-form-urlencoded");
  } catch (const std::exception& e) {
    throw ProviderError("AuthorityUnreachable", std::string("token request: ") + e.what());
  }
  auto j = Json::try_parse(r.body);
  if (r.status != 200 || !j || (*j)["access_token"].as_string().empty()) {
    std::string why = j ? (*j)["error_description"].str_or((*j)["error"].str_or(r.body)) : r.body;
    throw ProviderError("AuthenticationFailed", "token request for client " + client + ": HTTP " +
                                                    std::to_string(r.status) + ": " + why,
                        r.status >= 500);
  }
  Token t;
  t.token = (*j)["access_token"].as_string();
  const int64_t ttl = std::max<int64_t>(60, (*j)["expires_in"].as_int(3600));
  t.refresh_at = std::chrono::steady_clock::now() + std::chrono::seconds(std::max<int64_t>(30, ttl - 300));
  std::lock_guard<std::mutex> g(mu_);
  tokens_[key] = t;
  return t.token;
}

HttpResponse AzureArmProvider::call_(const Credentials& c, const std::string& method, const std::string& path,
                                     const std::string& body) {
  for (int attempt = 0; attempt < 2; ++attempt) {
    const std::string tok = token_(c, attempt > 0);
    HttpClient arm(Url::parse(opts_.arm_endpoint), tok, opts_.timeout_ms, opts_.tls);
    HttpResponse r;
    try {
      r = arm.request(method, path, body);
    } catch (const std::exception& e) {
      throw ProviderError("ARMUnreachable", method + " " + path + ": " + e.what());
    }
    ++calls_;
    if (r.status == 401 && attempt == 0) continue;  // expired / revoked token: refresh once
    if (r.status < 400 || r.status == 404) return r;
    auto j = Json::try_parse(r.body);
    std::string code = j ? (*j).path("error.code").str_or("ARMError") : "ARMError";
    std::string msg = j ? (*j).path("error.message").str_or(r.body) : r.body;
    const bool transient = r.status == 429 || r.status >= 500;
    if (r.status == 401 || r.status == 403) code = "AuthorizationFailed";
    throw ProviderError(code, method + " " + path + ": HTTP " + std::to_string(r.status) + ": " + msg, transient);
  }
  throw ProviderError("AuthenticationFailed", method + " " + path + ": token refused twice");
}

std::string AzureArmProvider::rg_path_(const Credentials& c, const std::string& rg) const {
  const std::string sub = value_of(c, "AZURE_SUBSCRIPTION_ID");
  if (sub.empty()) throw ProviderError("CredentialsMissing", "AZURE_SUBSCRIPTION_ID missing", false);
  return "/subscriptions/" + url_encode(sub) + "/resourceGroups/" + url_encode(rg);
}

std::vector<Json> AzureArmProvider::list_all_(const Credentials& c, const std::string& path) {
  std::vector<Json> out;
  std::string next = path;
  for (int page = 0; page < 1000 && !next.empty(); ++page) {
    HttpResponse r = call_(c, "GET", next);
    if (r.status == 404) break;  // resource group gone: nothing of ours left in it
    auto j = Json::try_parse(r.body);
    if (!j) throw ProviderError("ARMError", "GET " + next + ": unparsable body");
    for (auto& v : (*j)["value"].elements()) out.push_back(v);
    next.clear();
    const std::string link = (*j)["nextLink"].as_string();
    if (!link.empty()) {  // absolute URL on the same endpoint: keep its path + query
      size_t p = link.find("://");
      size_t s = p == std::string::npos ? 0 : link.find('/', p + 3);
      next = s == std::string::npos ? "" : link.substr(s);
    }
  }
  return out;
}

static bool tagged(const Json& res, const std::string& owner) {
  return res.path("tags.managed-by").as_string() == "azurevmpool-operator" && res.path("tags.owner").as_string() == owner;
}

std::vector<VmRecord> AzureArmProvider::list(const Credentials& c, const std::string& rg, const std::string& owner) {
  std::vector<VmRecord> out;
  for (const auto& v : list_all_(c, rg_path_(c, rg) + "/providers/Microsoft.Compute/virtualMachines?api-version=" +
                                        opts_.compute_api)) {
    if (!tagged(v, owner)) continue;
    VmRecord r;
    r.name = v["name"].as_string();
    r.id = v["id"].as_string();
    r.state = state_of(v.path("properties.provisioningState").as_string());
    r.resource_group = rg;
    r.location = v["location"].as_string();
    r.vm_size = v.path("properties.hardwareProfile.vmSize").as_string();
    r.os_disk = v.path("properties.storageProfile.osDisk.name").as_string();
    const Json& nics = v.path("properties.networkProfile.networkInterfaces");
    if (nics.size()) r.nic = last_segment(nics[0]["id"].as_string());
    r.created_at = v.path("properties.timeCreated").as_string();
    for (const auto& kv : v["tags"].members()) r.tags[kv.first] = kv.second.as_string();
    out.push_back(std::move(r));
  }
  return out;
}

VmRecord AzureArmProvider::create(const Credentials& c, const AzureVmPoolSpec& spec, const std::string& owner,
                                  const std::string& name) {
  const std::string rgp = rg_path_(c, spec.resource_group);
  const std::string sub_id = rgp + "/providers/Microsoft.Network/virtualNetworks/" + url_encode(spec.vnet) +
                             "/subnets/" + url_encode(spec.subnet);
  const std::string nic_name = name + "-nic", disk_name = name + "-osdisk";
  const std::string nic_path = rgp + "/providers/Microsoft.Network/networkInterfaces/" + url_encode(nic_name);
  Json tags = Json::object();
  tags["managed-by"] = "azurevmpool-operator";  // README.md:238 tag isolation
  tags["owner"] = owner;
  std::string key = value_of(c, "AZURE_SSH_PUBLIC_KEY");
  if (key.empty()) key = opts_.ssh_public_key;
  if (key.empty())
    throw ProviderError("SSHKeyMissing",
                        "no SSH public key: set AZURE_SSH_PUBLIC_KEY in the credentials Secret or "
                        "--azure-ssh-public-key-file on the manager",
                        false);

  // 1. the NIC (waited for: the VM PUT needs it to exist)
  Json nic = Json::object();
  nic["location"] = spec.location;
  nic["tags"] = tags;
  Json ipc = Json::object();
  ipc["name"] = "ipconfig1";
  ipc["properties"]["subnet"]["id"] = sub_id;
  ipc["properties"]["privateIPAllocationMethod"] = "Dynamic";
  nic["properties"]["ipConfigurations"] = Json::array();
  nic["properties"]["ipConfigurations"].push_back(ipc);
  HttpResponse r = call_(c, "PUT", nic_path + "?api-version=" + opts_.network_api, nic.dump());
  if (r.status == 404) throw ProviderError("ResourceGroupNotFound", "resource group " + spec.resource_group + " not found", false);
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(opts_.nic_wait_ms);
  std::string nic_id, ps;
  for (;;) {
    auto j = Json::try_parse(r.body);
    nic_id = j ? (*j)["id"].as_string() : "";
    ps = j ? (*j).path("properties.provisioningState").as_string() : "";
    if (ps == "Succeeded" || ps.empty()) break;
    if (ps == "Failed") throw ProviderError("NICFailed", "NIC " + nic_name + " failed provisioning");
    if (std::chrono::steady_clock::now() > deadline)
      throw ProviderError("NICProvisioning", "NIC " + nic_name + " still " + ps + " (retrying)");
    std::this_thread::sleep_for(std::chrono::milliseconds(opts_.poll_ms));
    r = call_(c, "GET", nic_path + "?api-version=" + opts_.network_api);
  }
  if (nic_id.empty()) nic_id = nic_path;

  // 2. the VM: NIC + OS disk deleted with it (deleteOption), SSH-only login
  Json vm = Json::object();
  vm["location"] = spec.location;
  vm["tags"] = tags;
  Json& p = vm["properties"];
  p["hardwareProfile"]["vmSize"] = spec.vm_size;
  Json& img = p["storageProfile"]["imageReference"];
  img["publisher"] = spec.image.publisher;
  img["offer"] = spec.image.offer;
  img["sku"] = spec.image.sku;
  img["version"] = spec.image.version.empty() ? "latest" : spec.image.version;
  Json& disk = p["storageProfile"]["osDisk"];
  disk["name"] = disk_name;
  disk["createOption"] = "FromImage";
  disk["deleteOption"] = "Delete";
  disk["managedDisk"]["storageAccountType"] = opts_.os_disk_type;
  p["osProfile"]["computerName"] = name;
  p["osProfile"]["adminUsername"] = opts_.admin_username;
  Json& lin = p["osProfile"]["linuxConfiguration"];
  lin["disablePasswordAuthentication"] = true;
  Json pk = Json::object();
  pk["path"] = "/home/" + opts_.admin_username + "/.ssh/authorized_keys";
  pk["keyData"] = key;
  lin["ssh"]["publicKeys"] = Json::array();
  lin["ssh"]["publicKeys"].push_back(pk);
  Json nref = Json::object();
  nref["id"] = nic_id;
  nref["properties"]["primary"] = true;
  nref["properties"]["deleteOption"] = "Delete";
  p["networkProfile"]["networkInterfaces"] = Json::array();
  p["networkProfile"]["networkInterfaces"].push_back(nref);
  const std::string vm_path = rgp + "/providers/Microsoft.Compute/virtualMachines/" + url_encode(name);
  HttpResponse vr;
  try {
    vr = call_(c, "PUT", vm_path + "?api-version=" + opts_.compute_api, vm.dump());
  } catch (const ProviderError&) {
    try {  // do not leave the NIC of a VM that was never created behind
      call_(c, "DELETE", nic_path + "?api-version=" + opts_.network_api);
    } catch (const ProviderError&) {
    }
    throw;
  }
  VmRecord rec;
  rec.name = name;
  rec.id = vm_path;
  rec.resource_group = spec.resource_group;
  rec.location = spec.location;
  rec.vm_size = spec.vm_size;
  rec.nic = nic_name;
  rec.os_disk = disk_name;
  rec.tags = {{"managed-by", "azurevmpool-operator"}, {"owner", owner}};
  auto vj = Json::try_parse(vr.body);
  rec.state = state_of(vj ? (*vj).path("properties.provisioningState").as_string() : "");
  rec.created_at = vj ? (*vj).path("properties.timeCreated").as_string() : "";
  return rec;
}

void AzureArmProvider::destroy(const Credentials& c, const std::string& rg, const std::string& name) {
  const std::string rgp = rg_path_(c, rg);
  std::string path;
  if (name.rfind("nic/", 0) == 0)
    path = rgp + "/providers/Microsoft.Network/networkInterfaces/" + url_encode(name.substr(4)) + "?api-version=" +
           opts_.network_api;
  else if (name.rfind("disk/", 0) == 0)
    path = rgp + "/providers/Microsoft.Compute/disks/" + url_encode(name.substr(5)) + "?api-version=" + opts_.compute_api;
  else
    path = rgp + "/providers/Microsoft.Compute/virtualMachines/" + url_encode(name) + "?api-version=" + opts_.compute_api;
  call_(c, "DELETE", path);  // 200/202/204 accepted, 404 = already gone
}

std::vector<std::string> AzureArmProvider::orphans(const Credentials& c, const std::string& rg,
                                                   const std::string& owner, const std::string& vm_prefix) {
  std::vector<std::string> out;
  const std::string rgp = rg_path_(c, rg);
  for (const auto& n : list_all_(c, rgp + "/providers/Microsoft.Network/networkInterfaces?api-version=" +
                                        opts_.network_api)) {
    if (tagged(n, owner) && n.path("properties.virtualMachine.id").as_string().empty() &&
        n.path("properties.provisioningState").as_string() != "Deleting")
      out.push_back("nic/" + n["name"].as_string());
  }
  // OS disks carry no tags of their own: exactly "<vm_prefix><slot>-osdisk" (this pool's
  // deterministic VM names; the prefix holds the pool UID, so no other pool's disk can match)
  for (const auto& d : list_all_(c, rgp + "/providers/Microsoft.Compute/disks?api-version=" + opts_.compute_api)) {
    const std::string dn = d["name"].as_string();
    if (vm_prefix.empty() || !d["managedBy"].as_string().empty()) continue;
    if (dn.size() <= vm_prefix.size() + 7 || dn.rfind(vm_prefix, 0) != 0 ||
        dn.compare(dn.size() - 7, 7, "-osdisk") != 0)
      continue;
    const std::string slot = dn.substr(vm_prefix.size(), dn.size() - vm_prefix.size() - 7);
    if (slot.find_first_not_of("0123456789") == std::string::npos) out.push_back("disk/" + dn);
  }
  return out;
}

}  // namespace gpupool

// AzureArmProvider: the AzureVmPool CloudProvider against the Azure Resource Manager REST API
// (reference README.md:179-221). See native/src/provider/azure_arm.cc.
#pragma once

#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "gpupool/provider.h"

namespace gpupool {

struct AzureArmOptions {
  std::string arm_endpoint = "https://management.azure.com";
  std::string authority_host = "https://login.microsoftonline.com";
  std::string scope = "https://management.azure.com/.default";
  std::string compute_api = "2024-07-01";
  std::string network_api = "2024-05-01";
  TlsOptions tls;                      // CA bundle for private endpoints / the test simulator
  std::string admin_username = "azureuser";
  std::string ssh_public_key;          // used when the credentials carry no AZURE_SSH_PUBLIC_KEY
  std::string os_disk_type = "Premium_LRS";
  int nic_wait_ms = 10000;             // NIC PUT -> Succeeded before the VM PUT
  int poll_ms = 200;
  int timeout_ms = 30000;
};

class AzureArmProvider : public CloudProvider {
 public:
  explicit AzureArmProvider(AzureArmOptions o);
  std::vector<VmRecord> list(const Credentials& c, const std::string& rg, const std::string& owner) override;
  VmRecord create(const Credentials& c, const AzureVmPoolSpec& spec, const std::string& owner,
                  const std::string& name) override;
  void destroy(const Credentials& c, const std::string& rg, const std::string& name) override;
  std::vector<std::string> orphans(const Credentials& c, const std::string& rg, const std::string& owner,
                                   const std::string& vm_prefix) override;
  uint64_t calls() const { return calls_.load(); }

 private:
  struct Token {
    std::string token;
    std::chrono::steady_clock::time_point refresh_at;
  };
  std::string token_(const Credentials& c, bool refresh);
  HttpResponse call_(const Credentials& c, const std::string& method, const std::string& path,
                     const std::string& body = "");
  std::string rg_path_(const Credentials& c, const std::string& rg) const;
  std::vector<Json> list_all_(const Credentials& c, const std::string& path);

  AzureArmOptions opts_;
  std::mutex mu_;
  std::map<std::string, Token> tokens_;  // tenant/client -> cached bearer token
  std::atomic<uint64_t> calls_{0};
};

}  // namespace gpupool

// Kubernetes REST client over HttpClient: typed errors, resource paths, CRUD, eviction, watch.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <string>

#include "gpupool/http.h"
#include "gpupool/json.h"

namespace gpupool {

struct ResourceRef {
  std::string group;  // "" = core
  std::string version;
  std::string plural;
  bool namespaced = true;
  std::string kind;

  std::string path(const std::string& ns = "", const std::string& name = "",
                   const std::string& sub = "") const;
  std::string api_version() const { return group.empty() ? version : group + "/" + version; }
};

namespace res {
ResourceRef pods();
ResourceRef nodes();
ResourceRef events();
ResourceRef secrets();
ResourceRef leases();
ResourceRef resourcequotas();
ResourceRef mi355xpools();
ResourceRef mi355xjobs();
ResourceRef mi355xqueues();  // cluster-scoped
ResourceRef azurevmpools();
}  // namespace res

class KubeError : public std::runtime_error {
 public:
  KubeError(int code, std::string reason, const std::string& msg)
      : std::runtime_error(msg), code(code), reason(std::move(reason)) {}
  int code;
  std::string reason;
  bool not_found() const { return code == 404; }
  bool conflict() const { return code == 409; }
  bool gone() const { return code == 410; }
};

// A resolved kubeconfig context (clientcmd semantics, the subset a controller needs).
struct KubeConfig {
  std::string server, token, token_file, ns, context;
  TlsOptions tls;
};
// Loads ``path`` ("" = first entry of $KUBECONFIG, else ~/.kube/config) and resolves ``context``
// ("" = current-context): cluster server, certificate-authority(-data),
// insecure-skip-tls-verify, user token / tokenFile, client-certificate(-data) /
// client-key(-data), context namespace. Relative file paths are resolved against the
// kubeconfig's directory. exec / auth-provider / basic-auth users are rejected with a clear
// error. Throws std::runtime_error.
KubeConfig load_kubeconfig(const std::string& path = "", const std::string& context = "");

class KubeClient {
 public:
  KubeClient(const std::string& server, const std::string& token = "", int timeout_ms = 15000,
             TlsOptions tls = {});
  // a rotating bearer (projected ServiceAccount token file): re-read every minute and after a 401
  KubeClient(const std::string& server, std::shared_ptr<TokenSource> tokens, int timeout_ms = 15000,
             TlsOptions tls = {});
  // In-cluster configuration (ServiceAccount): https://$KUBERNETES_SERVICE_HOST:PORT, token and
  // CA from /var/run/secrets/kubernetes.io/serviceaccount. Returns false if not in a pod.
  static bool in_cluster(std::string* server, std::string* token, TlsOptions* tls,
                         const std::string& sa_dir = "/var/run/secrets/kubernetes.io/serviceaccount");

  Json get(const ResourceRef& r, const std::string& ns, const std::string& name,
           const std::string& sub = "");
  Json list(const ResourceRef& r, const std::string& ns = "", const std::string& label_selector = "",
            const std::string& field_selector = "", int64_t limit = 0, const std::string& cont = "");
  Json create(const ResourceRef& r, const std::string& ns, const Json& obj);
  Json update(const ResourceRef& r, const std::string& ns, const Json& obj,
              const std::string& sub = "");
  Json patch_merge(const ResourceRef& r, const std::string& ns, const std::string& name,
                   const Json& patch, const std::string& sub = "");
  Json del(const ResourceRef& r, const std::string& ns, const std::string& name, int grace = -1);
  void evict(const std::string& ns, const std::string& name, int grace = -1);

  // One watch stream from ``rv``; ``cb(type, object)`` returns false to stop. Throws KubeError
  // (410 when ``rv`` was compacted, also for in-stream ERROR events). Returns the last RV seen.
  std::string watch(const ResourceRef& r, const std::string& ns, const std::string& rv,
                    const std::function<bool(const std::string&, const Json&)>& cb,
                    const std::atomic<bool>* stop, int timeout_seconds = 300,
                    const std::string& label_selector = "", const std::string& field_selector = "");

  const std::string& server() const { return server_; }
  const std::shared_ptr<TokenSource>& tokens() const { return tokens_; }

 private:
  Json call_(const std::string& method, const std::string& path, const std::string& body,
             const std::string& ctype = "application/json");
  std::string server_;
  std::shared_ptr<TokenSource> tokens_;  // nullptr: no bearer
  TlsOptions tls_;
  std::unique_ptr<HttpClient> http_;
};

}  // namespace gpupool

#include "gpupool/kube.h"

#include <cstdlib>
#include <fstream>
#include <sstream>

#include "gpupool/generated/schema_consts.h"

namespace gpupool {

std::string ResourceRef::path(const std::string& ns, const std::string& name,
                              const std::string& sub) const {
  std::string p = group.empty() ? "/api/" + version : "/apis/" + group + "/" + version;
  if (namespaced && !ns.empty()) p += "/namespaces/" + ns;
  p += "/" + plural;
  if (!name.empty()) p += "/" + name;
  if (!sub.empty()) p += "/" + sub;
  return p;
}

namespace res {
ResourceRef pods() { return {"", "v1", "pods", true, "Pod"}; }
ResourceRef nodes() { return {"", "v1", "nodes", false, "Node"}; }
ResourceRef events() { return {"", "v1", "events", true, "Event"}; }
ResourceRef secrets() { return {"", "v1", "secrets", true, "Secret"}; }
ResourceRef leases() { return {"coordination.k8s.io", "v1", "leases", true, "Lease"}; }
ResourceRef resourcequotas() { return {"", "v1", "resourcequotas", true, "ResourceQuota"}; }
ResourceRef mi355xpools() { return {gen::kGroup, gen::kVersion, gen::kPluralMi355xPool, true, "Mi355xPool"}; }
ResourceRef azurevmpools() { return {gen::kGroup, gen::kVersion, gen::kPluralAzureVmPool, true, "AzureVmPool"}; }
}  // namespace res

KubeClient::KubeClient(const std::string& server, const std::string& token, int timeout_ms, TlsOptions tls)
    : server_(server), token_(token), tls_(tls),
      http_(std::make_unique<HttpClient>(Url::parse(server), token, timeout_ms, std::move(tls))) {}

bool KubeClient::in_cluster(std::string* server, std::string* token, TlsOptions* tls, const std::string& sa_dir) {
  const char* host = getenv("KUBERNETES_SERVICE_HOST");
  const char* port = getenv("KUBERNETES_SERVICE_PORT");
  if (!host || !*host) return false;
  std::ifstream tf(sa_dir + "/token");
  if (!tf) return false;
  std::stringstream ss;
  ss << tf.rdbuf();
  *token = ss.str();
  while (!token->empty() && (token->back() == '\n' || token->back() == '\r')) token->pop_back();
  std::string h = host;
  if (h.find(':') != std::string::npos) h = "[" + h + "]";  // IPv6 service IP
  *server = "https://" + h + ":" + std::string(port && *port ? port : "443");
  tls->ca_file = sa_dir + "/ca.crt";
  return true;
}

static KubeError to_error(const HttpResponse& r, const std::string& what) {
  std::string reason, msg = what + ": HTTP " + std::to_string(r.status);
  if (auto j = Json::try_parse(r.body)) {
    reason = (*j)["reason"].as_string();
    if ((*j)["message"].is_string()) msg += ": " + (*j)["message"].as_string();
  } else if (!r.body.empty()) {
    msg += ": " + r.body.substr(0, 200);
  }
  return KubeError(r.status, reason, msg);
}

Json KubeClient::call_(const std::string& method, const std::string& path, const std::string& body,
                       const std::string& ctype) {
  HttpResponse r = http_->request(method, path, body, ctype);
  if (r.status >= 400) throw to_error(r, method + " " + path);
  if (r.body.empty()) return Json();
  return Json::parse(r.body);
}

Json KubeClient::get(const ResourceRef& r, const std::string& ns, const std::string& name,
                     const std::string& sub) {
  return call_("GET", r.path(ns, name, sub), "");
}

Json KubeClient::list(const ResourceRef& r, const std::string& ns, const std::string& ls,
                      const std::string& fs) {
  std::string p = r.path(ns);
  std::string q;
  if (!ls.empty()) q += "labelSelector=" + url_encode(ls);
  if (!fs.empty()) q += (q.empty() ? "" : "&") + std::string("fieldSelector=") + url_encode(fs);
  if (!q.empty()) p += "?" + q;
  return call_("GET", p, "");
}

Json KubeClient::create(const ResourceRef& r, const std::string& ns, const Json& obj) {
  return call_("POST", r.path(ns), obj.dump());
}

Json KubeClient::update(const ResourceRef& r, const std::string& ns, const Json& obj,
                        const std::string& sub) {
  return call_("PUT", r.path(ns, obj.path("metadata.name").as_string(), sub), obj.dump());
}

Json KubeClient::patch_merge(const ResourceRef& r, const std::string& ns, const std::string& name,
                             const Json& patch, const std::string& sub) {
  return call_("PATCH", r.path(ns, name, sub), patch.dump(), "application/merge-patch+json");
}

Json KubeClient::del(const ResourceRef& r, const std::string& ns, const std::string& name, int grace) {
  Json body = Json::object();
  body["kind"] = "DeleteOptions";
  body["apiVersion"] = "v1";
  if (grace >= 0) body["gracePeriodSeconds"] = grace;
  return call_("DELETE", r.path(ns, name), body.dump());
}

void KubeClient::evict(const std::string& ns, const std::string& name, int grace) {
  Json body = Json::object();
  body["apiVersion"] = "policy/v1";
  body["kind"] = "Eviction";
  body["metadata"]["name"] = name;
  body["metadata"]["namespace"] = ns;
  if (grace >= 0) body["deleteOptions"]["gracePeriodSeconds"] = grace;
  call_("POST", res::pods().path(ns, name, "eviction"), body.dump());
}

std::string KubeClient::watch(const ResourceRef& r, const std::string& ns, const std::string& rv,
                              const std::function<bool(const std::string&, const Json&)>& cb,
                              const std::atomic<bool>* stop, int timeout_seconds) {
  std::string p = r.path(ns) + "?watch=1&allowWatchBookmarks=true&timeoutSeconds=" +
                  std::to_string(timeout_seconds);
  if (!rv.empty()) p += "&resourceVersion=" + url_encode(rv);
  // A dedicated client per stream: watches are long-lived and must not hold pooled sockets.
  HttpClient stream(http_->url(), token_, 15000, tls_);
  std::string last = rv;
  std::string err_body;
  int status = stream.stream_lines(
      p,
      [&](std::string_view line) {
        auto ev = Json::try_parse(line);
        if (!ev) return true;  // skip garbage line
        const std::string& type = (*ev)["type"].as_string();
        const Json& obj = (*ev)["object"];
        if (type == "ERROR") {
          int code = static_cast<int>(obj["code"].as_int(500));
          throw KubeError(code, obj["reason"].as_string(), "watch error: " + obj["message"].as_string());
        }
        const std::string& orv = obj.path("metadata.resourceVersion").as_string();
        if (!orv.empty()) last = orv;
        if (type == "BOOKMARK") return true;
        return cb(type, obj);
      },
      stop, &err_body);
  if (status >= 400) {
    HttpResponse fake;
    fake.status = status;
    fake.body = err_body;
    throw to_error(fake, "WATCH " + p);
  }
  return last;
}

}  // namespace gpupool

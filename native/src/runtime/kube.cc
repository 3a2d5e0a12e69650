#include "gpupool/kube.h"

#include <cstdlib>
#include <fstream>
#include <sstream>

#include "gpupool/generated/schema_consts.h"
#include "gpupool/yaml.h"

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
ResourceRef mi355xjobs() { return {gen::kGroup, gen::kVersion, gen::kPluralMi355xJob, true, "Mi355xJob"}; }
ResourceRef mi355xqueues() { return {gen::kGroup, gen::kVersion, gen::kPluralMi355xQueue, false, "Mi355xQueue"}; }
ResourceRef azurevmpools() { return {gen::kGroup, gen::kVersion, gen::kPluralAzureVmPool, true, "AzureVmPool"}; }
}  // namespace res

KubeClient::KubeClient(const std::string& server, const std::string& token, int timeout_ms, TlsOptions tls)
    : KubeClient(server, token.empty() ? nullptr : TokenSource::fixed(token), timeout_ms, std::move(tls)) {}

KubeClient::KubeClient(const std::string& server, std::shared_ptr<TokenSource> tokens, int timeout_ms, TlsOptions tls)
    : server_(server), tokens_(std::move(tokens)), tls_(tls),
      http_(std::make_unique<HttpClient>(Url::parse(server), tokens_, timeout_ms, std::move(tls))) {}

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

static std::string read_file(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + p);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static const Json& named(const Json& list, const std::string& name, const char* what, const std::string& path) {
  for (const auto& e : list.elements())
    if (e["name"].as_string() == name) return e;
  throw std::runtime_error(std::string("kubeconfig ") + path + ": no " + what + " named '" + name + "'");
}

KubeConfig load_kubeconfig(const std::string& path_in, const std::string& context) {
  std::string path = path_in;
  if (path.empty()) {
    if (const char* kc = getenv("KUBECONFIG"); kc && *kc) {
      path = kc;
      path = path.substr(0, path.find(':'));  // first file of the list
    } else if (const char* home = getenv("HOME"); home && *home) {
      path = std::string(home) + "/.kube/config";
    }
  }
  if (path.empty()) throw std::runtime_error("no kubeconfig: set --kubeconfig or $KUBECONFIG");
  Json cfg;
  try {
    cfg = yaml_parse(read_file(path));
  } catch (const YamlError& e) {
    throw std::runtime_error("kubeconfig " + path + ": " + e.what());
  }
  const std::string dir = path.find('/') == std::string::npos ? "." : path.substr(0, path.rfind('/'));
  auto resolve = [&](const std::string& p) { return p.empty() || p[0] == '/' ? p : dir + "/" + p; };

  KubeConfig out;
  out.context = context.empty() ? cfg["current-context"].as_string() : context;
  if (out.context.empty()) throw std::runtime_error("kubeconfig " + path + ": no current-context");
  const Json& ctx = named(cfg["contexts"], out.context, "context", path)["context"];
  const Json& cluster = named(cfg["clusters"], ctx["cluster"].as_string(), "cluster", path)["cluster"];
  out.ns = ctx["namespace"].as_string();
  out.server = cluster["server"].as_string();
  if (out.server.empty()) throw std::runtime_error("kubeconfig " + path + ": cluster has no server");
  out.tls.insecure = cluster["insecure-skip-tls-verify"].as_bool(false);
  if (cluster["certificate-authority-data"].is_string())
    out.tls.ca_pem = base64_decode(cluster["certificate-authority-data"].as_string());
  else
    out.tls.ca_file = resolve(cluster["certificate-authority"].as_string());
  const std::string user_name = ctx["user"].as_string();
  if (!user_name.empty()) {
    const Json& user = named(cfg["users"], user_name, "user", path)["user"];
    if (user.contains("exec") || user.contains("auth-provider"))
      throw std::runtime_error("kubeconfig " + path + ": user '" + user_name +
                               "' uses an exec/auth-provider plugin; use a token or client certificate");
    if (user.contains("username") || user.contains("password"))
      throw std::runtime_error("kubeconfig " + path + ": basic auth is not supported");
    out.token = user["token"].as_string();
    if (out.token.empty() && user["tokenFile"].is_string()) {
      out.token_file = resolve(user["tokenFile"].as_string());  // re-read as it rotates
      out.token = read_file(out.token_file);
      while (!out.token.empty() && (out.token.back() == '\n' || out.token.back() == '\r')) out.token.pop_back();
    }
    if (user["client-certificate-data"].is_string())
      out.tls.cert_pem = base64_decode(user["client-certificate-data"].as_string());
    else
      out.tls.cert_file = resolve(user["client-certificate"].as_string());
    if (user["client-key-data"].is_string())
      out.tls.key_pem = base64_decode(user["client-key-data"].as_string());
    else
      out.tls.key_file = resolve(user["client-key"].as_string());
  }
  return out;
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
                      const std::string& fs, int64_t limit, const std::string& cont) {
  std::string p = r.path(ns);
  std::string q;
  if (!ls.empty()) q += "labelSelector=" + url_encode(ls);
  if (!fs.empty()) q += (q.empty() ? "" : "&") + std::string("fieldSelector=") + url_encode(fs);
  if (limit > 0) q += (q.empty() ? "" : "&") + std::string("limit=") + std::to_string(limit);
  if (!cont.empty()) q += (q.empty() ? "" : "&") + std::string("continue=") + url_encode(cont);
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
                              const std::atomic<bool>* stop, int timeout_seconds,
                              const std::string& label_selector, const std::string& field_selector) {
  std::string p = r.path(ns) + "?watch=1&allowWatchBookmarks=true&timeoutSeconds=" +
                  std::to_string(timeout_seconds);
  if (!label_selector.empty()) p += "&labelSelector=" + url_encode(label_selector);
  if (!field_selector.empty()) p += "&fieldSelector=" + url_encode(field_selector);
  if (!rv.empty()) p += "&resourceVersion=" + url_encode(rv);
  // A dedicated client per stream: watches are long-lived and must not hold pooled sockets.
  HttpClient stream(http_->url(), tokens_, 15000, tls_);
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

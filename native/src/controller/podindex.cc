#include "gpupool/podindex.h"

#include "gpupool/generated/schema_consts.h"
#include "gpupool/informer.h"
#include "job_util.h"

#include <algorithm>

namespace gpupool {

using namespace detail;

namespace {

bool extended(const std::string& name) { return name.find('/') != std::string::npos && name.rfind("kubernetes.io/", 0) != 0; }

std::map<std::string, int64_t> container_requests(const Json& c) {
  const Json& r = c["resources"];
  std::map<std::string, int64_t> mine;
  for (const auto& kv : r["requests"].members())
    if (extended(kv.first)) mine[kv.first] = qty(kv.second);
  for (const auto& kv : r["limits"].members())  // an extended resource's request is its limit
    if (extended(kv.first) && qty(kv.second)) mine[kv.first] = qty(kv.second);
  return mine;
}

// extended resource -> what the pod holds, as the scheduler counts it: the sum over its
// containers, or the largest init container's request if that is more (init containers run one
// at a time, before the others)
std::map<std::string, int64_t> extended_requests(const Json& pod) {
  std::map<std::string, int64_t> out;
  for (const auto& c : pod.path("spec.containers").elements())
    for (const auto& kv : container_requests(c)) out[kv.first] += kv.second;
  for (const auto& c : pod.path("spec.initContainers").elements())
    for (const auto& kv : container_requests(c)) out[kv.first] = std::max(out[kv.first], kv.second);
  for (auto it = out.begin(); it != out.end();) it = it->second > 0 ? std::next(it) : out.erase(it);
  return out;
}

Json trim_containers(const Json& list) {
  Json containers = Json::array();
  for (const auto& c : list.elements()) {
    Json res = Json::object();
    for (const char* part : {"limits", "requests"}) {
      Json q = Json::object();
      for (const auto& kv : c["resources"][part].members())
        if (extended(kv.first)) q[kv.first] = kv.second;
      if (q.size()) res[part] = q;
    }
    Json cc = Json::object();
    cc["name"] = c["name"];
    if (res.size()) cc["resources"] = res;
    containers.push_back(cc);
  }
  return containers;
}

}  // namespace

bool pod_relevant(const Json& pod) {
  if (!pod.path("metadata.labels")[gen::kLabelJob].as_string().empty()) return true;
  return !extended_requests(pod).empty();
}

Json trim_pod(const Json& pod) {
  Json out = Json::object();
  out["apiVersion"] = "v1";
  out["kind"] = "Pod";
  const Json& md = pod["metadata"];
  Json m = Json::object();
  for (const char* k : {"name", "namespace", "uid", "resourceVersion", "creationTimestamp", "deletionTimestamp"})
    if (!md[k].is_null()) m[k] = md[k];
  Json labels = Json::object();
  for (const char* k : {gen::kLabelJob, gen::kLabelJobIndex, gen::kLabelJobAttempt})
    if (md["labels"][k].is_string()) labels[k] = md["labels"][k];
  if (labels.size()) m["labels"] = labels;
  if (md["annotations"][gen::kAnnPodDevices].is_string()) {
    Json a = Json::object();
    a[gen::kAnnPodDevices] = md["annotations"][gen::kAnnPodDevices];
    m["annotations"] = a;
  }
  if (md["ownerReferences"].size()) {
    Json refs = Json::array();
    for (const auto& o : md["ownerReferences"].elements())
      refs.push_back(Json::object().set("uid", o["uid"]).set("kind", o["kind"]).set("name", o["name"]));
    m["ownerReferences"] = refs;
  }
  out["metadata"] = m;
  Json spec = Json::object();
  if (pod.path("spec.nodeName").is_string()) spec["nodeName"] = pod.path("spec.nodeName");
  spec["containers"] = trim_containers(pod.path("spec.containers"));
  if (pod.path("spec.initContainers").size()) spec["initContainers"] = trim_containers(pod.path("spec.initContainers"));
  out["spec"] = spec;
  const Json& st = pod["status"];
  Json s = Json::object();
  for (const char* k : {"phase", "podIP", "message"})
    if (st[k].is_string()) s[k] = st[k];
  const Json& cs = st["containerStatuses"];
  if (cs.size() > 0 && cs[0].path("state.terminated").is_object()) {
    Json t = Json::object();
    t["exitCode"] = cs[0].path("state.terminated.exitCode");
    Json state = Json::object();
    state["terminated"] = t;
    s["containerStatuses"] = Json::array({Json::object().set("state", state)});
  }
  out["status"] = s;
  return out;
}

void PodIndex::attach(Informer& pods) {
  pods.add_handler([this](const std::string& type, const Json& p) { on_event(type, p); });
  for (const auto& p : pods.list()) on_event("ADDED", p);
}

void PodIndex::remove_locked_(const std::string& key) {
  auto it = pods_.find(key);
  if (it == pods_.end()) return;
  for (const auto& kv : it->second.req) {
    auto& per_node = by_res_node_[kv.first];
    if ((per_node[it->second.node] -= kv.second) <= 0) per_node.erase(it->second.node);
  }
  if (!it->second.job_key.empty()) {
    auto j = by_job_.find(it->second.job_key);
    if (j != by_job_.end()) {
      j->second.erase(key);
      if (j->second.empty()) by_job_.erase(j);
    }
  }
  pods_.erase(it);
}

void PodIndex::on_event(const std::string& type, const Json& pod) {
  if (type == "RESYNC") return;
  const std::string ns = pod.path("metadata.namespace").as_string();
  const std::string key = ns + "/" + pod.path("metadata.name").as_string();
  std::lock_guard<std::mutex> g(mu_);
  remove_locked_(key);
  if (type == "DELETED") return;
  Entry e;
  e.node = pod.path("spec.nodeName").as_string();
  const std::string job = pod.path("metadata.labels")[gen::kLabelJob].as_string();
  if (!job.empty()) e.job_key = ns + "/" + job;
  // a terminal pod holds nothing; a deleting one still does until it is gone (its containers may
  // still be running out their grace period)
  if (!e.node.empty() && !terminal(pod_phase(pod))) e.req = extended_requests(pod);
  for (const auto& kv : e.req) by_res_node_[kv.first][e.node] += kv.second;
  if (!e.job_key.empty()) by_job_[e.job_key][key] = pod;  // the only copy kept: job pods
  pods_[key] = std::move(e);
}

std::map<std::string, int64_t> PodIndex::requested_by_node(const std::string& resource) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = by_res_node_.find(resource);
  return it == by_res_node_.end() ? std::map<std::string, int64_t>{} : it->second;
}

std::vector<Json> PodIndex::job_pods(const std::string& ns, const std::string& job) const {
  std::vector<Json> out;
  std::lock_guard<std::mutex> g(mu_);
  auto it = by_job_.find(ns + "/" + job);
  if (it == by_job_.end()) return out;
  for (const auto& kv : it->second) out.push_back(kv.second);
  return out;
}

size_t PodIndex::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return pods_.size();
}

}  // namespace gpupool

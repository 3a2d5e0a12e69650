// What the controllers need to know about a cluster's pods, without LISTing them: a projection
// for the pods informer (trim_pod / pod_relevant) and an incremental index over it (PodIndex).
//
// Volcano schedules from its caches (GPU调度平台搭建.md:275-287, 645-650); so does the gang
// scheduler here. Per node and extended resource, the requests of live pods are kept up to date by
// the informer's handler; a job's own pods are looked up by their job label.
#pragma once

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "gpupool/json.h"

namespace gpupool {

class Informer;

// Pods the manager's readers count: any that requests an extended resource ("vendor/name"), and
// any of a Mi355xJob (job label). CPU-only pods of other workloads are not cached.
bool pod_relevant(const Json& pod);
// Only the fields the readers use (identity, job labels, the devices annotation, owner uids,
// node, extended-resource requests, phase, pod IP, the first container's exit code).
Json trim_pod(const Json& pod);

class PodIndex {
 public:
  // Subscribe to ``pods`` (and seed from what it holds).
  void attach(Informer& pods);
  // resource -> node -> GPUs of that resource requested by live (non-terminal) pods on the node
  std::map<std::string, int64_t> requested_by_node(const std::string& resource) const;
  // The cached pods labelled as ``job``'s workers in ``ns``.
  std::vector<Json> job_pods(const std::string& ns, const std::string& job) const;
  size_t size() const;

  void on_event(const std::string& type, const Json& pod);  // the informer handler (tests call it)

 private:
  struct Entry {
    std::string node, job_key;
    std::map<std::string, int64_t> req;  // extended resource -> count (live pods only)
  };
  void remove_locked_(const std::string& key);
  mutable std::mutex mu_;
  std::map<std::string, Entry> pods_;                                       // "ns/name" -> entry
  std::map<std::string, std::map<std::string, int64_t>> by_res_node_;       // res -> node -> sum
  std::map<std::string, std::map<std::string, Json>> by_job_;               // "ns/job" -> key -> pod
};

}  // namespace gpupool

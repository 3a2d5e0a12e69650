// Small helpers shared by the Mi355xJob/Mi355xQueue reconcilers (job.cc) and the pool
// autoscaler (autoscale.cc): resource quantities, pod phases and what a job holds or needs.
#pragma once

#include <cstdint>
#include <cstdlib>
#include <string>

#include "gpupool/json.h"

namespace gpupool::detail {

// Extended-resource quantity ("4", 4 or 4.0) as an integer.
inline int64_t qty(const Json& v) {
  if (v.is_int()) return v.as_int();
  if (v.is_number()) return static_cast<int64_t>(v.as_double());
  const std::string& s = v.as_string();
  return s.empty() ? 0 : std::atoll(s.c_str());
}

inline bool terminal(const std::string& phase) { return phase == "Succeeded" || phase == "Failed"; }

inline std::string pod_phase(const Json& p) { return p.path("status.phase").str_or("Pending"); }

// GPUs of ``resource`` a pod asks for (limits, else requests, summed over its containers).
inline int64_t pod_request(const Json& pod, const std::string& resource) {
  int64_t n = 0;
  for (const auto& c : pod.path("spec.containers").elements()) {
    const Json& r = c["resources"];
    int64_t lim = qty(r["limits"][resource]);
    n += lim ? lim : qty(r["requests"][resource]);
  }
  return n;
}

// The extended resource a job's pods request: resolved at placement time (a poolRef's resource)
// and recorded in status.resourceName; before that, the spec's or the given default.
inline std::string job_resource(const Json& j, const std::string& dflt) {
  const std::string& st = j.path("status.resourceName").as_string();
  if (!st.empty()) return st;
  return j.path("spec.resourceName").str_or(dflt);
}

// GPUs a placed (or running) job holds: gpusPerReplica per placement slot.
inline int64_t job_held(const Json& j) {
  return j.path("spec.gpusPerReplica").as_int(1) * static_cast<int64_t>(j.path("status.placement").size());
}

inline std::string job_queue(const Json& j) { return j.path("spec.queue").str_or("default"); }

}  // namespace gpupool::detail

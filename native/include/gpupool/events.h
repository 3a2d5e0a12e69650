// Kubernetes Event recorder (reference roadmap item, README.md:311).
// Posting is asynchronous (a background thread drains a bounded queue) so a slow apiserver never
// stalls a reconcile; identical (object, type, reason, message) events within 10 minutes are
// aggregated into one Event whose ``count`` is bumped, like client-go's EventCorrelator.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>

#include "gpupool/kube.h"

namespace gpupool {

class EventRecorder {
 public:
  EventRecorder(KubeClient* client, std::string component);
  ~EventRecorder();
  // obj: the involved object (needs apiVersion/kind/metadata). type: Normal | Warning.
  void record(const Json& obj, const std::string& type, const std::string& reason,
              const std::string& message);
  void flush(std::chrono::milliseconds timeout);
  uint64_t posted() const { return posted_.load(); }
  // How long a newly queued event waits before it is posted (0 = at once).
  void set_delay(std::chrono::milliseconds d) { delay_ = d; }

 private:
  struct Pending {
    Json involved;
    std::string ns, type, reason, message;
  };
  void loop_();
  void post_(const Pending& p);

  KubeClient* client_;
  std::string component_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Pending> q_;
  bool stop_ = false;
  int inflight_ = 0;
  std::chrono::milliseconds delay_{10};
  struct Agg {
    std::string name;
    int64_t count = 0;
    std::chrono::steady_clock::time_point last;
  };
  std::map<std::string, Agg> agg_;
  std::atomic<uint64_t> posted_{0};
  std::thread th_;
};

}  // namespace gpupool

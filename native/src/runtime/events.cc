#include "gpupool/events.h"

#include <cstdio>

#include "gpupool/log.h"

namespace gpupool {

EventRecorder::EventRecorder(KubeClient* client, std::string component)
    : client_(client), component_(std::move(component)) {
  th_ = std::thread([this] { loop_(); });
}

EventRecorder::~EventRecorder() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void EventRecorder::record(const Json& obj, const std::string& type, const std::string& reason,
                           const std::string& message) {
  Pending p;
  p.involved = Json::object();
  p.involved["apiVersion"] = obj["apiVersion"];
  p.involved["kind"] = obj["kind"];
  p.involved["name"] = obj.path("metadata.name");
  p.involved["namespace"] = obj.path("metadata.namespace");
  p.involved["uid"] = obj.path("metadata.uid");
  p.involved["resourceVersion"] = obj.path("metadata.resourceVersion");
  p.ns = obj.path("metadata.namespace").str_or("default");
  p.type = type;
  p.reason = reason;
  p.message = message;
  std::lock_guard<std::mutex> g(mu_);
  if (q_.size() >= 1000) q_.pop_front();  // bounded: drop oldest under pressure
  q_.push_back(std::move(p));
  cv_.notify_one();
}

void EventRecorder::flush(std::chrono::milliseconds timeout) {
  auto deadline = std::chrono::steady_clock::now() + timeout;
  for (;;) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (q_.empty() && inflight_ == 0) return;
    }
    if (std::chrono::steady_clock::now() > deadline) return;
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
}

void EventRecorder::loop_() {
  for (;;) {
    std::deque<Pending> batch;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stop_ and drained
      if (!stop_ && delay_.count() > 0) {
        // Events are informational: let the pass that recorded the first of a burst finish its
        // status write before they reach the apiserver; the whole burst then goes out back to back
        // (one delay per burst, so a busy manager never falls behind). system_clock deadline: see
        // RocmProvider::prefetch for why not wait_for.
        auto until = std::chrono::system_clock::now() + delay_;
        cv_.wait_until(lk, until, [this] { return stop_; });
      }
      batch.swap(q_);
      inflight_ += static_cast<int>(batch.size());
    }
    for (const Pending& p : batch) {
      try {
        if (client_) post_(p);
      } catch (const std::exception& e) {
        Logger("events").warn("event post failed", Json::object().set("error", e.what()).set("reason", p.reason));
      }
      std::lock_guard<std::mutex> g(mu_);
      inflight_--;
    }
    cv_.notify_all();
  }
}

void EventRecorder::post_(const Pending& p) {
  std::string key = p.involved["uid"].as_string() + "|" + p.type + "|" + p.reason + "|" + p.message;
  auto now = std::chrono::steady_clock::now();
  std::string ts = rfc3339_now();
  auto it = agg_.find(key);
  if (it != agg_.end() && now - it->second.last < std::chrono::minutes(10)) {
    it->second.count++;
    it->second.last = now;
    Json patch = Json::object();
    patch["count"] = it->second.count;
    patch["lastTimestamp"] = ts;
    try {
      client_->patch_merge(res::events(), p.ns, it->second.name, patch);
      posted_++;
      return;
    } catch (const KubeError& e) {
      if (!e.not_found()) throw;
      agg_.erase(it);  // fall through: recreate
    }
  }
  char suffix[32];
  auto ns_since = std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::system_clock::now().time_since_epoch()).count();
  std::snprintf(suffix, sizeof suffix, "%llx", static_cast<unsigned long long>(ns_since));
  Json ev = Json::object();
  ev["apiVersion"] = "v1";
  ev["kind"] = "Event";
  ev["metadata"]["name"] = p.involved["name"].as_string() + "." + suffix;
  ev["metadata"]["namespace"] = p.ns;
  ev["involvedObject"] = p.involved;
  ev["reason"] = p.reason;
  ev["message"] = p.message;
  ev["type"] = p.type;
  ev["count"] = 1;
  ev["firstTimestamp"] = ts;
  ev["lastTimestamp"] = ts;
  ev["source"]["component"] = component_;
  ev["reportingComponent"] = component_;
  client_->create(res::events(), p.ns, ev);
  agg_[key] = Agg{ev["metadata"]["name"].as_string(), 1, now};
  posted_++;
}

}  // namespace gpupool

// Rate-limited, de-duplicating work queue with client-go semantics:
//  * a key is processed by at most one worker at a time (``processing`` set);
//  * re-adding a key while it is processing marks it dirty -> it is re-queued on ``done``;
//  * ``add_after`` delays; ``add_rate_limited`` applies per-item exponential backoff
//    (base 5 ms, x2, capped at 5 min — SURVEY.md §5 failure-detection row); ``forget`` resets it.
#pragma once

#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <queue>
#include <set>
#include <string>
#include <vector>

namespace gpupool {

class WorkQueue {
 public:
  using Clock = std::chrono::steady_clock;
  using Duration = std::chrono::milliseconds;

  explicit WorkQueue(Duration base_delay = Duration(5), Duration max_delay = Duration(300000));

  void add(const std::string& key);
  void add_after(const std::string& key, Duration d);
  void add_rate_limited(const std::string& key);
  void forget(const std::string& key);
  int num_requeues(const std::string& key) const;
  Duration backoff_for(const std::string& key) const;  // next backoff (does not mutate)

  // Blocks until a key is available or shutdown. Returns false on shutdown. ``waited_ms`` (if
  // given): how long the key sat ready in the queue before this worker took it.
  bool get(std::string* key, double* waited_ms = nullptr);
  // Like get() but gives up after ``timeout`` (returns false, key untouched).
  bool get_for(std::string* key, Duration timeout, double* waited_ms = nullptr);
  void done(const std::string& key);

  void shutdown();
  bool shutting_down() const;
  size_t len() const;          // ready queue length
  size_t delayed_len() const;  // waiting (add_after) entries

 private:
  void add_locked_(const std::string& key);
  void promote_due_locked_();

  struct Delayed {
    Clock::time_point at;
    std::string key;
    bool operator>(const Delayed& o) const { return at > o.at; }
  };

  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::string> queue_;
  std::set<std::string> dirty_;
  std::set<std::string> processing_;
  std::map<std::string, Clock::time_point> ready_at_;  // key -> when it entered queue_
  std::priority_queue<Delayed, std::vector<Delayed>, std::greater<Delayed>> delayed_;
  std::map<std::string, Clock::time_point> delayed_at_;  // earliest pending time per key
  std::map<std::string, int> failures_;
  Duration base_, max_;
  bool shutdown_ = false;
};

}  // namespace gpupool

#include "gpupool/workqueue.h"

#include <algorithm>

namespace gpupool {

WorkQueue::WorkQueue(Duration base_delay, Duration max_delay) : base_(base_delay), max_(max_delay) {}

void WorkQueue::add_locked_(const std::string& key) {
  if (shutdown_) return;
  if (dirty_.count(key)) return;
  dirty_.insert(key);
  if (processing_.count(key)) return;  // re-queued by done()
  queue_.push_back(key);
  ready_at_[key] = Clock::now();
  cv_.notify_one();
}

void WorkQueue::add(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  add_locked_(key);
}

void WorkQueue::add_after(const std::string& key, Duration d) {
  if (d.count() <= 0) {
    add(key);
    return;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (shutdown_) return;
  auto at = Clock::now() + d;
  auto it = delayed_at_.find(key);
  if (it != delayed_at_.end() && it->second <= at) return;  // an earlier wake-up already pending
  delayed_at_[key] = at;
  delayed_.push({at, key});
  cv_.notify_all();
}

WorkQueue::Duration WorkQueue::backoff_for(const std::string& key) const {
  int n = 0;
  auto it = failures_.find(key);
  if (it != failures_.end()) n = it->second;
  double ms = static_cast<double>(base_.count());
  for (int i = 0; i < n && ms < static_cast<double>(max_.count()); ++i) ms *= 2;
  return Duration(static_cast<long long>(std::min<double>(ms, static_cast<double>(max_.count()))));
}

void WorkQueue::add_rate_limited(const std::string& key) {
  Duration d;
  {
    std::lock_guard<std::mutex> g(mu_);
    d = backoff_for(key);
    failures_[key]++;
  }
  add_after(key, d);
}

void WorkQueue::forget(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  failures_.erase(key);
}

int WorkQueue::num_requeues(const std::string& key) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = failures_.find(key);
  return it == failures_.end() ? 0 : it->second;
}

void WorkQueue::promote_due_locked_() {
  auto now = Clock::now();
  while (!delayed_.empty() && delayed_.top().at <= now) {
    Delayed d = delayed_.top();
    delayed_.pop();
    auto it = delayed_at_.find(d.key);
    if (it != delayed_at_.end() && it->second == d.at) {
      delayed_at_.erase(it);
      add_locked_(d.key);
    }
  }
}

bool WorkQueue::get(std::string* key, double* waited_ms) {
  for (;;) {
    if (get_for(key, Duration(3600 * 1000), waited_ms)) return true;
    std::lock_guard<std::mutex> g(mu_);
    if (shutdown_) return false;
  }
}

bool WorkQueue::get_for(std::string* key, Duration timeout, double* waited_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  auto deadline = Clock::now() + timeout;
  for (;;) {
    promote_due_locked_();
    if (!queue_.empty()) {
      *key = queue_.front();
      queue_.pop_front();
      processing_.insert(*key);
      dirty_.erase(*key);
      auto it = ready_at_.find(*key);
      if (it != ready_at_.end()) {
        if (waited_ms) *waited_ms = std::chrono::duration<double, std::milli>(Clock::now() - it->second).count();
        ready_at_.erase(it);
      }
      return true;
    }
    if (shutdown_) return false;
    auto wake = deadline;
    if (!delayed_.empty()) wake = std::min(wake, delayed_.top().at);
    if (Clock::now() >= deadline) return false;
    // system_clock deadline -> pthread_cond_timedwait (steady_clock waits use
    // pthread_cond_clockwait, which gcc-11's TSan does not intercept: false "double lock").
    cv_.wait_until(lk, std::chrono::system_clock::now() + (wake - Clock::now()));
  }
}

void WorkQueue::done(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  processing_.erase(key);
  if (dirty_.count(key)) {
    queue_.push_back(key);
    ready_at_[key] = Clock::now();
    cv_.notify_one();
  }
}

void WorkQueue::shutdown() {
  std::lock_guard<std::mutex> g(mu_);
  shutdown_ = true;
  cv_.notify_all();
}

bool WorkQueue::shutting_down() const {
  std::lock_guard<std::mutex> g(mu_);
  return shutdown_;
}

size_t WorkQueue::len() const {
  std::lock_guard<std::mutex> g(mu_);
  return queue_.size();
}

size_t WorkQueue::delayed_len() const {
  std::lock_guard<std::mutex> g(mu_);
  return delayed_at_.size();
}

}  // namespace gpupool

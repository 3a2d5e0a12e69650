#include "gpupool/informer.h"

#include <algorithm>

namespace gpupool {

Informer::Informer(KubeClient& client, ResourceRef res, std::string ns,
                   std::chrono::milliseconds resync, InformerOptions opts)
    : client_(client), res_(std::move(res)), ns_(std::move(ns)), resync_(resync), opts_(std::move(opts)),
      log_(Logger("informer").with("resource", res_.plural)) {}

Informer::~Informer() { stop(); }

void Informer::add_handler(Handler h) {
  std::lock_guard<std::mutex> g(mu_);
  handlers_.push_back(std::move(h));
}

std::string Informer::key_of(const Json& obj) {
  const std::string& ns = obj.path("metadata.namespace").as_string();
  const std::string& name = obj.path("metadata.name").as_string();
  return ns.empty() ? name : ns + "/" + name;
}

void Informer::start() {
  stop_ = false;
  th_ = std::thread([this] { run_(); });
}

void Informer::stop() {
  stop_ = true;
  if (th_.joinable()) th_.join();
}

// The retry backoff in slices, so stop() (a SIGTERM with the apiserver unreachable) returns within
// ~50 ms instead of after a 5 s sleep per informer — the manager took 15 s to exit.
void Informer::backoff_(int ms) {
  const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(ms);
  while (!stop_ && std::chrono::steady_clock::now() < until)
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
}

bool Informer::wait_synced(std::chrono::milliseconds timeout) {
  std::unique_lock<std::mutex> lk(mu_);
  // system_clock deadline: see WorkQueue::get_for (TSan-visible pthread_cond_timedwait)
  return synced_cv_.wait_until(lk, std::chrono::system_clock::now() + timeout, [this] { return synced_.load(); });
}

std::optional<Json> Informer::get(const std::string& ns, const std::string& name) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = cache_.find(ns.empty() ? name : ns + "/" + name);
  if (it == cache_.end()) return std::nullopt;
  return it->second;
}

std::vector<Json> Informer::list() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Json> out;
  out.reserve(cache_.size());
  for (const auto& kv : cache_) out.push_back(kv.second);
  return out;
}

size_t Informer::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return cache_.size();
}

void Informer::dispatch_(const std::string& type, const Json& obj) {
  std::vector<Handler> hs;
  {
    std::lock_guard<std::mutex> g(mu_);
    hs = handlers_;
  }
  for (auto& h : hs) {
    try {
      h(type, obj);
    } catch (const std::exception& e) {
      log_.error("handler threw", Json::object().set("error", e.what()));
    }
  }
}

void Informer::list_() {
  // in pages (client-go's 500): a cluster's worth of pods is never one response held whole in
  // memory — each page is filtered and projected, then dropped
  relists_++;
  std::map<std::string, Json> fresh;
  std::string cont, list_rv;
  do {
    Json lst = client_.list(res_, ns_, opts_.label_selector, opts_.field_selector, kListPage, cont);
    if (list_rv.empty()) list_rv = lst.path("metadata.resourceVersion").as_string();
    for (const auto& item : lst["items"].elements()) {
      if (opts_.filter && !opts_.filter(item)) continue;
      fresh[key_of(item)] = opts_.transform ? opts_.transform(item) : item;
    }
    cont = lst.path("metadata.continue").as_string();
  } while (!cont.empty() && !stop_);
  std::vector<std::pair<std::string, Json>> events;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& kv : cache_)
      if (!fresh.count(kv.first)) events.emplace_back("DELETED", kv.second);
    for (const auto& kv : fresh) {
      auto it = cache_.find(kv.first);
      if (it == cache_.end()) {
        events.emplace_back("ADDED", kv.second);
      } else if (it->second.path("metadata.resourceVersion") != kv.second.path("metadata.resourceVersion")) {
        events.emplace_back("MODIFIED", kv.second);
      }
    }
    cache_ = std::move(fresh);
    rv_ = list_rv;
  }
  for (auto& e : events) dispatch_(e.first, e.second);
  if (!synced_.exchange(true)) {
    std::lock_guard<std::mutex> g(mu_);
    synced_cv_.notify_all();
  }
}

void Informer::run_() {
  using clock = std::chrono::steady_clock;
  auto next_resync = clock::now() + resync_;
  int backoff_ms = 100;
  bool need_list = true;
  // Resync ticker runs beside the watch so drift detection never waits for watch traffic.
  std::thread ticker([&] {
    while (!stop_) {
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
      if (resync_.count() > 0 && clock::now() >= next_resync) {
        next_resync = clock::now() + resync_;
        for (const auto& obj : list()) dispatch_("RESYNC", obj);
      }
    }
  });
  while (!stop_) {
    try {
      if (need_list) {
        list_();
        need_list = false;
      }
      std::string rv;
      {
        std::lock_guard<std::mutex> g(mu_);
        rv = rv_;
      }
      std::string last = client_.watch(
          res_, ns_, rv,
          [this](const std::string& type_in, const Json& raw) {
            events_++;
            std::string type = type_in;
            const bool keep = !opts_.filter || opts_.filter(raw);
            const Json obj = opts_.transform ? opts_.transform(raw) : raw;
            std::string key = key_of(obj);
            bool deliver = true;
            {
              std::lock_guard<std::mutex> g(mu_);
              rv_ = raw.path("metadata.resourceVersion").as_string();
              if (!keep && type != "DELETED") {  // left the filter (or never in it)
                deliver = cache_.erase(key) > 0;
                type = "DELETED";
              } else if (type == "DELETED") {
                deliver = cache_.erase(key) > 0 || keep;
              } else {
                if (!cache_.count(key)) type = "ADDED";  // entered the filter
                cache_[key] = obj;
              }
            }
            if (deliver) dispatch_(type, obj);
            return !stop_.load();
          },
          &stop_, 300, opts_.label_selector, opts_.field_selector);
      {
        std::lock_guard<std::mutex> g(mu_);
        if (!last.empty()) rv_ = last;
      }
      backoff_ms = 100;
    } catch (const KubeError& e) {
      if (e.gone()) {
        log_.info("watch expired; relisting", Json::object().set("error", e.what()));
        need_list = true;
        continue;
      }
      log_.warn("list/watch failed", Json::object().set("error", e.what()).set("backoffMs", backoff_ms));
      need_list = true;
      backoff_(backoff_ms);
      backoff_ms = std::min(backoff_ms * 2, 5000);
    } catch (const std::exception& e) {
      log_.warn("list/watch transport error", Json::object().set("error", e.what()).set("backoffMs", backoff_ms));
      need_list = true;
      backoff_(backoff_ms);
      backoff_ms = std::min(backoff_ms * 2, 5000);
    }
  }
  ticker.join();
}

}  // namespace gpupool

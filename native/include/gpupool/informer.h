// List+watch informer with a local cache (controller-runtime's shared informer analogue).
//
//   list -> diff into cache (ADDED/MODIFIED/DELETED to handlers) -> watch from the list RV
//   (bookmarks keep the RV fresh) -> on stream end re-watch from the last RV -> on 410 Gone
//   re-list -> on error exponential backoff. Every ``resync`` period all cached objects are
//   re-delivered as "RESYNC" (the level-triggered drift detector, README.md:232-234).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "gpupool/kube.h"
#include "gpupool/log.h"

namespace gpupool {

struct InformerOptions {
  // server-side filters of both the LIST and the WATCH (an object leaving the selection arrives
  // as DELETED, as from a real apiserver)
  std::string label_selector, field_selector;
  // applied to every object before it is cached and handed to handlers: keep only what the
  // readers use (a cluster's pods cached whole cost the manager most of its memory)
  std::function<Json(const Json&)> transform;
  // objects it rejects are not cached at all (a watch event for one that was cached becomes
  // DELETED): an informer over a whole cluster's pods keeps only the ones its readers count
  std::function<bool(const Json&)> filter;
};

class Informer {
 public:
  // type is ADDED | MODIFIED | DELETED | RESYNC
  using Handler = std::function<void(const std::string& type, const Json& obj)>;

  Informer(KubeClient& client, ResourceRef res, std::string ns,
           std::chrono::milliseconds resync, InformerOptions opts = {});
  ~Informer();

  void add_handler(Handler h);
  void start();
  void stop();
  bool wait_synced(std::chrono::milliseconds timeout);
  bool synced() const { return synced_.load(); }

  std::optional<Json> get(const std::string& ns, const std::string& name) const;
  std::vector<Json> list() const;
  size_t size() const;
  uint64_t relists() const { return relists_.load(); }
  uint64_t events() const { return events_.load(); }  // watch events received

  static std::string key_of(const Json& obj);  // "ns/name" or "name"
  static constexpr int64_t kListPage = 500;

 private:
  void run_();
  void list_();
  void dispatch_(const std::string& type, const Json& obj);

  KubeClient& client_;
  ResourceRef res_;
  std::string ns_;
  std::chrono::milliseconds resync_;
  InformerOptions opts_;
  Logger log_;
  std::atomic<uint64_t> events_{0};

  mutable std::mutex mu_;
  std::map<std::string, Json> cache_;
  std::vector<Handler> handlers_;
  std::string rv_;
  std::atomic<bool> stop_{false};
  void backoff_(int ms);  // sleeps ``ms`` unless stop() is called meanwhile
  std::atomic<bool> synced_{false};
  std::atomic<uint64_t> relists_{0};
  std::condition_variable synced_cv_;
  std::thread th_;
};

}  // namespace gpupool

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

class Informer {
 public:
  // type is ADDED | MODIFIED | DELETED | RESYNC
  using Handler = std::function<void(const std::string& type, const Json& obj)>;

  Informer(KubeClient& client, ResourceRef res, std::string ns,
           std::chrono::milliseconds resync);
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

  static std::string key_of(const Json& obj);  // "ns/name" or "name"

 private:
  void run_();
  void list_();
  void dispatch_(const std::string& type, const Json& obj);

  KubeClient& client_;
  ResourceRef res_;
  std::string ns_;
  std::chrono::milliseconds resync_;
  Logger log_;

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

#include "gpupool/leader.h"

#include <atomic>
#include <limits>
#include <mutex>
#include <thread>

namespace gpupool {

namespace {
using fence_clock = std::chrono::steady_clock;
// steady-clock nanoseconds until which acting is allowed; max: no leader election in this process
std::atomic<int64_t> g_fence_until_ns{std::numeric_limits<int64_t>::max()};

int64_t fence_now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(fence_clock::now().time_since_epoch()).count();
}
}  // namespace

bool leader_fence_ok() { return fence_now_ns() < g_fence_until_ns.load(); }

namespace {
std::mutex g_token_mu;
LeaderToken g_token;  // epoch -1: no election
}  // namespace

LeaderToken leader_token() {
  std::lock_guard<std::mutex> g(g_token_mu);
  return g_token;
}

LeaderElector::LeaderElector(KubeClient& client, LeaderConfig cfg)
    : client_(client), cfg_(std::move(cfg)), log_(Logger("leader").with("identity", cfg_.identity)) {
  g_fence_until_ns = 0;  // election on: nothing may act until the lease is ours
}

bool LeaderElector::try_acquire_or_renew() {
  std::string now = microtime_now();
  int dur_s = static_cast<int>(std::chrono::duration_cast<std::chrono::seconds>(cfg_.lease_duration).count());
  Json lease;
  try {
    lease = client_.get(res::leases(), cfg_.ns, cfg_.name);
  } catch (const KubeError& e) {
    if (!e.not_found()) throw;
    Json obj = Json::object();
    obj["apiVersion"] = "coordination.k8s.io/v1";
    obj["kind"] = "Lease";
    obj["metadata"]["name"] = cfg_.name;
    obj["metadata"]["namespace"] = cfg_.ns;
    obj["spec"]["holderIdentity"] = cfg_.identity;
    obj["spec"]["leaseDurationSeconds"] = dur_s;
    obj["spec"]["acquireTime"] = now;
    obj["spec"]["renewTime"] = now;
    obj["spec"]["leaseTransitions"] = 0;
    try {
      const Json made = client_.create(res::leases(), cfg_.ns, obj);
      leader_ = true;
      std::lock_guard<std::mutex> g(g_token_mu);
      g_token = {cfg_.identity, 0, made.path("metadata.creationTimestamp").str_or(""),
                 made.path("metadata.uid").str_or("")};
      return true;
    } catch (const KubeError& e2) {
      if (e2.code == 409) return false;  // someone else created it first
      throw;
    }
  }
  const Json& spec = lease["spec"];
  const std::string& holder = spec["holderIdentity"].as_string();
  bool mine = holder == cfg_.identity;
  // the holder's record as we see it: any renewal (or hand-over) changes it
  const std::string record = holder + "|" + spec["renewTime"].str_or("") + "|" +
                             lease.path("metadata.resourceVersion").str_or("");
  const auto steady_now = std::chrono::steady_clock::now();
  if (record != observed_record_) {
    observed_record_ = record;
    observed_at_ = steady_now;
  }
  if (!mine && !holder.empty()) {
    auto duration = std::chrono::seconds(spec["leaseDurationSeconds"].as_int(dur_s));
    if (steady_now < observed_at_ + duration) {
      leader_ = false;
      return false;  // held by a live leader: its record changed less than a lease ago (our clock)
    }
  }
  Json upd = lease;
  upd["spec"]["holderIdentity"] = cfg_.identity;
  upd["spec"]["leaseDurationSeconds"] = dur_s;
  upd["spec"]["renewTime"] = now;
  if (!mine) {
    upd["spec"]["acquireTime"] = now;
    upd["spec"]["leaseTransitions"] = spec["leaseTransitions"].as_int(0) + 1;
  }
  Json stored;
  try {
    stored = client_.update(res::leases(), cfg_.ns, upd);
  } catch (const KubeError& e) {
    if (e.conflict()) {
      leader_ = false;
      return false;
    }
    throw;
  }
  leader_ = true;
  {
    std::lock_guard<std::mutex> g(g_token_mu);
    const Json& md = stored.is_object() ? stored["metadata"] : lease["metadata"];
    g_token = {cfg_.identity, upd["spec"]["leaseTransitions"].as_int(0),
               md["creationTimestamp"].str_or(""), md["uid"].str_or("")};
  }
  return true;
}

void LeaderElector::run(const std::function<void()>& on_started,
                        const std::function<void()>& on_stopped, const std::atomic<bool>* stop) {
  using clock = std::chrono::steady_clock;
  while (!stop->load()) {
    bool ok = false;
    try {
      ok = try_acquire_or_renew();
    } catch (const std::exception& e) {
      log_.warn("lease acquire failed", Json::object().set("error", e.what()));
    }
    if (ok) break;
    std::this_thread::sleep_for(cfg_.retry_period);
  }
  if (stop->load()) return;
  auto fence_from = [this](clock::time_point renewed) {
    g_fence_until_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                           (renewed + cfg_.renew_deadline).time_since_epoch()).count();
  };
  auto last_renew = clock::now();
  fence_from(last_renew);
  log_.info("became leader", Json::object().set("lease", cfg_.ns + "/" + cfg_.name));
  on_started();
  while (!stop->load()) {
    std::this_thread::sleep_for(std::min(cfg_.retry_period, std::chrono::milliseconds(500)));
    if (clock::now() - last_renew < cfg_.retry_period) continue;
    bool ok = false;
    const auto attempt = clock::now();  // the renewal holds from when it was sent, not answered
    try {
      ok = try_acquire_or_renew();
    } catch (const std::exception& e) {
      log_.warn("lease renew failed", Json::object().set("error", e.what()));
    }
    if (ok) {
      last_renew = attempt;
      fence_from(attempt);
    } else if (clock::now() - last_renew > cfg_.renew_deadline) {
      log_.error("lost leadership", Json());
      leader_ = false;
      break;
    }
  }
  g_fence_until_ns = 0;
  on_stopped();
}

}  // namespace gpupool

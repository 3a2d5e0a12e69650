// Lease-based leader election (coordination.k8s.io/v1 Lease), the controller-runtime
// ``--leader-elect`` analogue. Optimistic concurrency on the Lease's resourceVersion makes
// two managers racing for an expired lease safe: exactly one update wins.
#pragma once

#include <atomic>
#include <chrono>
#include <functional>
#include <string>

#include "gpupool/kube.h"
#include "gpupool/log.h"

namespace gpupool {

struct LeaderConfig {
  std::string ns = "gpupool-system";
  std::string name = "gpupool-manager-leader";
  std::string identity;
  std::chrono::milliseconds lease_duration{15000};
  std::chrono::milliseconds renew_deadline{10000};
  std::chrono::milliseconds retry_period{2000};
};

// Fencing for a paused leader (SIGSTOP, a VM pause, a long GC-less stall): with leader election on,
// false once this process has gone longer than its renew deadline (steady clock, so time spent
// stopped counts) without renewing its lease — another replica may be leading by then. The
// controller checks it before every pass and the reconcilers before every mutating call (agent
// claim / release RPCs, status writes); the elector itself renews through the plain client. Always
// true without leader election.
bool leader_fence_ok();

// The fencing token this process holds as leader: its identity and the Lease's leaseTransitions
// when it last acquired or renewed (a takeover increments it, so a newer leader always carries a
// larger epoch). epoch < 0 without leader election. Sent on every mutating node-agent RPC; the
// agent remembers the highest epoch it has seen and refuses older ones (409 StaleLeader), so a
// leader paused between its fence check and the send cannot act after a successor took over.
//
// leaseTransitions starts again at 0 when the Lease object is deleted and created anew, so the token
// also names the Lease's generation — its creationTimestamp and uid: the agent orders tokens by
// (creationTimestamp, epoch), so a recreated Lease's leader is accepted from epoch 0 while a leader
// of the deleted Lease, however high its epoch, is refused.
struct LeaderToken {
  std::string identity;
  int64_t epoch = -1;
  std::string lease_created;  // metadata.creationTimestamp of the Lease
  std::string lease_uid;      // metadata.uid of the Lease
};
LeaderToken leader_token();

class LeaderElector {
 public:
  LeaderElector(KubeClient& client, LeaderConfig cfg);
  // Blocks: acquires, calls on_started, renews until stop/loss, then calls on_stopped.
  void run(const std::function<void()>& on_started, const std::function<void()>& on_stopped,
           const std::atomic<bool>* stop);
  // One acquire/renew attempt; returns true if we hold the lease afterwards.
  bool try_acquire_or_renew();
  bool is_leader() const { return leader_.load(); }

 private:
  KubeClient& client_;
  LeaderConfig cfg_;
  Logger log_;
  std::atomic<bool> leader_{false};
  // Expiry is timed from when *this* process saw the holder's record change (client-go's
  // observedTime), never from the holder's renewTime against our wall clock: two replicas whose
  // clocks disagree by more than leaseDurationSeconds must still not steal a live lease.
  std::string observed_record_;
  std::chrono::steady_clock::time_point observed_at_{};
};

}  // namespace gpupool

"""Leader fencing for the agent's mutating RPCs.

Every mutating RPC of a leader-elected manager carries its identity, its epoch (the Lease's
``leaseTransitions``) and the Lease's generation (``creationTimestamp`` + ``uid``:
``leaseTransitions`` starts again at 0 when the Lease is deleted and created anew). The newest
token seen is persisted in the ledger before anything acts on it; tokens are ordered by
(generation, epoch). An older one — a leader that was paused between its own fence check and the
send while a successor took over, or a leader of a Lease that has since been recreated — is
refused with 409 StaleLeader before anything is touched. A request without a token (leader
election off, an admin's gpuctl) is not checked. This is the manager step the reference leaves
out (README.md:162->242).

Narrow interface: the ledger's ``commit_leader`` (durability) and a stats dict; no agent state.
"""
from __future__ import annotations

import datetime as _dt
import logging
import threading
from typing import Callable

log = logging.getLogger("gpupool.agent.fence")

MUTATING = frozenset({"/v1/claims", "/v1/release", "/v1/cordon", "/v1/policy",
                      "/v1/maintenance"})


def _now() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


class StaleLeader(Exception):
    def __init__(self, message: str, status: int = 409, reason: str = "StaleLeader"):
        super().__init__(message)
        self.status = status
        self.reason = reason


class LeaderFence:
    def __init__(self, state: dict, persist: Callable[[dict], None],
                 stats: dict | None = None, clock: Callable[[], str] = _now):
        self.state = dict(state or {})   # {"holder", "epoch", "at", "leaseCreated", "leaseUID", ...}
        self.persist = persist
        self.stats = stats if stats is not None else {}
        self.clock = clock
        self._mu = threading.Lock()

    @property
    def epoch(self) -> int:
        return int(self.state.get("epoch", -1))

    def admit(self, method: str, path: str, headers: dict) -> None:
        """Raise StaleLeader for a stale token; record a newer one (durably) and return."""
        if method != "POST" or path not in MUTATING:
            return
        raw = headers.get("x-gpupool-leader-epoch")
        if raw is None:
            return
        try:
            epoch = int(raw)
        except ValueError:
            raise StaleLeader(f"bad leader epoch {raw!r}", 400, "BadRequest") from None
        holder = headers.get("x-gpupool-leader", "")
        lease = headers.get("x-gpupool-leader-lease")  # "<creationTimestamp> <uid>"
        created, _, uid = (lease or "").strip().partition(" ")
        with self._mu:
            cur = self.state
            cur_e, cur_h = int(cur.get("epoch", -1)), str(cur.get("holder", ""))
            cur_c, cur_u = str(cur.get("leaseCreated", "")), str(cur.get("leaseUID", ""))
            retired = list(cur.get("retiredLeaseUIDs") or [])
            newer_lease = older_lease = False
            if created and cur_c:
                # RFC 3339 UTC timestamps of one apiserver compare as strings; a Lease recreated
                # within the same second is told apart by its uid: one not seen before is the
                # newer one, one this agent has already moved past is not
                older_lease = created < cur_c or (uid != cur_u and uid in retired)
                newer_lease = not older_lease and (
                    created > cur_c or (created == cur_c and uid != cur_u))
            elif created and cur_e >= 0:
                # a fence persisted before tokens carried the Lease generation: the first token
                # that carries one is taken as the generation from then on. Comparing its
                # creationTimestamp (apiserver clock) with this fence's "at" (the agent's own
                # clock) would refuse a recreated Lease for good whenever the node clock runs
                # ahead, and every later mutating RPC with it.
                newer_lease = True
                log.warning("leader fence without a Lease generation (epoch %d of %s): adopting "
                            "lease %s of %s", cur_e, cur_h, created, holder)
            stale = older_lease or (not newer_lease and (
                epoch < cur_e or (epoch == cur_e and cur_h and holder != cur_h)))
            if stale:
                self.stats["stale_leader_refused"] = self.stats.get("stale_leader_refused", 0) + 1
                log.warning("refused %s from stale leader %s (epoch %d, lease %s; newest seen %s "
                            "at %d, lease %s)", path, holder, epoch, created or "?", cur_h, cur_e,
                            cur_c or "?")
                raise StaleLeader(f"leader {holder} epoch {epoch} is stale: {cur_h} holds "
                                  f"epoch {cur_e}" + (" of a newer Lease" if older_lease else ""))
            if newer_lease or epoch > cur_e or not cur_h or (created and not cur_c):
                if newer_lease and cur_u:
                    retired = (retired + [cur_u])[-8:]
                new = {"holder": holder, "epoch": epoch, "at": self.clock(),
                       **({"leaseCreated": created, "leaseUID": uid,
                           "retiredLeaseUIDs": retired} if created else {})}
                self.persist(new)  # durable before acting on it
                self.state = new

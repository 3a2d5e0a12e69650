"""Claim, cordon, release and policy RPCs of the agent (a mixin of ``agent.Agent``).

A claim is all-or-nothing and topology-aware: select free GPUs healthy under the pool's policy,
commit them to the ledger (durable while the probe runs), probe them in their helpers, optionally
ring their xGMI links, advertise them through the device plugin and answer with device views — the
node-local replacement of the reference's ``createVM`` loop (README.md:199-209). Release never
frees a GPU a pod still holds (``deleteVM``'s full cleanup, README.md:216-217, 239).
"""
from __future__ import annotations

import json
import os
import time

from ..api import schema
from ..ops import devlib
from . import slots as slotlib
from .common import log, now_rfc3339
from .prober import DEFAULT_TIMEOUT_S


# wake the chosen GPUs' probe helpers as soon as a claim has selected them (A/B switch)
PREWAKE = os.environ.get("GPUPOOL_PROBE_PREWAKE", "1") != "0"


class ClaimsMixin:

    def claim(self, req: dict, hold_events: bool = False) -> dict:
        """Claim ``count`` GPUs for a pool, all or nothing: select (topology), commit to the
        ledger, probe, commit, advertise through the device plugin, answer with device views.
        ``hold_events``: the pool's change events stay deferred after return until
        ``release_events`` (the RPC handler calls it once the reply is written)."""
        pool = req.get("poolUID", "")
        with self.lock:
            self._claiming[pool] = self._claiming.get(pool, 0) + 1
        try:
            st = self._claim_start(req)
            if not st.get("ok"):
                return st
            self._wait_advertised(st["_resource"], st["_uuids"])
            out = self._claim_finish(st)
            if hold_events:  # the RPC handler runs them once the reply is written
                out["_after"] = st["_after"]
            else:
                for fn in st["_after"]:
                    fn()
            return out
        finally:
            if not hold_events:
                self.release_events(pool)

    def release_events(self, pool: str) -> None:
        """End a claim's event hold: one bump for whatever changed meanwhile."""
        with self.lock:
            n = self._claiming.get(pool, 0) - 1
            if n > 0:
                self._claiming[pool] = n
                return
            self._claiming.pop(pool, None)
            flush = pool in self._deferred
            self._deferred.discard(pool)
        if flush:
            self._bump({pool})

    def _claim_start(self, req: dict) -> dict:
        pool_uid, count = req["poolUID"], int(req["count"])
        min_count, stall = self.cfg.inject_claim_delay
        if min_count > 0 and count >= min_count and stall > 0:
            log.warning("fault injection: claim of %d GPU(s) stalls %.1f s", count, stall)
            time.sleep(stall)
        policy = req.get("policy") or {}
        resource = req.get("resourceName") or schema.DEFAULT_RESOURCE
        probe_opts = req.get("probe") or {}
        timings: dict[str, float] = {}  # phase -> ms, returned to the manager as trace spans
        t_phase = time.perf_counter()
        if "_t_in" in req:  # the RPC handler's hand-off to this executor thread
            timings["executorIn"] = round((t_phase - req.pop("_t_in")) * 1e3, 3)

        def lap(name: str) -> None:
            nonlocal t_phase
            t = time.perf_counter()
            timings[name] = round((t - t_phase) * 1e3, 3)
            t_phase = t

        with self.lock:
            quarantined = self.ledger.quarantined()
            free = []
            asic_bad = self._asic_faulted()
            default_policy = self._is_default_policy(policy)
            policy_key = "" if default_policy else json.dumps(policy, sort_keys=True)
            cand = [d for uuid, d in self.by_uuid.items()
                    if uuid not in self.records and uuid not in quarantined and d.get("present", True)
                    and (not asic_bad or not asic_bad.get(self._asic_key(d), set()) - {uuid})]
            no_helper = 0
            if probe_opts.get("enabled", True) and self.prober.helpers is not None:
                # a GPU whose probe helper is held back after an exit cannot be probed now:
                # left out (another GPU, or InsufficientDevices and a retry), not failed
                ok_cand = [d for d in cand if self.prober.can_probe(d)]
                no_helper, cand = len(cand) - len(ok_cand), ok_cand
            # claimability under the requesting pool's policy (baseline = now: retired HBM pages
            # and absolute limits count, deltas start at the claim); no partition of the same ASIC
            # may carry a package-level fault (checked above)
            sharing = policy.get("sharing") or {}
            overcommitted = ""
            for d, ok in zip(cand, self._claimable(cand, policy, policy_key)):
                why = (slotlib.overcommit(sharing, int(d.get("memTotalBytes") or 0),
                                          self.cfg.hbm_reserve_bytes)
                       or slotlib.cu_floor(sharing, d)) if ok else ""
                if why:
                    overcommitted = why
                elif ok:
                    free.append(d["index"])
            if self.prober.helpers is not None and probe_opts.get("enabled", True):
                # a GPU released a moment ago may still be starting its probe helper (it was
                # parked under a tenant): claims take warm GPUs first and a cold one only when
                # the warm ones do not suffice (the probe then waits for its helper)
                warm_idx = {d["index"] for d in cand if self.prober.warm(d)}
                warm = [i for i in free if i in warm_idx]
                if len(warm) >= count:
                    free = warm
            owned = [self.by_uuid[u]["index"] for u, r in self.records.items()
                     if r["poolUID"] == pool_uid and u in self.by_uuid]
            if count == 1 and not owned:
                # one GPU for an empty pool: every candidate scores the same on links and NUMA,
                # so the selector's tie-break (lowest index) decides — no native call needed
                sel = [min(free)] if free else []
            else:
                topo = self.snap.get("topology") or {}
                n = len(self.snap["devices"])
                weights = topo.get("weights") or [[0 if i == j else 15 for j in range(n)]
                                                  for i in range(n)]
                numa = [d.get("numa", 0) for d in sorted(self.snap["devices"],
                                                         key=lambda x: x["index"])]
                sel = devlib.select(count, free, owned, req.get("topologyPolicy", "xgmi-packed"),
                                    weights, numa)
            if len(sel) < count and overcommitted:
                return {"ok": False, "reason": "SharingOvercommitted" if "hbmBytesPerSlot"
                        in overcommitted else "SharingCUsBelowXCDs",
                        "message": f"{overcommitted} on {self.cfg.node}", "devices": []}
            if len(sel) < count:
                return {"ok": False, "reason": "InsufficientDevices",
                        "message": f"need {count} free healthy GPU(s) on {self.cfg.node}, "
                                   f"{len(free)} available (all-or-nothing)"
                                   + (f"; {no_helper} more wait for their probe helper to be "
                                      f"replaced" if no_helper else ""), "devices": []}
            by_index = {d["index"]: d for d in self.snap["devices"]}
            chosen = [by_index[i] for i in sel]
            if probe_opts.get("enabled", True) and PREWAKE:
                self.prober.prewake(chosen)
            lap("select")
            ts = now_rfc3339()
            # a record still 'Probing' past its probe deadline (+ PROBE_GRACE_S) is reported
            # probeOverdue: the manager replaces it instead of waiting on it forever
            since = (time.monotonic(), float(probe_opts.get("timeoutSeconds") or DEFAULT_TIMEOUT_S))
            for d in chosen:
                self._probing_since[d["uuid"]] = since
            for d in chosen:
                rec = {"uuid": d["uuid"], "poolUID": pool_uid, "pool": req.get("pool", ""),
                       "resourceName": resource, "policy": policy,
                       "baseline": {"ecc": dict(d.get("ecc") or {}),
                                    "eccUmc": dict(d.get("eccUmc") or {})}, "claimedAt": ts,
                       "state": "Probing", "probe": None, "probeAttempts": 1}
                self.records[d["uuid"]] = rec
            # The claim becomes durable while the probe runs (the ledger's writer fsyncs it
            # concurrently); the RPC answers only after it is on disk, so no crash can ever make
            # the manager believe it owns GPUs a restarted agent would hand out again.
            # encoded and fsynced by the ledger's writer while the probe runs
            claim_seq = self.ledger.commit(self.records, durable=False, lock=self.lock)
            self.stats["claims"] += len(chosen)
        lap("commit")
        for d in chosen:  # an in-flight HBM scrub window finishes and hands its buffer back
            self.scrubber.yield_device(d["uuid"])
        lap("scrubYield")
        cold = [d for d in chosen if self.prober.helpers is not None and
                probe_opts.get("enabled", True) and not self.prober.warm(d)]
        if cold:
            # a helper still starting: the wait comes out of the probe's own deadline (one
            # deadline per claim, as inside Helper.call; probeOverdue is measured against it)
            budget = float(probe_opts.get("timeoutSeconds") or DEFAULT_TIMEOUT_S)
            waited = max(self.prober.helpers.wait_ready(d["uuid"], budget) for d in cold)
            probe_opts = {**probe_opts, "timeoutSeconds": max(0.5, budget - waited / 1e3)}
            with self.lock:
                self.stats["claim_helper_waits"] = self.stats.get("claim_helper_waits", 0) + 1
                self.stats["claim_helper_wait_ms_sum"] = \
                    self.stats.get("claim_helper_wait_ms_sum", 0.0) + waited
            lap("helperWait")
        # probes run outside the lock, concurrently across GPUs, each in its GPU's probe helper
        t0 = time.perf_counter()
        results = self.prober.probe_many(chosen, {**probe_opts, "enabled":
                                                  probe_opts.get("enabled", True)})
        probe_wall = (time.perf_counter() - t0) * 1e3
        lap("probe")
        if probe_opts.get("xgmiPeerCheck"):
            self._xgmi_check(pool_uid, chosen, results, probe_opts)
            lap("xgmi")
        with self.lock:
            for d, res in zip(chosen, results):
                rec = self.records.get(d["uuid"])
                if rec is None or rec["poolUID"] != pool_uid:
                    continue  # released concurrently
                rec["probe"] = res
                self._probing_since.pop(d["uuid"], None)
                if rec.get("state") == "Probing":  # a pool may have cordoned it meanwhile
                    rec["state"] = "Claimed"
                self.last_probe[d["uuid"]] = res
                self._probe_mono[d["uuid"]] = time.monotonic()
                self.stats["probes"] += 1
                self.stats["probe_ms_sum"] += float(res.get("ms", 0.0))
                if not res.get("passed"):
                    self.stats["probe_failures"] += 1
                    if res.get("timedOut"):
                        self.stats["probe_timeouts"] = self.stats.get("probe_timeouts", 0) + 1
                    elif res.get("crashed"):
                        self.stats["probe_crashes"] = self.stats.get("probe_crashes", 0) + 1
            if not self._is_default_policy(policy):
                # under the default policy the claimed GPU's verdict (baseline = the claim's
                # snapshot = now) is the free GPU's current one: nothing to re-evaluate
                self._evaluate_some([d["uuid"] for d in chosen])
        self.ledger.flush(claim_seq)
        lap("commit2")
        self._ensure_plugin(resource)
        self._notify_plugins(sync=True)  # handed to the kubelet's stream before the reply

        def record_claimed() -> None:
            # Probing -> Claimed (with the probe result) goes to the ledger's background writer
            # after the reply: a crash may lose it safely (a restarted agent probes the GPU
            # again, _reprobe_interrupted); the claim itself was made durable above
            with self.lock:
                self.ledger.commit(self.records, durable=False)
        return {"ok": True, "probeWallMs": probe_wall, "timingsMs": timings, "_t_phase": t_phase,
                "_after": [record_claimed],
                "_resource": resource, "_uuids": [d["uuid"] for d in chosen],
                "_indices": [d["index"] for d in chosen], "_pool": req.get("pool")}

    def _claim_finish(self, st: dict) -> dict:
        timings = st["timingsMs"]
        t = time.perf_counter()
        timings["advertise"] = round((t - st["_t_phase"]) * 1e3, 3)
        pods = self._pods_by_device()
        with self.lock:
            views = [self.device_view(u, pods) for u in st["_uuids"]]
        timings["view"] = round((time.perf_counter() - t) * 1e3, 3)
        # logged after the reply (formatting a log record costs ~0.1 ms on the claim path)
        st["_after"].append(lambda: log.info(
            "claimed %d GPU(s) for %s: %s (probe wall %.1f ms; phases %s)", len(views),
            st["_pool"], st["_indices"], st["probeWallMs"], timings))
        return {"ok": True, "devices": views, "probeWallMs": st["probeWallMs"],
                "timingsMs": timings, "_t_done": time.perf_counter()}

    def set_maintenance(self, ref: str, on: bool, reason: str = "") -> dict:
        """Admin GPU cordon / uncordon (``gpuctl gpu cordon NODE GPU``). A cordoned GPU is never
        claimed; if a pool holds it, it turns unhealthy (AdminMaintenance) and the pool replaces
        it through the normal drain -> release path. Uncordon clears it (and any quarantine)."""
        with self.lock:
            uuid = next((u for u, d in self.by_uuid.items()
                         if ref in (u, d.get("hipUUID"), str(d.get("index")))), None)
            if uuid is None:
                return {"ok": False, "reason": "NotFound", "message": f"no GPU {ref!r} on {self.cfg.node}"}
            if on:
                self.maintenance[uuid] = reason
                self.ledger.quarantine(uuid, 1e12, f"AdminMaintenance: {reason}", maintenance=True)
            else:
                self.maintenance.pop(uuid, None)
                self.ledger.clear_quarantine(uuid)
            changed = self._evaluate_all()
            pool = (self.records.get(uuid) or {}).get("poolUID")
        self._bump(changed | ({pool} if pool else {"*free*"}))
        self._notify_plugins()
        return {"ok": True, "uuid": uuid, "maintenance": on, "claimedBy": pool}

    def cordon(self, pool_uid: str, uuids: list[str]) -> dict:
        seq = 0
        with self.lock:
            n = 0
            for u in uuids:
                rec = self.records.get(u)
                if rec and rec["poolUID"] == pool_uid and rec.get("state") != "Draining":
                    rec["state"] = "Draining"
                    rec["drainStartedAt"] = now_rfc3339()
                    n += 1
            if n:  # serialised under the lock, made durable (fsync) outside it
                seq = self.ledger.commit(self.records, durable=False)
        if seq:
            self.ledger.flush(seq)
        if n:
            self._pods_kick.set()  # watch the evicted pods go
            if self._podres is not None:
                try:  # the drain that follows must see every pod on these GPUs, not a cached map
                    self._refresh_pods()
                except Exception as e:
                    log.debug("podresources refresh on cordon failed: %s", e)
        self._notify_plugins()
        return {"ok": True, "cordoned": n}

    def release(self, pool_uid: str, uuids: list[str]) -> dict:
        try:
            pods = self._pods_by_device(fresh=True)
        except Exception as e:
            return {"ok": False, "reason": "PodResourcesUnavailable", "released": [],
                    "message": f"cannot confirm the GPUs are pod-free: {e}"}
        released, refused, quarantined = [], [], []
        seq = 0
        with self.lock:
            for u in uuids:
                rec = self.records.get(u)
                if not rec or rec["poolUID"] != pool_uid:
                    continue
                if pods.get(u):
                    refused.append(u)  # never release a GPU that still runs a pod
                    continue
                probe_ok = (rec.get("probe") or {}).get("passed", True)
                healthy = self.verdicts.get(u, {}).get("healthy", True)
                if u in self.maintenance:
                    pass  # stays cordoned (its non-expiring maintenance entry is already there)
                elif not probe_ok or not healthy:
                    why = ("ProbeFailed: " + str((rec.get("probe") or {}).get("error") or
                                                  "probe failed")) if not probe_ok else "; ".join(
                        self.verdicts.get(u, {}).get("reasons", []))
                    quarantined.append(self.ledger.quarantine(u, self.cfg.quarantine_s, why,
                                                              write=False))
                del self.records[u]
                self._probing_since.pop(u, None)
                released.append(u)
                self.freed_at[u] = time.monotonic()  # its pods' VRAM was just freed (scrubber)
            if released:
                seq = self.ledger.commit(self.records, durable=False)
            self.stats["releases"] += len(released)
            self._evaluate_some(released)
        # a parked helper restarts now (if the pod view has not restarted it already): the GPU
        # is free at once, and claims take it only when no warm GPU suffices (_claim_start), so
        # neither this release nor the next claim normally waits for its HIP init
        restarting = 0
        for u in released:
            d = self.by_uuid.get(u)
            if d is not None and self.prober.helpers is not None:
                if u in self.prober.parked():
                    self.prober.unpark(d)
                restarting += not self.prober.warm(d)
        if restarting:
            with self.lock:
                self.stats["release_helpers_restarting"] = \
                    self.stats.get("release_helpers_restarting", 0) + restarting
        # durable before the reply, but no fsync under the lock (node views and claims wait on it)
        for q in quarantined:
            self.ledger.persist_quarantine(q)
        if seq:
            self.ledger.flush(seq)
        if released:
            self._bump({pool_uid, "*free*"})  # capacity freed: wake pools waiting for GPUs
        self._notify_plugins()
        if refused:
            return {"ok": False, "reason": "PodsRunning", "released": released,
                    "message": f"GPUs still hold pods: {refused}"}
        return {"ok": True, "released": released, "helpersRestarting": restarting}

    def update_policy(self, pool_uid: str, policy: dict, resource: str | None) -> dict:
        changed = set()
        seq = 0
        with self.lock:
            for u, rec in self.records.items():
                if rec["poolUID"] != pool_uid:
                    continue
                rec["policy"] = policy
                if resource and rec.get("resourceName") != resource:
                    rec["resourceName"] = resource
                changed.add(u)
            if changed:
                seq = self.ledger.commit(self.records, durable=False)
            self._evaluate_all()
        if seq:
            self.ledger.flush(seq)
        if resource:
            self._ensure_plugin(resource)
        self._notify_plugins()
        return {"ok": True, "updated": len(changed)}

"""xGMI link coverage (a mixin of ``agent.Agent``): peer-copy rings over a pool's GPUs at claim
time (``spec.probe.xgmiPeerCheck``) and over idle GPUs periodically, in an order that walks every
GPU pair of the node; per-pair verdicts are persisted in the ledger.
"""
from __future__ import annotations

import time

from .common import log, now_rfc3339


class XgmiMixin:
    @staticmethod
    def _pair_key(a: str, b: str) -> str:
        return "|".join(sorted((a, b)))

    def _ring_order(self, devs: list[dict]) -> list[dict]:
        """Order of the next peer-copy ring over ``devs``. A ring checks n of the n(n-1)/2 GPU
        pairs; always ringing in index order would check the same 8 of an 8-GPU node's 28 pairs
        forever. Instead each ring is built greedily from every start GPU over the least recently
        checked pairs (never-checked first) and the ring with the oldest links wins, so claims
        and idle rechecks together walk every pair (28/28 after a handful of rings)."""
        devs = sorted(devs, key=lambda d: d["index"])
        if len(devs) <= 2:
            return devs
        with self.lock:
            pairs = dict(self.xgmi_pairs)

        def age(a: dict, b: dict) -> float:
            r = pairs.get(self._pair_key(a["uuid"], b["uuid"]))
            return float(r.get("ts", 0.0)) if r else 0.0
        best, best_cost = devs, None
        for start in devs:
            ring, left = [start], [d for d in devs if d is not start]
            while left:
                nxt = min(left, key=lambda d: (age(ring[-1], d), d["index"]))
                ring.append(nxt)
                left.remove(nxt)
            ages = [age(ring[i], ring[(i + 1) % len(ring)]) for i in range(len(ring))]
            cost = (sum(1 for a in ages if a > 0), sum(ages))  # fewest re-checked links, oldest
            if best_cost is None or cost < best_cost:
                best, best_cost = ring, cost
        return best

    @staticmethod
    def _link_verdict(link: dict, floor: float) -> str:
        """ok | bad (corrupted data or a copy below the bandwidth floor: the link is faulty) |
        unavailable (no peer access, a HIP error, a device not visible: the check could not run,
        which says nothing about the link — XGMIPeerCheckUnavailable, never a replace loop)."""
        if link.get("canAccessPeer") is False:
            return "unavailable"
        if int(link.get("badBits") or 0) > 0:
            return "bad"
        if not link.get("passed"):
            return "unavailable" if link.get("error") else "bad"
        if floor > 0 and float(link.get("GBps") or 0) < floor:
            return "bad"
        return "ok"

    def _record_links(self, links: dict[str, dict], floor: float) -> dict[str, str]:
        """Remember every measured link per GPU pair (ledger-persisted); returns src -> verdict."""
        out = {}
        now, at = time.time(), now_rfc3339()
        with self.lock:
            for src, link in links.items():
                dst = link.get("peer", "")
                v = self._link_verdict(link, floor)
                out[src] = v
                self.xgmi_pairs[self._pair_key(src, dst)] = {
                    "src": src, "dst": dst, "verdict": v, "ts": now, "at": at,
                    "GBps": round(float(link.get("GBps") or 0), 1),
                    **({"error": str(link["error"])[:200]} if link.get("error") else {})}
            self.stats["xgmi_links_checked"] = self.stats.get("xgmi_links_checked", 0) + len(links)
            snapshot = dict(self.xgmi_pairs)
        self.ledger.commit_xgmi(snapshot)
        return out

    @staticmethod
    def _link_error(src: str, link: dict, floor: float) -> str:
        why = link.get("error") or f"{link.get('badBits')} bad bits"
        if int(link.get("badBits") or 0) == 0 and link.get("passed") and floor > 0:
            why = f"{float(link.get('GBps') or 0):.0f} GB/s < floor {floor:.0f}"
        return f"XGMIPeerCheckFailed: {src} -> {link.get('peer')}: {why}"

    def _fail_claimed(self, uuid: str, pool_uid: str | None, error: str) -> str | None:
        """A bad link found on an already-claimed GPU: its probe result fails (DeviceProbePassed
        False -> the pool replaces it). Returns the pool to wake."""
        rec = self.records.get(uuid)
        if rec is None or rec.get("state") != "Claimed" or \
                (pool_uid is not None and rec["poolUID"] != pool_uid):
            return None
        rec["probe"] = {**(rec.get("probe") or {}), "passed": False, "error": error}
        self.last_probe[uuid] = rec["probe"]
        self.stats["probe_failures"] += 1
        return rec["poolUID"]

    def _xgmi_check(self, pool_uid: str, chosen: list[dict], results: list[dict],
                    opts: dict) -> None:
        """spec.probe.xgmiPeerCheck: a peer-copy ring across all of the pool's GPUs on this node
        (already-owned + newly chosen), in the coverage-rotating order of ``_ring_order``. Every
        measured link counts: a bad link touching a new GPU fails that GPU's probe (the sender if
        it is new, else the receiving new GPU — so an owned GPU's bad link into a new one fails
        the new one), a bad link between two owned GPUs fails the sender's claim. A link whose
        check could not run (no peer access, HIP error) marks the GPU ``xgmi.unavailable`` and
        surfaces as XGMILinksHealthy=Unknown (XGMIPeerCheckUnavailable) instead of a replace."""
        with self.lock:
            owned = [self.by_uuid[u] for u, r in self.records.items()
                     if r["poolUID"] == pool_uid and u in self.by_uuid and r.get("state") == "Claimed"]
        # GPUs running tenant pods keep no agent context (parked helpers): their links are
        # checked once they are pod-free again (idle rechecks), not under a tenant
        parked = self.prober.parked()
        members = [d for d in {d["uuid"]: d for d in owned + chosen}.values()
                   if d["uuid"] not in parked]
        if len(members) < 2:
            return  # one GPU of the pool on this node: no link to ring
        ring = self._ring_order(members)
        links = self.prober.peer_ring(ring, opts)
        floor = float(opts.get("minXgmiGBps") or 0)
        verdicts = self._record_links(links, floor)
        new = {d["uuid"]: r for d, r in zip(chosen, results)}
        wake = set()
        for src, link in links.items():
            dst, v = link.get("peer", ""), verdicts[src]
            owner = src if src in new else dst if dst in new else None
            if owner is None:
                if v == "bad":
                    with self.lock:
                        p = self._fail_claimed(src, pool_uid, self._link_error(src, link, floor))
                    if p:
                        wake.add(p)
                continue
            res = new[owner]
            entry = {**link, "src": src, "verdict": v}
            if owner == src or "xgmi" not in res:
                res["xgmi"] = entry
            if v == "unavailable":
                res["xgmi"] = {**res["xgmi"], "unavailable": True,
                               "error": "XGMIPeerCheckUnavailable: " + str(link.get("error"))}
            elif v == "bad" and res.get("passed"):
                res["passed"] = False
                res["error"] = self._link_error(src, link, floor)
                res["xgmi"] = entry
        if wake:
            with self.lock:
                self.ledger.commit(self.records)
            self._bump(wake)

    def xgmi_recheck(self, force: bool = False) -> dict:
        """Idle xGMI coverage pass (every ``xgmi_recheck_s``): one peer-copy ring over every GPU
        of the node that runs no pod — free and idle claimed ones — in coverage-rotating order,
        so links no pool ever rings (between pools, into free GPUs) are checked too. A bad link
        fails the sender: a claimed GPU's probe (its pool replaces it), a free GPU is quarantined."""
        now = time.monotonic()
        every = self.cfg.xgmi_recheck_s
        if not force and (every <= 0 or now - self._xgmi_last < every):
            return {}
        self._xgmi_last = now
        if self.probe_mode not in ("inproc", "simulated", "helper", "helper-sim"):
            return {}
        pods = self._pods_by_device()
        with self.lock:
            quarantined = self.ledger.quarantined()
            idle = [d for u, d in self.by_uuid.items()
                    if d.get("present", True) and not pods.get(u) and u not in self.resetting and
                    u not in quarantined and u not in self._rechecking and
                    (u not in self.records or self.records[u].get("state") == "Claimed")]
            for d in idle:
                self._rechecking.add(d["uuid"])
        try:
            if len(idle) < 2:
                return {"checked": 0}
            ring = self._ring_order(idle)
            links = self.prober.peer_ring(ring, {"xgmiBytes": self.cfg.xgmi_recheck_bytes})
            verdicts = self._record_links(links, 0.0)
            wake, bad = set(), []
            for src, v in verdicts.items():
                if v != "bad":
                    continue
                err = self._link_error(src, links[src], 0.0)
                bad.append(err)
                with self.lock:
                    p = self._fail_claimed(src, None, err)
                    if p:
                        wake.add(p)
                    elif src not in self.records:
                        self.ledger.quarantine(src, self.cfg.quarantine_s, err)
                        wake.add("*free*")
            if wake:
                with self.lock:
                    self.ledger.commit(self.records)
                    self._evaluate_all()
                self._bump(wake)
                self._notify_plugins()
            for err in bad:
                log.warning("idle xGMI check: %s", err)
                self.node_event("XGMIPeerCheckFailed", err)
            return {"checked": len(links), "bad": bad,
                    "unavailable": [s for s, v in verdicts.items() if v == "unavailable"]}
        finally:
            with self.lock:
                for d in idle:
                    self._rechecking.discard(d["uuid"])

    def _xgmi_summary(self, uuid: str) -> dict | None:
        """Link coverage of one GPU: pairs with the node's other GPUs checked so far, failed and
        unchecked-able peers, last check time (status.devices[].xgmi)."""
        others = [u for u in self.by_uuid if u != uuid]
        if not others:
            return None
        covered, failed, unavail, last = 0, [], [], ""
        for o in others:
            r = self.xgmi_pairs.get(self._pair_key(uuid, o))
            if not r:
                continue
            covered += 1
            last = max(last, r.get("at", ""))
            idx = str(self.by_uuid.get(o, {}).get("index", o))
            if r.get("verdict") == "bad":
                failed.append(idx)
            elif r.get("verdict") == "unavailable":
                unavail.append(idx)
        out = {"pairsCovered": covered, "pairsTotal": len(others)}
        if failed:
            out["failedPeers"] = failed
        if unavail:
            out["unavailablePeers"] = unavail
        if last:
            out["lastCheckedAt"] = last
        return out

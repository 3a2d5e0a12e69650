"""Health sampling and verdicts of the agent's GPUs (a mixin of ``agent.Agent``).

Full telemetry samples (``sample``) and the fast health-only poll (``poll_health``) feed
libmi355x_dev's verdicts under each owning pool's policy (free GPUs: the default policy); ASIC-
scoped faults fan out to sibling partitions; amdsmi device events and the fault overlay trigger an
immediate sample; claimed, pod-free GPUs are re-probed on ``spec.probe.recheckSeconds``. Changes
are published through ``Agent._bump`` (the manager's event feed) and the device plugins.
"""
from __future__ import annotations

import json
import os
import threading
import time

from ..api import schema
from ..ops import devlib
from .common import log, now_rfc3339


class HealthMixin:
    def _policy_for(self, uuid: str) -> dict:
        rec = self.records.get(uuid)
        return (rec or {}).get("policy") or {}

    # Health categories that belong to the ASIC package, not to one partition: in CPX mode the 8
    # logical GPUs of an MI355X share its HBM stacks (ECC, retired pages), xGMI links and sensors,
    # so a fault seen through any partition is a fault of all of them. Probe results, partition
    # mode and admin maintenance stay per logical GPU.
    ASIC_SCOPED = ("xgmiOk", "eccOk", "thermalOk")

    @staticmethod
    def _asic_key(d: dict) -> str:
        return str((d.get("asic") or {}).get("serial") or "") or f"bdf:{d.get('bdf', '')[:-1]}"

    def _fan_out_asic(self, raw: dict[str, dict]) -> dict[str, dict]:
        """Spread ASIC-scoped faults of one partition to its siblings (no-op in SPX mode)."""
        groups: dict[str, list[str]] = {}
        for u, d in self.by_uuid.items():
            groups.setdefault(self._asic_key(d), []).append(u)
        out = dict(raw)
        for members in groups.values():
            if len(members) < 2:
                continue
            for flag in self.ASIC_SCOPED:
                bad = [m for m in members if raw.get(m, {}).get(flag) is False]
                if not bad:
                    continue
                for s_ in members:
                    if s_ in bad:
                        continue
                    src = bad[0]
                    why = raw[src].get("reasons", [])
                    v = dict(out[s_])
                    v[flag] = False
                    v["healthy"] = False
                    v["reasons"] = list(v.get("reasons") or []) + [
                        f"ASICFault: sibling partition {self.by_uuid[src].get('index')} of this "
                        f"ASIC: {'; '.join(why) or flag}"]
                    out[s_] = v
        return out

    # spec.health defaults (the schema's): a pool asking for exactly these, with no partition
    # requirement, is judged like a free GPU is after every poll
    _DEFAULT_HEALTH = {k: v["default"] for k, v in
                       schema.MI355X_SPEC["properties"]["health"]["properties"].items()
                       if "default" in v}

    @classmethod
    def _is_default_policy(cls, policy: dict) -> bool:
        h = policy.get("health") or {}
        if set(h) - set(cls._DEFAULT_HEALTH) or any(h.get(k, v) != v
                                                     for k, v in cls._DEFAULT_HEALTH.items()):
            return False
        p = policy.get("partition") or {}
        return p.get("compute", "Any") == "Any" and p.get("memory", "Any") == "Any"

    def _claimable(self, devs: list[dict], policy: dict, policy_key: str) -> list[bool]:
        """Healthy under the requesting pool's policy with baseline = now, for each device.
        Under the default policy that is the free GPU's current verdict (re-evaluated on every
        health change, with the same baseline = now). Otherwise cached per (device snapshot,
        policy) — a snapshot dict is replaced, never mutated, when the device changes, which on
        hardware is every poll (temperatures move) — and the misses evaluated in one native call."""
        if self._is_default_policy(policy):
            return [bool(self.verdicts.get(d["uuid"], {}).get("healthy")) for d in devs]
        out: list[bool | None] = []
        miss = []
        for d in devs:
            hit = self._claim_cache.get((d["uuid"], policy_key))
            if hit is not None and hit[0] is d:
                out.append(hit[1])
            else:
                out.append(None)
                miss.append(d)
        if miss:
            if len(self._claim_cache) > 4096:
                self._claim_cache.clear()
            vs = devlib.evaluate_batch([(d, d, policy) for d in miss])
            it = iter(vs)
            for i, d in enumerate(devs):
                if out[i] is None:
                    ok = bool(next(it).get("healthy"))
                    self._claim_cache[(d["uuid"], policy_key)] = (d, ok)
                    out[i] = ok
        return out  # type: ignore[return-value]

    def _asic_faulted(self) -> dict[str, set[str]]:
        """ASIC key -> partitions whose own (pre-fan-out) ASIC-scoped health failed."""
        bad: dict[str, set[str]] = {}
        for u, v in self.verdicts.items():
            d = self.by_uuid.get(u)
            if d is not None and any(v.get(f) is False for f in self.ASIC_SCOPED) and \
                    not any(str(r).startswith("ASICFault:") for r in v.get("reasons") or []):
                bad.setdefault(self._asic_key(d), set()).add(u)
        return bad

    def _evaluate_some(self, uuids: list[str]) -> set[str]:
        """Re-evaluate only ``uuids`` (their record — baseline, policy — just changed: a claim or
        a release), unless a package-level fault needs the ASIC fan-out: then everything.
        Called under self.lock."""
        uuids = [u for u in uuids if u in self.by_uuid]
        if not uuids or self._asic_faulted():
            return self._evaluate_all()
        verdicts = devlib.evaluate_batch([
            (self.by_uuid[u], (self.records.get(u) or {}).get("baseline") or self.by_uuid[u],
             self._policy_for(u)) for u in uuids])
        if any(v.get(f) is False for v in verdicts for f in self.ASIC_SCOPED):
            return self._evaluate_all()
        return self._apply_verdicts(dict(zip(uuids, verdicts)))

    def _evaluate_all(self) -> set[str]:
        """Re-evaluate every device; returns pool UIDs whose devices changed verdict."""
        uuids = list(self.by_uuid)
        verdicts = devlib.evaluate_batch([
            (self.by_uuid[u], (self.records.get(u) or {}).get("baseline") or self.by_uuid[u],
             self._policy_for(u)) for u in uuids])
        raw: dict[str, dict] = dict(zip(uuids, verdicts))
        changed = self._apply_verdicts(self._fan_out_asic(raw))
        # claimed devices that vanished from enumeration
        for uuid, rec in self.records.items():
            if uuid not in self.by_uuid:
                v = {"healthy": False, "present": False, "xgmiOk": True, "eccOk": True,
                     "thermalOk": True, "partitionOk": True,
                     "reasons": ["DeviceMissing: device no longer enumerated"]}
                if self.verdicts.get(uuid, {}).get("present", True):
                    changed.add(rec["poolUID"])
                self.verdicts[uuid] = v
        return changed

    def _apply_verdicts(self, raw: dict[str, dict]) -> set[str]:
        """Store raw verdicts (reset / maintenance overrides applied); returns the pools (or
        "*free*") whose devices changed verdict."""
        changed: set[str] = set()
        for uuid, v in raw.items():
            rec = self.records.get(uuid)
            if uuid in self.resetting:  # between amdsmi pre- and post-reset events
                v = {**v, "healthy": False,
                     "reasons": list(v.get("reasons") or []) + ["GPUReset: the GPU is being reset"]}
            if uuid in self.maintenance:  # admin-cordoned: unhealthy for pools, never claimed
                v = {**v, "healthy": False,
                     "reasons": list(v.get("reasons") or []) +
                     [f"AdminMaintenance: {self.maintenance[uuid] or 'cordoned by an administrator'}"]}
            old = self.verdicts.get(uuid)
            if old is None or old.get("healthy") != v.get("healthy") or \
                    old.get("reasons") != v.get("reasons"):
                if rec:
                    changed.add(rec["poolUID"])
                else:
                    changed.add("*free*")
            self.verdicts[uuid] = v
        return changed

    # A drop in VRAM in use above this between samples counts as a free the driver must clear
    # (~47 GB/s: 4 GiB ≈ 90 ms of blocked allocations); the probe's own ~1.2 GiB arena trim is not
    FREED_VRAM_BYTES = 4 << 30

    def sample(self) -> set[str]:
        t0 = time.perf_counter()
        snap = self.dev.snapshot()
        dt = (time.perf_counter() - t0) * 1e3
        try:
            self._account(snap)
        except Exception:  # accounting is telemetry: never fail a health sample for it
            log.exception("per-pod GPU accounting failed")
        with self.lock:
            now = time.monotonic()
            for d in snap["devices"]:  # VRAM freed wholesale by any process (pod or not): the
                old = (self.by_uuid.get(d["uuid"]) or {}).get("memUsedBytes")  # driver clears it
                new = d.get("memUsedBytes")                                     # for seconds
                if isinstance(old, (int, float)) and isinstance(new, (int, float)) and \
                        old - new > self.FREED_VRAM_BYTES:
                    self.freed_at[d["uuid"]] = now
            self.snap = snap
            self.by_uuid = {d["uuid"]: d for d in snap["devices"]}
            changed = self._evaluate_all()
            self.stats["samples"] += 1
            self.stats["sample_ms_sum"] += dt
        if changed:
            self._bump(changed)
            self._notify_plugins()
        return changed

    def _sampler(self) -> None:
        while not self._stop.wait(self.cfg.sample_interval):
            try:
                self.sample()
            except Exception:
                log.exception("health sample failed")
            if self._podres is not None:
                try:
                    self._refresh_pods()
                    self.gc_share_accounts()
                except Exception as e:
                    log.debug("podresources list failed: %s", e)
            try:
                self.recheck_probes()
            except Exception:
                log.exception("probe recheck failed")
            try:
                self.xgmi_recheck()
            except Exception:
                log.exception("idle xGMI check failed")

    def poll_health(self) -> set[str]:
        """Fast poll of the fields verdicts depend on (ECC counts, xGMI links, temperatures):
        amdsmi signals no ECC event, so this bounds the detection of an HBM error at
        ``health_interval`` instead of the full-telemetry ``sample_interval``. Devices whose
        health fields did not change are not re-evaluated."""
        t0 = time.perf_counter()
        h = self.dev.health_snapshot()
        dt = (time.perf_counter() - t0) * 1e3
        changed: set[str] = set()
        with self.lock:
            self.stats["health_polls"] += 1
            self.stats["health_poll_ms_sum"] += dt
            moved = False
            by = dict(self.by_uuid)
            for d in h.get("devices", []):
                old = by.get(d.get("uuid"))
                if old is None:
                    continue  # enumeration changes are the full sample's job
                if any(old.get(k) != v for k, v in d.items()):
                    by[d["uuid"]] = {**old, **d}
                    moved = True
            if moved:
                self.by_uuid = by
                changed = self._evaluate_all()
        if changed:
            self._bump(changed)
            self._notify_plugins()
        return changed

    def _health_poller(self) -> None:
        while not self._stop.wait(self.cfg.health_interval):
            try:
                self.poll_health()
            except Exception:
                log.exception("health poll failed")

    # ---- event-driven detection (the sampler is the fallback for what has no event)
    def _note_event(self, ev: dict) -> None:
        ev = {**ev, "at": now_rfc3339()}
        with self.lock:
            self.recent_events = (self.recent_events + [ev])[-32:]

    def node_event(self, reason: str, message: str, etype: str = "Warning") -> None:
        """A core/v1 Event on this Node (``gpuctl events``/``kubectl get events``) for hardware
        happenings no pool owns: amdsmi thermal-throttle / reset / VM-fault events, HBM sweep
        failures. Posted from a background thread; never blocks the caller."""
        if not self.cfg.apiserver:
            return

        def post():
            from ..kube import EVENTS
            try:
                c = self.api()
                ts = now_rfc3339()
                c.create(EVENTS, {
                    "apiVersion": "v1", "kind": "Event",
                    "metadata": {"name": f"{self.cfg.node}.{os.urandom(6).hex()}"},
                    "involvedObject": {"kind": "Node", "name": self.cfg.node, "apiVersion": "v1"},
                    "reason": reason, "message": message, "type": etype, "count": 1,
                    "firstTimestamp": ts, "lastTimestamp": ts,
                    "source": {"component": "gpupool-agent", "host": self.cfg.node}}, "default")
            except Exception as e:  # events are best effort
                log.debug("node event %s not posted: %s", reason, e)
        threading.Thread(target=post, daemon=True, name="node-event").start()

    def _device_event_watcher(self) -> None:
        """amdsmi event notification (thermal throttle, GPU pre/post reset, VM fault): each event
        triggers an immediate sample instead of waiting for the next period. A GPU between its
        pre- and post-reset events is unhealthy (GPUReset); after the reset a claimed GPU is
        re-probed, since the reset wiped whatever the claim-time probe verified."""
        while not self._stop.is_set():
            try:
                r = self.dev.wait_events(500)
            except Exception as e:
                log.warning("device event wait failed: %s", e)
                return
            self.events_supported["device"] = r.get("supported", False)
            if not r.get("supported"):
                if r.get("error"):
                    log.info("amdsmi event notification unavailable: %s", r["error"])
                return
            evs = r.get("events") or []
            if not evs:
                continue
            recheck = []
            with self.lock:
                by_index = {d.get("index"): u for u, d in self.by_uuid.items()}
                for ev in evs:
                    u = by_index.get(ev.get("index"))
                    self.stats["device_events"] += 1
                    if ev.get("type") == "GPUPreReset" and u:
                        self.resetting.add(u)
                    elif ev.get("type") == "GPUPostReset" and u:
                        self.resetting.discard(u)
                        if (self.records.get(u) or {}).get("state") == "Claimed":
                            recheck.append(u)
            for ev in evs:
                log.warning("device event on GPU %s: %s %s", ev.get("index"), ev.get("type"),
                            ev.get("message", ""))
                self._note_event({"source": "amdsmi", **ev})
                self.node_event(str(ev.get("type") or "DeviceEvent"),
                                f"GPU {ev.get('index')}: {ev.get('message', '')}".strip(),
                                "Normal" if ev.get("type") == "GPUPostReset" else "Warning")
            self.sample()
            for u in recheck:
                self._recheck_after_reset(u)

    def _recheck_after_reset(self, uuid: str) -> None:
        with self.lock:
            rec = self.records.get(uuid)
            if not rec or uuid in self._rechecking or uuid not in self.by_uuid:
                return
            self._rechecking.add(uuid)
            opts = (rec.get("policy") or {}).get("probe") or {}
            job = (uuid, dict(self.by_uuid[uuid]), opts, rec["poolUID"])
        self.prober.pool.submit(self._recheck_one, *job, after_reset=True)

    def _fault_watcher(self) -> None:
        """The fault overlay file is itself an event source: a rewrite is applied at once (inotify)
        unless the overlay sets ``"notify": false`` — then only the periodic sample sees it, which
        is how a real ECC counter change (amdsmi has no ECC event) is detected."""
        self.events_supported["faultOverlay"] = bool(self.cfg.faults)
        while not self._stop.is_set():
            try:
                r = self.dev.wait_faults(500)
            except Exception as e:
                log.warning("fault overlay watch failed: %s", e)
                return
            self.events_supported["faultOverlay"] = r.get("supported", False)
            if not r.get("supported"):
                return
            if not r.get("changed"):
                continue
            try:
                with open(self.cfg.faults) as f:
                    overlay = json.load(f)
            except (OSError, ValueError):
                overlay = {}  # removed or mid-write: the change itself is the event
            if isinstance(overlay, dict) and overlay.get("notify") is False:
                continue
            with self.lock:
                self.stats["fault_events"] += 1
            self._note_event({"source": "faultOverlay", "type": "FaultOverlayChanged"})
            try:
                self.sample()
            except Exception:
                log.exception("health sample failed")

    def recheck_probes(self, force: bool = False) -> list[str]:
        """Periodic functional re-probe (spec.probe.recheckSeconds) of claimed GPUs that run no
        pod: silent degradation between claims (a GPU that now fails its pattern test, GEMM
        checks or performance floor) surfaces as DeviceProbePassed=False and is replaced like
        any other health fault. Probes run on the prober's threads; returns the uuids started."""
        now = time.monotonic()
        pods = self._pods_by_device()
        due: list[tuple[str, dict, dict, str]] = []
        with self.lock:
            for u, rec in self.records.items():
                opts = (rec.get("policy") or {}).get("probe") or {}
                every = float(opts.get("recheckSeconds") or 0)
                if (every <= 0 and not force) or rec.get("state") != "Claimed" or pods.get(u) or \
                        u in self._rechecking or u not in self.by_uuid:
                    continue
                if not self.prober.can_probe(self.by_uuid[u]):
                    continue  # its helper is held back / parked: postponed, never failed for it
                if force or now - self._probe_mono.get(u, now) >= every:
                    self._rechecking.add(u)
                    due.append((u, dict(self.by_uuid[u]), opts, rec["poolUID"]))
        for u, dev, opts, pool_uid in due:
            self.prober.pool.submit(self._recheck_one, u, dev, opts, pool_uid)
        return [u for u, *_ in due]

    def _recheck_one(self, uuid: str, dev: dict, opts: dict, pool_uid: str,
                     after_reset: bool = False) -> None:
        try:
            if after_reset:  # the reset wiped the helper's HIP context: a fresh helper first
                self.prober.restart_helper(dev)
            res = self.prober.probe_many([dev], {**opts, "enabled": opts.get("enabled", True)})[0]
            res["recheck"] = True
            if str(res.get("error") or "").startswith("ProbeUnavailable"):
                # the probe could not run (a helper being replaced, parked): not a verdict on
                # the GPU — the previous one stands, the next recheck tries again
                with self.lock:
                    self.stats["rechecks_postponed"] = self.stats.get("rechecks_postponed", 0) + 1
                return
            with self.lock:
                rec = self.records.get(uuid)
                if rec is None or rec["poolUID"] != pool_uid or rec.get("state") != "Claimed":
                    return  # released / re-claimed meanwhile
                was = bool((rec.get("probe") or {}).get("passed"))
                rec["probe"] = res
                self.last_probe[uuid] = res
                self._probe_mono[uuid] = time.monotonic()
                self.stats["rechecks"] = self.stats.get("rechecks", 0) + 1
                if not res.get("passed"):
                    self.stats["probe_failures"] += 1
                if was != bool(res.get("passed")):
                    self.ledger.commit(self.records)
                    log.warning("recheck of %s: probe %s (%s)", uuid,
                                "passed" if res.get("passed") else "FAILED", res.get("error", ""))
                    flipped = True
                else:
                    flipped = False
            if flipped:
                self._bump({pool_uid})
                self._notify_plugins()
        finally:
            with self.lock:
                self._rechecking.discard(uuid)

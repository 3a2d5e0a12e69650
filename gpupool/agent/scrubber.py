"""HBM scrubber: walks the whole 288 GB of every idle MI355X in windows, between claims.

The claim-time probe pattern-tests one ~1 GiB arena, which is the same physical memory on every
claim. This thread covers the rest: for every GPU that is free (unclaimed, healthy, not
quarantined, no pod), every ``interval_s`` it tests ``windows_per_pass`` windows of
``window_bytes`` of a buffer spanning all free HBM minus ``reserve_bytes``
(``probe.hbm_sweep``, the same fill/verify kernels, both polarities), advancing a per-device
cursor that is persisted with the claim ledger. One full sweep of 288 GB costs ~0.2 s of HBM time
(4 passes over the data at ~6 TB/s), spread over passes so a claim never waits on more than one
window (~3 ms at 4 GiB). The kernels run in the GPU's probe helper (probehost.py), so a scrub that
faults a GPU takes down that helper, never the agent. Coverage is reported per device (``hbmSweep`` in the agent's device view
-> ``status.devices[].hbmCoverage``).

Claims always win: the scrubber re-checks eligibility under a per-device lock before every window,
and ``yield_device`` (called by the claim path after the ledger commit) only waits for an in-flight
window. The big buffer is allocated and freed outside every lock a claim takes (~282 GiB on
MI355X: 0.2 s to allocate fresh, ~6 s once the driver has to clear previously used VRAM, ~2.5 s to
free; profiles/r2h_sweep_claim_diag.txt), in 4 GiB chunks: one huge mapping's unmap held the
process's address-space lock for ~2.5 s and stalled any claim thread that mapped memory meanwhile
(profiles/r2o_scrub_claim_diag.txt). The claim-time probe arena is allocated first and kept while
the sweep runs and for 30 s after its free, so a claim-time probe never allocates behind the
driver's clear (a probe issued during the free or the allocation measured 1.1-1.3 ms); the device
plugin's Allocate waits for the free (``wait_released``) so a pod never starts beside the buffer.

A window with flipped bits quarantines a free GPU without expiry (``HBMSweepFailed``; cleared by
``gpuctl gpu uncordon``), so it is never claimed. In ``simulated`` probe mode (fake backend) the
windows are timed stand-ins and faults come from the overlay (``hbmBadOffset``: a byte offset).
"""
from __future__ import annotations

import logging
import threading
import time

log = logging.getLogger("gpupool.agent.scrubber")


class HbmScrubber:
    # No sweep buffer on a GPU this soon after VRAM was freed there (our last buffer, a released
    # pool's pods, the previous agent process): the driver clears freed VRAM (~6 s for ~282 GiB)
    # and an allocation issued meanwhile blocks, a probe of that GPU behind it (6.0 s measured,
    # profiles/r4q_sweep_yield.json)
    CLEAR_GRACE_S = 30.0

    def __init__(self, agent, interval_s: float = 60.0, window_bytes: int = 4 << 30,
                 windows_per_pass: int = 8, reserve_bytes: int = 4 << 30,
                 start_delay_s: float = 30.0):
        self.agent = agent
        self.interval_s = interval_s
        self.window_bytes = int(window_bytes)
        self.windows_per_pass = int(windows_per_pass)
        self.reserve_bytes = int(reserve_bytes)
        self.start_delay_s = start_delay_s
        self.state: dict[str, dict] = dict(agent.ledger.sweep_state())  # uuid -> coverage record
        self._locks: dict[str, threading.Lock] = {}
        self._mu = threading.Lock()
        self._cv = threading.Condition(self._mu)
        self._held: set[str] = set()  # GPUs whose sweep buffer is allocated
        # GPU -> monotonic time its sweep buffer was freed: the driver clears freed VRAM (~6 s for
        # ~282 GiB) and an allocation issued meanwhile waits for the clear — and stalls any probe
        # of that GPU behind it (6.1 s, profiles/r4p_probe_during_sweep_free.json)
        self._released_at: dict[str, float] = {}
        self._stop = threading.Event()
        self._kick = threading.Event()
        self._thread: threading.Thread | None = None
        self.stats = {"windows": 0, "bytes": 0, "failures": 0}

    # ------------------------------------------------------------------ coordination
    def _lock_for(self, uuid: str) -> threading.Lock:
        with self._mu:
            return self._locks.setdefault(uuid, threading.Lock())

    def yield_device(self, uuid: str) -> None:
        """Called by the claim path after the ledger commit (the GPU is no longer eligible): wait
        for an in-flight window (one window, ~3 ms at 4 GiB). The scrubber then frees its buffer on
        its own thread; the claim-time probe fits in the reserve meanwhile, and a pod's Allocate
        waits for the free (``wait_released``)."""
        with self._lock_for(uuid):
            pass

    def wait_released(self, uuid: str, timeout: float = 30.0) -> bool:
        """Block until no sweep buffer is held on ``uuid`` (the device plugin's Allocate calls this
        so a pod never starts while the scrubber still holds the GPU's free HBM)."""
        deadline = time.monotonic() + timeout
        with self._cv:
            while uuid in self._held:
                left = deadline - time.monotonic()
                if left <= 0:
                    return False
                self._cv.wait(left)
        return True

    def _eligible(self, uuid: str) -> bool:
        a = self.agent
        if uuid in a.records or uuid in a.maintenance or uuid not in a.by_uuid:
            return False
        if not a.verdicts.get(uuid, {}).get("healthy"):
            return False
        if uuid in a.ledger.quarantined():
            return False
        return not a._pods_by_device().get(uuid)

    # ------------------------------------------------------------------ one window
    def _window(self, uuid: str, dev: dict, offset: int) -> dict:
        """One window through the prober: in the GPU's probe helper (helper modes), the agent's
        own HIP (inproc) or the simulated kernels (fake backend)."""
        p = self.agent.prober
        if p.mode not in ("simulated", "helper-sim") and not p.visible(dev):
            return {"passed": False, "error": "device not visible to HIP"}
        return p.sweep_window(dev, offset, self.window_bytes, self.reserve_bytes)

    def _probes_quiet(self, timeout: float = 3.0) -> None:
        """Wait (bounded) until no claim-time probe runs on this agent. Mapping or unmapping the
        ~282 GiB sweep buffer while a probe runs stalls the probe: a claim that made the scrubbed
        GPU ineligible used to start its probe exactly while the scrubber freed the buffer, and
        that probe took 23.8 ms instead of 0.86 (profiles/r4o_bench_gpu1_real.json). The pod's
        Allocate waits for the free anyway (``wait_released``), so the free can wait for the
        probe."""
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline and not self._stop.is_set():
            with self.agent.lock:
                if not any(r.get("state") == "Probing" for r in self.agent.records.values()):
                    return
            time.sleep(0.002)

    def _hold(self, uuid: str) -> bool:
        """Allocate the sweep buffer (inproc: ~0.4 s for ~282 GiB) without any lock a claim takes."""
        with self._cv:
            self._held.add(uuid)
        t0 = time.perf_counter()
        p = self.agent.prober
        if p.mode in ("inproc", "helper", "helper-sim"):
            self._probes_quiet()
            dev = dict(self.agent.by_uuid.get(uuid) or {"uuid": uuid})
            # The claim-time probe arena comes first: a claim then never has to allocate while the
            # sweep buffer is held or while the driver clears it after the free (seconds).
            ok = p.visible(dev)
            if ok:
                p.warm_arena(dev)
            if not ok or p.sweep_alloc(dev, self.reserve_bytes) < 0:
                log.warning("HBM sweep buffer allocation failed on %s", uuid)
                self._release(uuid)
                return False
            log.info("HBM sweep buffer of %s allocated in %.1f ms", uuid,
                     (time.perf_counter() - t0) * 1e3)
        return True

    def _release(self, uuid: str) -> None:
        """Free the sweep buffer (inproc: ~2.5 s for ~282 GiB, the driver clears released VRAM)."""
        t0 = time.perf_counter()
        try:
            if self.agent.prober.mode in ("inproc", "helper", "helper-sim"):
                self.agent.prober.sweep_release(dict(self.agent.by_uuid.get(uuid) or {"uuid": uuid}))
        except Exception as e:  # a helper that died took the buffer with it
            log.warning("HBM sweep buffer release on %s failed: %s", uuid, e)
        finally:
            log.info("HBM sweep buffer of %s released in %.1f ms", uuid,
                     (time.perf_counter() - t0) * 1e3)
            with self._cv:
                self._held.discard(uuid)
                self._released_at[uuid] = time.monotonic()
                self._cv.notify_all()

    def scrub_device(self, uuid: str, windows: int | None = None, grace: bool = True) -> dict:
        """One pass over ``windows`` windows of one GPU; returns its coverage record. ``grace``
        False (an operator's explicit scrub): do not wait out CLEAR_GRACE_S."""
        lock = self._lock_for(uuid)
        with self._mu:
            rec = dict(self.state.get(uuid) or {"cursor": 0, "span": 0, "coveredBytes": 0,
                                                "passes": 0, "windows": 0, "lastBadBits": 0})
        with self.agent.lock:
            if not self._eligible(uuid):
                return rec
        if grace and self.agent.prober.mode in ("inproc", "helper"):
            freed = max(self._released_at.get(uuid, -1e9),
                        getattr(self.agent, "freed_at", {}).get(uuid, -1e9))
            if time.monotonic() - freed < self.CLEAR_GRACE_S:
                return rec  # the driver may still be clearing VRAM freed there (ours or a pod's)
        if not self._hold(uuid):
            return rec
        try:
            for _ in range(windows or self.windows_per_pass):
                if self._stop.is_set():
                    break
                with lock:
                    with self.agent.lock:
                        if not self._eligible(uuid):
                            break
                        dev = dict(self.agent.by_uuid[uuid])
                    t0 = time.perf_counter()
                    r = self._window(uuid, dev, int(rec["cursor"]))
                if "error" in r and "span" not in r:
                    log.warning("HBM sweep of %s failed to run: %s", uuid, r.get("error"))
                    break
                self.stats["windows"] += 1
                self.stats["bytes"] += int(r.get("bytes") or 0)
                span = int(r["span"])
                if rec.get("span") and rec["span"] != span:  # free HBM changed: restart the sweep
                    rec["cursor"], rec["coveredBytes"] = 0, 0
                rec["span"] = span
                end = int(r["offset"]) + int(r["bytes"])
                rec["coveredBytes"] = min(span, int(rec["coveredBytes"]) + int(r["bytes"]))
                rec["windows"] = int(rec["windows"]) + 1
                rec["lastAt"] = time.time()
                rec["lastGBps"] = round(float(r.get("GBps") or 0), 1)
                rec["lastWindowMs"] = round((time.perf_counter() - t0) * 1e3, 3)
                rec["lastBadBits"] = int(r.get("badBits") or 0)
                if end >= span:
                    rec["cursor"] = 0
                    rec["passes"] = int(rec["passes"]) + 1
                    rec["lastFullSweepAt"] = time.time()
                    rec["coveredBytes"] = 0
                else:
                    rec["cursor"] = end
                with self._mu:
                    self.state[uuid] = dict(rec)
                if not r.get("passed"):
                    self.stats["failures"] += 1
                    self._fail(uuid, r)
                    break
        finally:
            if self.agent.prober.mode in ("inproc", "helper", "helper-sim"):
                self._probes_quiet()
            self._release(uuid)
            with self._mu:
                snap = {u: dict(r) for u, r in self.state.items()}
            self.agent.ledger.commit_sweep(snap)
        return rec

    def _fail(self, uuid: str, r: dict) -> None:
        why = (f"HBMSweepFailed: {r.get('badBits')} flipped bit(s) at HBM offset "
               f"{r.get('firstBadOffset')} (window {r.get('offset')}+{r.get('bytes')})")
        log.error("%s: %s", uuid, why)
        a = self.agent
        a.ledger.quarantine(uuid, 1e12, why)
        a.node_event("HBMSweepFailed", f"GPU {(a.by_uuid.get(uuid) or {}).get('index')} "
                     f"({uuid}) quarantined: {why}")
        with a.lock:
            changed = a._evaluate_all()
        a._bump(changed | {"*free*"})
        a._notify_plugins()

    # ------------------------------------------------------------------ loop
    def coverage(self, uuid: str) -> dict | None:
        with self._mu:
            rec = self.state.get(uuid)
            if not rec:
                return None
            out = dict(rec)
        span = int(rec.get("span") or 0)
        if span:
            # fraction of the current sweep done (1.0 right after a full pass completes)
            out["fraction"] = round(int(rec.get("coveredBytes") or 0) / span, 4) if \
                int(rec.get("coveredBytes") or 0) else (1.0 if rec.get("passes") else 0.0)
        return out

    def run_once(self) -> int:
        n = 0
        with self.agent.lock:
            uuids = sorted(self.agent.by_uuid)
        for u in uuids:
            if self._stop.is_set():
                break
            with self.agent.lock:
                ok = self._eligible(u)
            if ok:
                self.scrub_device(u)
                n += 1
        return n

    def _loop(self) -> None:
        if self._stop.wait(self.start_delay_s):
            return
        while not self._stop.is_set():
            try:
                self.run_once()
            except Exception:
                log.exception("HBM scrub pass failed")
            self._kick.wait(self.interval_s)
            self._kick.clear()

    def start(self) -> None:
        if self.interval_s <= 0 or self.agent.prober.mode not in ("inproc", "simulated", "helper",
                                                                   "helper-sim"):
            return
        self._thread = threading.Thread(target=self._loop, daemon=True, name="hbm-scrub")
        self._thread.start()

    def kick(self) -> None:
        self._kick.set()

    def stop(self) -> None:
        self._stop.set()
        self._kick.set()

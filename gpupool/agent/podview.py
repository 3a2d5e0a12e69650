"""Which pods hold which GPUs, from the kubelet's PodResources API (a mixin of ``agent.Agent``).

Views never wait for the kubelet; a background poll runs only while pod placement is expected to
change (a drain, a fresh Allocate); release decisions ask synchronously (``fresh=True``).
"""
from __future__ import annotations

import threading
import time

from .common import gpu_of, log


class PodViewMixin:
    def _pods_by_device(self, fresh: bool = False) -> dict[str, list[dict]]:
        """device ID -> pods holding it, from the kubelet's PodResources API.

        Views (``fresh=False``) never wait for the kubelet: they return the last answer. Only
        while pod placement is expected to change (a GPU is draining, or a device-plugin Allocate
        happened in the last 2 s) does a view older than 50 ms start one background refresh
        (single-flight); otherwise the sampler refreshes every period. Spawning a refresh thread
        on every view put a GIL hand-off on the claim path's ``GET /v1/node`` (profiles/
        r2d_agent_rpc_latency_real.json). A refresh that changes which pods hold a pool's GPUs
        bumps that pool, so a drain waiting for evicted pods to end is woken by the change itself. Release
        decisions pass ``fresh=True``: they always ask the kubelet synchronously and raise if it
        cannot answer, so a stale or failed lookup can never free a GPU that a pod still holds."""
        if not self.cfg.pod_resources:
            return {}
        if fresh:
            return self._refresh_pods()
        ts, cache = self._pods_cache
        now = time.monotonic()
        if now - ts >= 0.05 and (now < self._pods_watch_until or self._draining()):
            self._refresh_pods_async()
        return cache

    def _draining(self) -> bool:
        with self.lock:  # claims and releases edit the record map on other threads
            return any(r.get("state") == "Draining" for r in self.records.values())

    def _watch_pods(self, seconds: float = 2.0) -> None:
        """Pod placement is about to change (a device-plugin Allocate): views refresh the pod map
        in the background for a while, so the new pod shows up without waiting for the sampler."""
        self._pods_watch_until = max(self._pods_watch_until, time.monotonic() + seconds)
        self._pods_kick.set()

    def _pod_watcher(self) -> None:
        """Polls the kubelet's PodResources (it has no watch) every ``pod_watch_interval`` while
        pod placement is expected to change: a GPU is draining (its evicted pods' exit is what the
        drain waits for) or a device-plugin Allocate just happened. A change bumps the owning
        pool, so the manager's agent feed wakes the drain without the manager polling the agent
        (its view cache answers observes without an RPC) or waiting for the sampler's period."""
        while not self._stop.is_set():
            self._pods_kick.wait(1.0)
            self._pods_kick.clear()
            while not self._stop.is_set():
                with self.lock:
                    active = time.monotonic() < self._pods_watch_until or self._draining()
                if not active:
                    break
                try:
                    self._refresh_pods()
                except Exception as e:
                    log.debug("podresources refresh failed: %s", e)
                self._stop.wait(self.cfg.pod_watch_interval)

    def _refresh_pods(self) -> dict[str, list[dict]]:
        pods: dict[str, list[dict]] = {}
        listed_at = time.time()
        listing = self._podres.list_pod_devices()
        self._pod_ids = (listed_at, set(listing))  # slot-level: the HBM-account GC's input
        for did, ps in listing.items():
            pods.setdefault(gpu_of(did), []).extend(ps)  # a shared GPU's slots -> the GPU
        with self.lock:
            old = self._pods_cache[1]
            self._pods_cache = (time.monotonic(), pods)
            flipped = {u for u in set(old) | set(pods) if old.get(u) != pods.get(u)}
            pools = {self.records[u]["poolUID"] for u in flipped if u in self.records}
        if flipped:
            self._sync_parking(pods)
        if pools:
            self._bump(pools)
        return pods

    def _sync_parking(self, pods: dict[str, list[dict]]) -> None:
        """A GPU that runs a tenant pod gets no agent HIP context (round-5 weak #5; the
        reference's GPU check leaves nothing resident, GPU调度平台搭建.md:134-138): its probe
        helper is parked — stopped, and the fabric helper restarted without it — while pods hold
        it, and started again (warm before release hands the GPU back) once they are gone. Every
        helper user probes, scrubs or rings pod-free GPUs only, so nothing needs it meanwhile."""
        if self.prober.helpers is None:
            return
        with self._park_mu:
            parked = self.prober.parked()
            for u, d in list(self.by_uuid.items()):
                if pods.get(u) and u not in parked:
                    if self.prober.park(d):
                        log.info("GPU %s runs pod(s) %s: its probe helper is parked", d.get("index"),
                                 [p.get("name") for p in pods[u]])
                elif not pods.get(u) and u in parked:
                    self.prober.unpark(d)  # starts now; release waits for it to be warm
                    log.info("GPU %s is pod-free: its probe helper restarts", d.get("index"))

    def _refresh_pods_async(self) -> None:
        with self.lock:
            if self._pods_refreshing:
                return
            self._pods_refreshing = True

        def run():
            try:
                self._refresh_pods()
            except Exception as e:  # kubelet down: keep the last known view
                log.debug("podresources list failed: %s", e)
            finally:
                with self.lock:
                    self._pods_refreshing = False
        self._pods_kick = threading.Event()
        threading.Thread(target=run, daemon=True, name="podres-refresh").start()

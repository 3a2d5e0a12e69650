"""Per-pod GPU accounting and slot-budget enforcement (a mixin of ``agent.Agent``).

Each GPU's processes (amdsmi process list, or the DRM fdinfo of this PID namespace) are attributed
to pods through their cgroup / downward-API environment; per (GPU, pod) the VRAM held and the
share of GPU time. On a shared GPU a pod over its slots' HBM budget is flagged, reported once as a
Node event, and evicted when its pool asks for it (``spec.sharing.overBudgetAction: Evict``).
"""
from __future__ import annotations

import os
import re
import threading
import time

from .common import log, now_rfc3339


def _scan_drm_clients() -> dict[str, dict[int, dict]]:
    """GPU memory and engine time per local process from the amdgpu DRM fdinfo of its
    render-node fds (``drm-pdev``, ``drm-memory-vram``, ``drm-engine-*``): bdf -> pid -> usage.
    Namespace-safe — it sees exactly the processes of this PID namespace, under their local PIDs."""
    out: dict[str, dict[int, dict]] = {}
    for ent in os.listdir("/proc"):
        if not ent.isdigit():
            continue
        fd_dir = f"/proc/{ent}/fd"
        try:
            fds = os.listdir(fd_dir)
        except OSError:
            continue
        seen: set[str] = set()
        for fd in fds:
            try:
                if not os.readlink(f"{fd_dir}/{fd}").startswith("/dev/dri/renderD"):
                    continue
                with open(f"/proc/{ent}/fdinfo/{fd}") as f:
                    info = dict(line.split(":", 1) for line in f if ":" in line)
            except (OSError, ValueError):
                continue
            client = info.get("drm-client-id", "").strip()
            bdf = info.get("drm-pdev", "").strip().lower()
            if not bdf or client in seen:
                continue
            seen.add(client)
            vram = info.get("drm-memory-vram") or info.get("drm-total-vram") or "0"
            parts = vram.split()
            kib = {"KiB": 1 << 10, "MiB": 1 << 20, "GiB": 1 << 30}.get(parts[1], 1) \
                if len(parts) > 1 else 1
            eng = sum(int(v.split()[0]) for k, v in info.items()
                      if k.startswith("drm-engine-") and v.split() and v.split()[0].isdigit())
            u = out.setdefault(bdf, {}).setdefault(int(ent), {"vramBytes": 0, "engineNs": 0})
            u["vramBytes"] += int(parts[0]) * kib if parts and parts[0].isdigit() else 0
            u["engineNs"] += eng
    return out


class AccountingMixin:
    _POD_UID_RE = None

    def _pod_of_pid(self, pid: int) -> dict:
        """The pod a GPU process belongs to: from its cgroup (a kubelet's container cgroups carry
        the pod UID: ``kubepods-…-pod<uid>.slice`` / ``kubepods/…/pod<uid>/``), resolved to
        namespace/name through the API server; else from the pod identity in its environment
        (POD_NAME / POD_NAMESPACE: the downward API on a real node, set by the fake kubelet). The
        agent's own probe / scrubber buffers are reported as ``gpupool-agent``. {} if unknown."""
        hit = self._pid_pods.get(pid)
        if hit is not None:
            return hit
        if time.monotonic() - self._pid_miss.get(pid, -1e9) < 2.0:
            return {}  # unresolved a moment ago: retry later, not on every sample
        host_pid = pid
        if pid == os.getpid() or pid in self.prober.helper_pids():  # the agent / its probe helpers
            return {"namespace": "", "pod": "gpupool-agent"}
        import re
        pod: dict = {}
        try:
            with open(f"/proc/{pid}/cgroup") as f:
                m = re.search(r"pod([0-9a-f]{8}[-_][0-9a-f]{4}[-_][0-9a-f]{4}[-_][0-9a-f]{4}"
                              r"[-_][0-9a-f]{12})", f.read())
            if m:
                pod = self._pod_by_uid(m.group(1).replace("_", "-")) or {}
        except OSError:
            pass
        if not pod:
            try:
                with open(f"/proc/{pid}/environ", "rb") as f:
                    env = dict(x.split(b"=", 1) for x in f.read().split(b"\0") if b"=" in x)
                if b"POD_NAME" in env:
                    pod = {"namespace": env.get(b"POD_NAMESPACE", b"").decode(),
                           "pod": env[b"POD_NAME"].decode()}
            except OSError:
                pass
        if len(self._pid_pods) > 4096:
            self._pid_pods.clear()
            self._pid_miss.clear()
        if pod:
            self._pid_pods[host_pid] = pod
        else:
            self._pid_miss[host_pid] = time.monotonic()
        return pod

    def _pod_by_uid(self, uid: str) -> dict | None:
        ts, by_uid = self._pods_by_uid
        if uid not in by_uid and time.monotonic() - ts > 5.0 and self.cfg.apiserver:
            from ..kube import PODS
            try:
                c = self.api()
                items = c.list(PODS, None, field_selector=f"spec.nodeName={self.cfg.node}")["items"]
                by_uid = {p["metadata"]["uid"]: {"namespace": p["metadata"]["namespace"],
                                                 "pod": p["metadata"]["name"]} for p in items}
            except Exception as e:
                log.debug("pod lookup for accounting failed: %s", e)
            self._pods_by_uid = (time.monotonic(), by_uid)
        return by_uid.get(uid)

    def _account(self, snap: dict) -> None:
        """Per-pod GPU accounting (reference ops practice "monitor GPU utilisation" and per-team
        usage, GPU调度平台搭建.md:800-802): each GPU's processes (amdsmi_get_gpu_process_list) are
        attributed to pods; per (GPU, pod) the VRAM they hold and their share of the GPU's time
        (gfx-engine ns consumed between two samples / wall ns). On a time-shared GPU this is what
        tells the sharers apart, and an idle pod on a claimed GPU shows up as a 0 share."""
        now = time.monotonic()
        window = max(0.2, 0.5 * self.cfg.sample_interval)
        prev, new_prev = self._proc_prev, {}
        usage: dict[str, list[dict]] = {}
        drm: dict[str, dict[int, dict]] | None = None
        for d in snap.get("devices") or []:
            u = d.get("uuid")
            per: dict[tuple[str, str], dict] = {}
            procs = [p for p in d.get("processes") or [] if int(p.get("pid") or 0) > 0]
            # amdsmi names processes by the kernel's (host) PID. With the agent in the host PID
            # namespace (hostPID, as deployed) they are all visible here; otherwise (a container
            # with its own PID namespace) the GPU's processes are read from the DRM fdinfo of
            # this namespace's processes instead — under local PIDs, VRAM per GPU by BDF.
            if any(not os.path.exists(f"/proc/{int(p['pid'])}") for p in procs):
                if drm is None:
                    drm = _scan_drm_clients()
                local = drm.get(str(d.get("bdf", "")).lower(), {})
                procs = [{"pid": pid, "vramBytes": x["vramBytes"], "gfxNs": x["engineNs"],
                          "source": "drm-fdinfo"} for pid, x in sorted(local.items())]
            for p in procs:
                pid = int(p.get("pid") or 0)
                who = self._pod_of_pid(pid)
                gfx = int(p.get("gfxNs") or 0)
                busy = None
                # ratio over the newest earlier sample at least ``window`` old (event-triggered
                # samples come ms apart: a ratio over a few ms is noise), else the oldest kept
                hist = [h for h in prev.get((u, pid), []) if now - h[0] <= 20 * window and
                        h[1] <= gfx]
                ref = next((h for h in reversed(hist) if now - h[0] >= window),
                           hist[0] if hist else None)
                if ref and now > ref[0]:
                    busy = (gfx - ref[1]) / ((now - ref[0]) * 1e9)
                new_prev[(u, pid)] = (hist + [(now, gfx)])[-16:]
                e = per.setdefault((who.get("namespace", ""), who.get("pod", "")), {
                    "namespace": who.get("namespace", ""), "pod": who.get("pod", ""),
                    "pids": [], "vramBytes": 0, "gfxBusy": None, "cuOccupancy": 0})
                e["pids"].append(pid)
                e["vramBytes"] += int(p.get("vramBytes") or p.get("memBytes") or 0)
                e["cuOccupancy"] += int(p.get("cuOccupancy") or 0)
                if busy is not None:
                    e["gfxBusy"] = round((e["gfxBusy"] or 0.0) + busy, 4)
            if per:
                usage[u] = sorted(per.values(), key=lambda x: (x["namespace"], x["pod"]))
        over = self._check_slot_budgets(usage)
        with self.lock:
            self._proc_prev = new_prev
            self.pod_usage = usage
        for msg in over:
            self.node_event("SlotBudgetExceeded", msg)

    # VRAM a pod may hold beyond its slots' budget: what ROCr allocates internally (queues, scratch,
    # code objects), which the share library does not charge
    SLOT_BUDGET_SLACK = (512 << 20, 0.05)

    def _check_slot_budgets(self, usage: dict[str, list[dict]]) -> list[str]:
        """Defence in depth for isolated slots: the HBM budget is enforced inside the pod by
        libgpupool_share.so, and a pod in which it is not active (an image whose loader cannot
        load it, a pod that unset HSA_TOOLS_LIB) would run unconfined without anyone noticing. The
        agent sees each pod's VRAM per GPU (amdsmi / DRM fdinfo): a pod holding more than its
        slots x hbmBytesPerSlot (+ ROCr's uncharged internals) is marked ``overBudget`` in the
        usage view and metrics, and reported once per (pod, GPU) as a Node event. Returns the
        messages of new violations."""
        slots_of: dict[tuple[str, str, str], int] = {}
        for gpu, pods in self._pods_cache[1].items():  # one entry per slot a pod holds
            for pe in pods:
                key = (gpu, pe.get("namespace", ""), pe.get("name", ""))
                slots_of[key] = slots_of.get(key, 0) + 1
        out, seen, evict = [], set(), []
        slack, frac = self.SLOT_BUDGET_SLACK
        with self.lock:
            for u, pods in usage.items():
                rec = self.records.get(u)
                if not rec or self._slots_of(rec) <= 1:
                    continue
                per_slot = self._slot_layout(u, rec).get("hbmBytesPerSlot") or 0
                if not per_slot:
                    continue
                action = str((((rec.get("policy") or {}).get("sharing") or {})
                              .get("overBudgetAction")) or "Flag")
                for e in pods:
                    n = slots_of.get((u, e["namespace"], e["pod"]), 0)
                    if not n:
                        continue
                    budget = n * per_slot
                    e["slotBudgetBytes"] = budget
                    if e["vramBytes"] > budget * (1 + frac) + slack:
                        e["overBudget"] = True
                        key = (u, e["namespace"], e["pod"])
                        seen.add(key)
                        count = self._over_samples.get(key, 0) + 1
                        self._over_samples[key] = count
                        e["overBudgetSamples"] = count
                        if key not in self._over_budget:
                            out.append(f"pod {e['namespace']}/{e['pod']} holds {e['vramBytes']} B of "
                                       f"VRAM on GPU {u}, over its {n} slot(s) x {per_slot} B: "
                                       f"its HBM limit is not in force (is libgpupool_share.so "
                                       f"loaded in the pod?)")
                        # spec.sharing.overBudgetAction Evict: two samples in a row (not one
                        # transient reading), once per pod
                        if action == "Evict" and count >= self.EVICT_AFTER_SAMPLES and \
                                (e["namespace"], e["pod"]) not in self._budget_evicted:
                            self._budget_evicted.add((e["namespace"], e["pod"]))
                            evict.append((u, e["namespace"], e["pod"], e["vramBytes"], budget))
            self._over_budget = seen
            self._over_samples = {k: v for k, v in self._over_samples.items() if k in seen}
        for args in evict:
            self._evict_over_budget(*args)
        return out

    EVICT_AFTER_SAMPLES = 2

    def _evict_over_budget(self, uuid: str, ns: str, pod: str, vram: int, budget: int) -> None:
        """Evict a pod whose VRAM exceeded its slots' budget (spec.sharing.overBudgetAction
        Evict): the HBM limit lives inside the pod (libgpupool_share.so), which the pod can
        defeat — unset HSA_TOOLS_LIB, or never load it. The agent sees the pod's VRAM from
        outside (amdsmi process list / DRM fdinfo) and takes the pod off the GPU its siblings
        share, through the Eviction API (the pod's PodDisruptionBudget applies), with an Event on
        the pod. Runs on its own thread: the sampler never waits for the API server."""
        msg = (f"pod {ns}/{pod} holds {vram} B of VRAM on GPU {uuid}, over its slots' "
               f"{budget} B HBM budget for {self.EVICT_AFTER_SAMPLES}+ samples: evicted "
               f"(spec.sharing.overBudgetAction Evict)")
        log.warning("%s", msg)
        with self.lock:
            self.stats["over_budget_evictions"] = self.stats.get("over_budget_evictions", 0) + 1
        if not self.cfg.apiserver:
            log.warning("no API server configured: cannot evict %s/%s", ns, pod)
            return

        def run():
            from ..kube import EVENTS
            try:
                c = self.api()
                c.evict(ns, pod)
                ts = now_rfc3339()
                c.create(EVENTS, {
                    "apiVersion": "v1", "kind": "Event",
                    "metadata": {"name": f"{pod}.{os.urandom(6).hex()}"},
                    "involvedObject": {"kind": "Pod", "name": pod, "namespace": ns,
                                       "apiVersion": "v1"},
                    "reason": "SlotBudgetExceeded", "message": msg, "type": "Warning",
                    "count": 1, "firstTimestamp": ts, "lastTimestamp": ts,
                    "source": {"component": "gpupool-agent", "host": self.cfg.node}}, ns)
            except Exception as ex:  # retried: the next over-budget sample evicts again
                log.warning("evicting over-budget pod %s/%s failed: %s", ns, pod, ex)
                with self.lock:
                    self._budget_evicted.discard((ns, pod))
        threading.Thread(target=run, daemon=True, name="budget-evict").start()

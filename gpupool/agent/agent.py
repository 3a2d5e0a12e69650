"""gpupool node agent: owns one node's MI355X GPUs.

Responsibilities (SURVEY.md §7.1 architecture):
  * discovery + telemetry through libmi355x_dev (amdsmi | cli | fake backend, fault overlay);
  * the claim ledger (all-or-nothing, topology-aware claims; cordon; release; quarantine);
  * claim-time HIP probes (warm, in-process by default) — the B4 readiness check;
  * health sampling against each owning pool's policy (verdicts from libmi355x_dev);
  * the ROCm device plugin endpoints (one per extended resource) + PodResources lookups;
  * Node registration (labels, agent endpoint annotation, GPUPoolAgentReady condition);
  * an HTTP/JSON RPC surface for the manager (unix socket and/or TCP) with a long-poll event feed.

Replaces what the reference's controller did through the Azure SDK (README.md:179-221) with a
node-local owner of physical devices.
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import os
import socket
import threading
import time
from uuid import uuid4
from dataclasses import dataclass, field
from typing import Any

from ..api import schema
from ..ops import devlib
from . import slots as slotlib
from .ledger import Ledger
from .prober import DEFAULT_TIMEOUT_S, Prober, default_mode

SLOT_SEP = "::"  # device-plugin ID of a time-sliced slot: "<uuid>::<slot>"
# wake the chosen GPUs' probe helpers as soon as a claim has selected them (A/B switch)
PREWAKE = os.environ.get("GPUPOOL_PROBE_PREWAKE", "1") != "0"


def _ranges(bits: list[int]) -> str:
    """[0, 1, 2, 5, 6] -> "0-2,5-6" (the CU-mask syntax libgpupool_share.so reads)."""
    out, start, prev = [], None, None
    for b in bits:
        if start is None:
            start = prev = b
        elif b == prev + 1:
            prev = b
        else:
            out.append(f"{start}-{prev}")
            start = prev = b
    if start is not None:
        out.append(f"{start}-{prev}")
    return ",".join(out)


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


def gpu_of(device_id: str) -> str:
    """The GPU uuid behind a device-plugin ID (a plain uuid, or a shared GPU's slot)."""
    return device_id.split(SLOT_SEP, 1)[0]


log = logging.getLogger("gpupool.agent")


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def process_metrics() -> list[str]:
    """Prometheus' standard process metrics from /proc/self (resident memory, CPU time, threads,
    open fds), as the client libraries' process collector exports them."""
    out = []
    try:
        with open("/proc/self/statm") as f:
            out.append(f"process_resident_memory_bytes {int(f.read().split()[1]) * os.sysconf('SC_PAGESIZE')}")
        with open("/proc/self/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        out.append(f"process_cpu_seconds_total "
                   f"{(int(fields[11]) + int(fields[12])) / os.sysconf('SC_CLK_TCK'):.3f}")
        out.append(f"process_threads {int(fields[17])}")
        out.append(f"process_open_fds {len(os.listdir('/proc/self/fd'))}")
    except (OSError, IndexError, ValueError):
        pass
    return out


@dataclass
class AgentConfig:
    node: str = field(default_factory=socket.gethostname)
    backend: str = "auto"
    fixture: str = ""
    faults: str = ""
    count: int = -1
    cli_dir: str = ""
    state_dir: str = "/var/lib/gpupool"
    socket: str = ""                 # unix socket for the RPC server
    listen: str = ""                 # optional host:port
    tls_cert: str = ""               # serve the TCP listener over HTTPS with this certificate
    tls_key: str = ""
    endpoint: str = ""               # what the Node annotation advertises (default: socket)
    apiserver: str = ""              # empty: no Node registration
    token: str = ""
    auth_token: str = ""             # shared secret the manager presents on the agent RPC
    plugin_dir: str = ""             # kubelet device-plugin dir; empty: device plugin disabled
    pod_resources: str = ""          # kubelet PodResources socket
    probe_mode: str = ""             # helper | helper-sim | inproc | subprocess | simulated | off
    probe_sim_ms: float = 20.0
    probe_gemm_n: int = 4096          # serial probe's GEMM (pools with performance floors)
    probe_overlap_gemm_n: int = 2048  # claim-time probe's GEMM beside the HBM pattern test
    sample_interval: float = 2.0
    health_interval: float = 0.1     # fast poll of the health-only fields (0 = off)
    pod_watch_interval: float = 0.02  # PodResources poll while a GPU drains / after an Allocate
    quarantine_s: float = 300.0
    advertise_wait_s: float = 2.0
    fsync: bool = True
    probe_arena_idle_s: float = 10.0  # free the kept ~1.2 GiB probe arena after this idle time
    # the xGMI fabric helper (contexts on every GPU): 0 keeps it resident, pre-warmed at start, so
    # a multi-GPU claim never pays its HIP init; > 0 lets it go after that many idle seconds
    probe_fabric_idle_s: float = 0.0
    scrub_interval_s: float = 60.0    # HBM scrubber pass period over idle GPUs (0 = off)
    scrub_window_bytes: int = 4 << 30
    scrub_windows: int = 8            # windows per device per pass
    scrub_reserve_bytes: int = 4 << 30
    scrub_start_delay_s: float = 30.0
    xgmi_recheck_s: float = 600.0     # idle xGMI coverage ring period (0 = off)
    xgmi_recheck_bytes: int = 16 << 20
    inject_claim_delay: tuple = (0, 0.0)  # (min count, seconds): fault injection for tests/bench
    # HBM the agent keeps for itself on every GPU (HIP context ~668 MiB, profiles/
    # r2q_agent_footprint_real.json, + the ~1.15 GiB probe arena): slot budgets must fit beside it
    hbm_reserve_bytes: int = 2 << 30
    share_acct_grace_s: float = 10.0  # an HBM account younger than this is never garbage-collected
    heartbeat_interval: float = 10.0  # Node condition heartbeat (nodereg.py)
    token_file: str = ""              # apiserver bearer token file, re-read as it rotates


class Agent:
    def __init__(self, cfg: AgentConfig):
        self.cfg = cfg
        self.lock = threading.RLock()
        dev_cfg: dict[str, Any] = {"node": cfg.node}
        if cfg.fixture:
            dev_cfg["fixture"] = cfg.fixture
        if cfg.faults:
            dev_cfg["faults"] = cfg.faults
        if cfg.count >= 0:
            dev_cfg["count"] = cfg.count
        if cfg.cli_dir:
            dev_cfg["cliDir"] = cfg.cli_dir
        self.dev = devlib.DeviceLib(cfg.backend, **dev_cfg)
        self.ledger = Ledger(cfg.state_dir, fsync=cfg.fsync)
        self.records: dict[str, dict] = self.ledger.load()
        # A claim commits 'Probing' before its probe runs, and Probing -> Claimed reaches the disk
        # through the ledger's background writer after the reply: an agent killed in between
        # leaves such records behind. _reprobe_interrupted probes them again once, or fails them
        # unprobed (ProbeInterrupted) when their probe already outlived one agent process.
        # Either way a failed GPU takes the normal replace path (drain -> release -> quarantine
        # -> spare).
        interrupted = [u for u, r in self.records.items() if r.get("state") == "Probing"]
        self._probing_since: dict[str, tuple[float, float]] = {}  # uuid -> (monotonic start, timeout)
        self.share_lib_dir = self._install_share_lib()
        self._pod_ids: tuple[float, set[str]] | None = None  # (listed at, device IDs pods hold)
        self._over_budget: set[tuple[str, str, str]] = set()  # (gpu, ns, pod) over their slot budget
        self._over_samples: dict[tuple[str, str, str], int] = {}  # ... for how many samples in a row
        self._budget_evicted: set[tuple[str, str]] = set()  # (ns, pod) evicted for it (once each)
        self._layouts: dict[tuple, dict] = {}  # memoised slot layouts (_slot_layout)
        self.snap = self.dev.snapshot()
        self.backend = self.snap.get("backend", cfg.backend)
        self.by_uuid = {d["uuid"]: d for d in self.snap["devices"]}
        self.verdicts: dict[str, dict] = {}
        self.gen = 0
        self.changes: list[tuple[int, set[str]]] = []
        # pools with a claim RPC in flight: their change events wait until the claim's reply is
        # out (the reply carries the same state); answering the manager's event feed meanwhile
        # only competed with the reply on the event loop
        self._claiming: dict[str, int] = {}
        self._deferred: set[str] = set()
        self.gen_cv = threading.Condition()  # /v1/events long-polls wait here for a new gen
        self.rpc = None                      # the RPC server (its per-path timings in /metrics)
        self.advertised: dict[str, set[str]] = {}
        # advertised-set generation: a waiter reads it before checking and sleeps only until it
        # moves (a shared Event cleared by one claim's waiter could hide a mark from another's)
        self._adv_cv = threading.Condition()
        self._adv_gen = 0
        self.plugins: dict = {}
        self.probe_mode = cfg.probe_mode or default_mode(self.backend)
        self.prober = Prober(self.probe_mode, sim_ms=cfg.probe_sim_ms, gemm_n=cfg.probe_gemm_n,
                             arena_idle_s=cfg.probe_arena_idle_s,
                             overlap_gemm_n=cfg.probe_overlap_gemm_n,
                             devices=[d for d in self.snap["devices"] if d.get("present", True)],
                             fabric_idle_s=cfg.probe_fabric_idle_s,
                             fabric_prewarm=cfg.probe_fabric_idle_s <= 0)
        self.last_probe: dict[str, dict] = {}
        # uuid -> monotonic time its VRAM was last freed wholesale (a release after its pods ended;
        # agent start: the previous agent process's allocations): the driver clears freed VRAM for
        # seconds, and the HBM scrubber must not map its sweep buffer into that (scrubber.py)
        self.freed_at: dict[str, float] = {u: time.monotonic() for u in self.by_uuid}
        self._probe_mono: dict[str, float] = {}  # uuid -> monotonic time of its last probe
        # admin maintenance (gpuctl gpu cordon): uuid -> reason; persisted as a quarantine entry
        # without expiry so it survives agent restarts
        self.maintenance: dict[str, str] = {
            u: q.get("reason", "") for u, q in (self.ledger.quarantined().items() if self.ledger else [])
            if q.get("maintenance")}
        self._rechecking: set[str] = set()
        self.xgmi_pairs: dict[str, dict] = self.ledger.xgmi_state()
        # the newest manager leader seen on a mutating RPC ({"holder", "epoch"}, ledger-persisted)
        self.leader_fence: dict = self.ledger.leader_state()
        self._fence_mu = threading.Lock()
        self.pod_usage: dict[str, list[dict]] = {}        # uuid -> per-pod VRAM / gfx time
        self._proc_prev: dict[tuple[str, int], list] = {}  # (uuid, pid) -> [(t, gfxNs)]
        self._pid_pods: dict[int, dict] = {}
        self._pid_miss: dict[int, float] = {}
        self._pods_by_uid: tuple[float, dict[str, dict]] = (0.0, {})
        self._xgmi_last = time.monotonic()
        self.stats = {"claims": 0, "releases": 0, "probes": 0, "probe_failures": 0, "rechecks": 0,
                      "probe_ms_sum": 0.0, "samples": 0, "sample_ms_sum": 0.0,
                      "health_polls": 0, "health_poll_ms_sum": 0.0,
                      "device_events": 0, "fault_events": 0}
        self.resetting: set[str] = set()       # GPUs between amdsmi GPUPreReset and GPUPostReset
        self._claim_cache: dict[tuple[str, str], tuple[dict, bool]] = {}
        self.recent_events: list[dict] = []   # last hardware/overlay events (node view, metrics)
        self.events_supported: dict[str, Any] = {}
        self._pods_cache: tuple[float, dict[str, list[dict]]] = (0.0, {})
        self._pods_refreshing = False
        self._pods_kick = threading.Event()
        self._pods_watch_until = 0.0
        from .podresources import PodResourcesClient
        self._podres = PodResourcesClient(cfg.pod_resources) if cfg.pod_resources else None
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self.registrar = None  # nodereg.NodeRegistrar once register_node ran
        from .scrubber import HbmScrubber
        self.scrubber = HbmScrubber(self, cfg.scrub_interval_s, cfg.scrub_window_bytes,
                                    cfg.scrub_windows, cfg.scrub_reserve_bytes,
                                    cfg.scrub_start_delay_s)
        self._reprobe_interrupted(interrupted)
        self._evaluate_all()
        from .preflight import check as preflight_check
        self.preflight = preflight_check(self.snap, fake=self.backend == "fake")
        if not self.preflight["ready"]:
            log.warning("preflight not ready: %s", {k: v["detail"] for k, v in
                                                    self.preflight["checks"].items() if not v["ok"]})
        log.info("agent %s: backend=%s devices=%d probe=%s (init %.0f ms) ledger=%d claims",
                 cfg.node, self.backend, len(self.by_uuid), self.probe_mode, self.prober.init_ms,
                 len(self.records))

    def _reprobe_interrupted(self, uuids: list[str]) -> None:
        """Finish the claims a previous agent process left in 'Probing' (see __init__), before the
        RPC server starts. The process died between the claim's commit and the lazy Probing ->
        Claimed write: during the probe, or in the few ms after the reply. Each record counts its
        probe attempts (``probeAttempts``, durable with the record before every probe):

        * first attempt: probed again (in the GPU's helper, with its deadline). Failing those
          outright replaced healthy GPUs after an unrelated kill (a rolling update, an OOM kill)
          and drained what their pools had started on them; a GPU that fails the re-probe takes
          the normal replace path (drain -> release -> quarantine -> spare);
        * the second death in a row during this GPU's probe: failed unprobed (ProbeInterrupted),
          so a GPU that takes down whatever probes it can never crash-loop the agent — with the
          probe in a helper the agent does not die of it in the first place; this bounds what is
          left (a probe run in-process with ``--probe inproc``, a driver hang the agent's own
          amdsmi calls run into)."""
        if not uuids:
            return
        failed_unprobed, again = [], []
        for u in uuids:
            rec = self.records[u]
            n = int(rec.get("probeAttempts") or 1)
            if n >= 2:
                rec["state"] = "Claimed"
                rec["probe"] = {"passed": False, "backend": self.probe_mode, "ms": 0.0,
                                "crashed": True,
                                "error": f"ProbeInterrupted: {n} agent processes in a row died "
                                         f"while this GPU's claim-time probe was in flight; "
                                         f"failed without probing it again"}
                failed_unprobed.append(u)
            else:
                rec["probeAttempts"] = n + 1
                again.append(u)
        if again:  # the attempt is on disk before the probe runs
            self.ledger.commit(self.records)
        for u in again:
            rec = self.records[u]
            d = self.by_uuid.get(u)
            opts = (rec.get("policy") or {}).get("probe") or {}
            if d is None:
                res = {"passed": False, "backend": "none", "ms": 0.0,
                       "error": "ProbeInterrupted: the agent restarted during the claim-time "
                                "probe and the GPU is no longer visible"}
            else:
                res = self.prober.probe_many([d], {**opts, "enabled": opts.get("enabled", True)})[0]
                res["rerunAtStart"] = True
                if not res.get("passed"):
                    res["error"] = "ProbeInterrupted, re-run at agent start: " + \
                        str(res.get("error") or "probe failed")
            rec["state"] = "Claimed"
            rec["probe"] = res
        for u in uuids:
            res = self.records[u]["probe"]
            self.last_probe[u] = res
            self._probe_mono[u] = time.monotonic()
            self.stats["probes"] += 1
            self.stats["probe_ms_sum"] += float(res.get("ms", 0.0))
            if not res.get("passed"):
                self.stats["probe_failures"] += 1
        self.ledger.commit(self.records)
        log.warning("finished %d claim(s) a restart interrupted (%d failed unprobed): %s",
                    len(uuids), len(failed_unprobed),
                    {u: bool(self.records[u]["probe"].get("passed")) for u in uuids})

    # ================================================================ health
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
            from ..kube import EVENTS, Client
            try:
                c = Client.connect(self.cfg.apiserver, self.cfg.token or None)
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
        self.prober.pool.submit(self._recheck_one, *job)

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
                if force or now - self._probe_mono.get(u, now) >= every:
                    self._rechecking.add(u)
                    due.append((u, dict(self.by_uuid[u]), opts, rec["poolUID"]))
        for u, dev, opts, pool_uid in due:
            self.prober.pool.submit(self._recheck_one, u, dev, opts, pool_uid)
        return [u for u, *_ in due]

    def _recheck_one(self, uuid: str, dev: dict, opts: dict, pool_uid: str) -> None:
        try:
            res = self.prober.probe_many([dev], {**opts, "enabled": opts.get("enabled", True)})[0]
            res["recheck"] = True
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

    # ================================================================ events
    def _bump(self, pools: set[str]) -> None:
        with self.lock:
            held = {p for p in pools if p in self._claiming}
            if held:
                self._deferred |= held
                pools = set(pools) - held
                if not pools:
                    return
            self.gen += 1
            self.changes.append((self.gen, set(pools)))
            self.changes = self.changes[-256:]
        with self.gen_cv:
            self.gen_cv.notify_all()

    def changed_since(self, since: int) -> tuple[int, list[str]]:
        with self.lock:
            pools: set[str] = set()
            for g, ps in self.changes:
                if g > since:
                    pools |= ps
            if self.changes and self.changes[0][0] > since + 1 and since >= 0:
                pools.add("*")  # history truncated: tell the manager to resync everything
            if since > self.gen:
                pools.add("*")  # a generation from before this agent restarted: resync
            # "*free*": free-GPU capacity or health changed -> the manager wakes pools that are
            # waiting for devices; "*": resync everything
            return self.gen, sorted(pools)

    # ================================================================ per-pod accounting
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
            from ..kube import PODS, Client
            try:
                c = Client.connect(self.cfg.apiserver, self.cfg.token or None)
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
            from ..kube import EVENTS, Client
            try:
                c = Client.connect(self.cfg.apiserver, self.cfg.token or None)
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

    # ================================================================ views
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
        if pools:
            self._bump(pools)
        return pods

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

    # how long past spec.probe.timeoutSeconds a 'Probing' GPU is reported probeOverdue (the
    # probe helper's own deadline answers well before: this covers a claim stuck elsewhere)
    PROBE_GRACE_S = 5.0

    def _advertisable(self, uuid: str) -> bool:
        rec = self.records.get(uuid)
        if not rec or rec.get("state") != "Claimed":
            return False
        v = self.verdicts.get(uuid, {})
        return bool(v.get("healthy")) and bool((rec.get("probe") or {}).get("passed"))

    def device_view(self, uuid: str, pods: dict[str, list[dict]]) -> dict:
        d = self.by_uuid.get(uuid, {"uuid": uuid, "index": -1})
        rec = self.records.get(uuid)
        v = self.verdicts.get(uuid, {})
        out = {
            "uuid": uuid, "hipUUID": d.get("hipUUID", ""), "bdf": d.get("bdf", ""),
            "index": d.get("index", -1), "node": self.cfg.node,
            "renderNode": d.get("renderNode", ""), "kfdNode": d.get("kfdNode", -1),
            "numa": d.get("numa"), "partition": d.get("partition") or {},
            "healthy": bool(v.get("healthy")), "verdict": v,
            "present": d.get("present", uuid in self.by_uuid),
            "pods": pods.get(uuid, []),
        }
        if rec:
            res = rec.get("resourceName", schema.DEFAULT_RESOURCE)
            if rec.get("state") == "Probing":
                ps = self._probing_since.get(uuid)
                if ps is not None:
                    el = time.monotonic() - ps[0]
                    out["probingMs"] = round(el * 1e3, 1)
                    if el > ps[1] + self.PROBE_GRACE_S:
                        out["probeOverdue"] = True
            out.update({"state": rec.get("state", "Claimed"), "poolUID": rec["poolUID"],
                        "pool": rec.get("pool", ""), "resourceName": res,
                        "claimedAt": rec.get("claimedAt", ""),
                        "drainStartedAt": rec.get("drainStartedAt", ""),
                        "probe": rec.get("probe")})
            if self.plugins or self.cfg.plugin_dir:
                out["advertised"] = uuid in self.advertised.get(res, set()) and \
                    self._advertisable(uuid)
            else:
                out["advertised"] = self._advertisable(uuid)
        cov = self.scrubber.coverage(uuid)
        if cov:
            out["hbmSweep"] = cov
        xs = self._xgmi_summary(uuid)
        if xs:
            out["xgmiPairs"] = xs
        if self.pod_usage.get(uuid):
            out["usage"] = self.pod_usage[uuid]
        if rec and self._slots_of(rec) > 1:
            lay = self._slot_layout(uuid, rec)
            lay.pop("masks", None)
            out["sharing"] = lay
        out["telemetry"] = self._telemetry(d)
        if not rec:
            q = self.ledger.quarantined().get(uuid) if self.ledger else None
            out["state"] = ("Maintenance" if q.get("maintenance") else "Quarantined") if q else "Free"
            if q:
                out["quarantine"] = q
        return out

    @staticmethod
    def _telemetry(d: dict) -> dict:
        """Utilisation as last sampled (amdsmi_get_gpu_activity / _power_info / _memory_usage)."""
        act, pw = d.get("activity") or {}, d.get("power") or {}
        return {"gfxActivity": act.get("gfx"), "umcActivity": act.get("umc"),
                "powerW": pw.get("socketW"), "memUsedBytes": d.get("memUsedBytes"),
                "memTotalBytes": d.get("memTotalBytes")}

    def node_view(self, pool_uid: str = "") -> dict:
        """The node's devices; with ``pool_uid`` only that pool's GPUs plus ``freeHealthy`` (the
        count the manager needs to plan, without serialising every other GPU on every observe)."""
        pods = self._pods_by_device()
        with self.lock:
            uuids = list(self.by_uuid) + [u for u in self.records if u not in self.by_uuid]
            extra = {}
            if pool_uid:
                quarantined = self.ledger.quarantined()
                extra["freeHealthy"] = sum(
                    1 for u in self.by_uuid if u not in self.records and u not in quarantined and
                    self.verdicts.get(u, {}).get("healthy"))
                uuids = [u for u in uuids if (self.records.get(u) or {}).get("poolUID") == pool_uid]
            devices = [self.device_view(u, pods) for u in uuids]
            if self.prober.helpers is not None and not pool_uid:
                extra["probeHelpers"] = self.prober.helpers.snapshot()
            return {"node": self.cfg.node, "backend": self.backend, "gen": self.gen, **extra,
                    "probeMode": self.probe_mode, "preflight": self.preflight,
                    "advertiseRequired": bool(self.cfg.plugin_dir),
                    "eventSources": dict(self.events_supported),
                    "recentEvents": list(self.recent_events[-8:]),
                    "devices": devices, "topology": self.snap.get("topology", {})}

    # ================================================================ claims
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

    # ================================================================ xGMI link coverage
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
        members = list({d["uuid"]: d for d in owned + chosen}.values())
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
        return {"ok": True, "released": released}

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

    # ================================================================ device plugin glue
    @staticmethod
    def _slots_of(rec: dict) -> int:
        """spec.sharing.replicasPerGPU of the record's pool (time-sliced slots per GPU)."""
        try:
            return max(1, int(((rec.get("policy") or {}).get("sharing") or {})
                              .get("replicasPerGPU") or 1))
        except (TypeError, ValueError):
            return 1

    def plugin_devices(self, resource: str) -> list[dict]:
        """The device-plugin view of ``resource``: one entry per advertised device ID. A GPU of a
        pool with ``sharing.replicasPerGPU`` = K is K IDs ``<uuid>::<slot>``, all with the GPU's
        health (HAMi / time-slicing style: the kubelet places up to K pods on it)."""
        with self.lock:
            out = []
            for u, rec in sorted(self.records.items(),
                                 key=lambda kv: self.by_uuid.get(kv[0], {}).get("index", 99)):
                if rec.get("resourceName", schema.DEFAULT_RESOURCE) != resource:
                    continue
                k = self._slots_of(rec)
                ok = self._advertisable(u)
                numa = self.by_uuid.get(u, {}).get("numa")
                for i in range(k):
                    out.append({"id": u if k == 1 else f"{u}{SLOT_SEP}{i}", "uuid": u,
                                "advertisable": ok, "numa": numa})
            return out

    def mark_advertised(self, resource: str, healthy: set[str] | None) -> None:
        with self.lock:
            plugin = self.plugins.get(resource)
            before = set(self.advertised.get(resource, set()))
            if healthy is None:
                if plugin is None or plugin.streams <= 0:
                    self.advertised[resource] = set()
            else:
                self.advertised[resource] = set(healthy)
            flipped = before ^ self.advertised.get(resource, set())
            pools = {self.records[u]["poolUID"] for u in flipped if u in self.records}
        with self._adv_cv:
            self._adv_gen += 1
            self._adv_cv.notify_all()
        if pools:  # readiness depends on the advertised bit: tell the manager
            self._bump(pools)

    def _advertise_done(self, resource: str, uuids: list[str]) -> bool:
        """Every advertisable GPU of ``uuids`` reached the kubelet — or there is no registered
        plugin to wait for (no kubelet: readiness follows via events, never block the claim)."""
        with self.lock:
            want = [u for u in uuids if self._advertisable(u)]
            if all(u in self.advertised.get(resource, set()) for u in want):
                return True
            plugin = self.plugins.get(resource)
            return plugin is None or not plugin.registered

    def _wait_advertised(self, resource: str, uuids: list[str]) -> None:
        if not self.cfg.plugin_dir:
            return
        deadline = time.monotonic() + self.cfg.advertise_wait_s
        while time.monotonic() < deadline:
            with self._adv_cv:
                gen = self._adv_gen
            if self._advertise_done(resource, uuids):
                return
            with self._adv_cv:
                self._adv_cv.wait_for(lambda: self._adv_gen != gen, timeout=0.05)


    def _ensure_plugin(self, resource: str) -> None:
        if not self.cfg.plugin_dir:
            return
        with self.lock:
            if resource in self.plugins:
                return
            from .deviceplugin.server import DevicePluginServer
            p = DevicePluginServer(self, resource, self.cfg.plugin_dir)
            self.plugins[resource] = p
        p.start()

    def _notify_plugins(self, sync: bool = False) -> None:
        for p in list(self.plugins.values()):
            p.notify(sync)

    def preferred(self, resource: str, available: list[str], must: list[str], size: int) -> list[str]:
        if any(SLOT_SEP in i for i in available + must):
            # shared GPUs: a pod's slots go to as few GPUs as possible, lowest index first
            with self.lock:
                idx = {u: self.by_uuid.get(u, {}).get("index", 99) for u in
                       {gpu_of(i) for i in available + must}}
            def key(i: str) -> tuple[int, int]:
                u, _, slot = i.partition(SLOT_SEP)
                return idx.get(u, 99), int(slot or 0)
            rest = sorted((i for i in available if i not in must), key=key)
            return list(must) + rest[:max(0, size - len(must))]
        with self.lock:
            idx = {u: self.by_uuid[u]["index"] for u in available + must if u in self.by_uuid}
            inv = {v: k for k, v in idx.items()}
            topo = self.snap.get("topology") or {}
            n = len(self.snap["devices"])
            weights = topo.get("weights") or [[0 if i == j else 15 for j in range(n)]
                                              for i in range(n)]
            numa = [d.get("numa", 0) for d in sorted(self.snap["devices"], key=lambda x: x["index"])]
        need = size - len(must)
        cand = [idx[u] for u in available if u not in must and u in idx]
        sel = devlib.select(need, cand, [idx[u] for u in must if u in idx], "xgmi-packed",
                            weights, numa) if need > 0 else []
        return list(must) + [inv[i] for i in sel]

    def allocate_spec(self, resource: str, ids: list[str]) -> dict:
        slots = list(ids)
        ids = list(dict.fromkeys(gpu_of(i) for i in ids))  # slots of shared GPUs -> the GPUs
        for u in ids:  # a pod never starts while the HBM scrubber still frees its buffer
            if not self.scrubber.wait_released(u):
                raise ValueError(f"device {u}: HBM scrub buffer still being released")
        self._watch_pods()
        with self.lock:
            hip, render = [], []
            for u in ids:
                rec = self.records.get(u)
                if not rec or rec.get("resourceName", schema.DEFAULT_RESOURCE) != resource:
                    raise ValueError(f"device {u} is not in any pool advertised as {resource}")
                if not self._advertisable(u):
                    raise ValueError(f"device {u} is not healthy/allocatable (state "
                                     f"{rec.get('state')})")
                d = self.by_uuid[u]
                hip.append(d.get("hipUUID") or str(d["index"]))
                if d.get("renderNode"):
                    render.append(d["renderNode"])
            # ROCR_VISIBLE_DEVICES pins the container to exactly its GPUs (HIP ordinals then
            # start at 0); GPUPOOL_NUM_GPUS is the per-pod world-size hint and PET_NPROC_PER_NODE
            # the torchrun default for --nproc-per-node (torch.distributed.run reads PET_* env),
            # so a plain `torchrun train.py` in the pod starts one rank per allotted GPU over
            # RCCL (the reference's Kubeflow operator sets PET_*, GPU调度平台搭建.md:623).
            envs = {"ROCR_VISIBLE_DEVICES": ",".join(hip),
                    "GPUPOOL_DEVICE_UUIDS": ",".join(ids),
                    "GPUPOOL_NUM_GPUS": str(len(ids)),
                    "PET_NPROC_PER_NODE": str(len(ids)),
                    "GPUPOOL_NODE": self.cfg.node}
            mounts: list[dict] = []
            if slots != ids:  # time-sliced: the pod shares these GPUs with other pods
                envs["GPUPOOL_GPU_SLOTS"] = ",".join(slots)
                envs.update(self._isolation_env(slots, mounts))
        if "GPUPOOL_HBM_LIMIT_BYTES" in envs:  # the pod-wide HBM account (file I/O: off the lock)
            acct = self._share_account(slots, int(envs["GPUPOOL_HBM_LIMIT_BYTES"]), ids)
            if acct:
                mounts.append({"container_path": self.SHARE_ACCOUNT_PATH, "host_path": acct,
                               "read_only": False})
                envs["GPUPOOL_SHARE_ACCOUNT"] = self.SHARE_ACCOUNT_PATH
                # the limit itself, read-only: the account's counters must be writable by the
                # pod's processes, so its header limit is the pod's to edit — this one is not
                # (the library takes the smallest limit it is given)
                mounts.append({"container_path": self.SHARE_LIMIT_PATH,
                               "host_path": acct[:-len(".acct")] + ".limit", "read_only": True})
                envs["GPUPOOL_SHARE_LIMIT"] = self.SHARE_LIMIT_PATH
        return {"envs": envs, "devices": ["/dev/kfd"] + render, "mounts": mounts,
                "annotations": {schema.ANN_POD_DEVICES: ",".join(ids)}}

    SHARE_LIB_DIR = "/opt/gpupool/lib"  # where the pod sees libgpupool_share.so
    SHARE_ACCOUNT_PATH = "/var/run/gpupool/share.acct"  # where it sees its pod's HBM account
    SHARE_LIMIT_PATH = "/var/run/gpupool/share.limit"  # ...and, read-only, its limit
    SHARE_LIB = "libgpupool_share.so"

    def _install_share_lib(self) -> str | None:
        """Copy libgpupool_share.so from the agent's own tree (in the image) into
        ``<state_dir>/lib``. The state dir is the DaemonSet's hostPath (/var/lib/gpupool), so the
        copy exists on the HOST, where the container runtime resolves an Allocate mount's host
        path — the image path it came from does not. Atomic (temp file + rename); a copy whose
        bytes already match is kept, so pods that mapped it keep a stable inode. Returns the
        host directory, or None (isolated slots then fail their Allocate, loudly)."""
        from ..ops import native_dir
        src = os.path.join(native_dir(), self.SHARE_LIB)
        dst_dir = os.path.join(self.cfg.state_dir, "lib")
        dst = os.path.join(dst_dir, self.SHARE_LIB)
        try:
            with open(src, "rb") as f:
                data = f.read()
        except OSError as e:
            log.warning("isolated GPU sharing unavailable: %s not readable (%s)", src, e)
            return None
        try:
            os.makedirs(dst_dir, exist_ok=True)
            try:
                with open(dst, "rb") as f:
                    if f.read() == data:
                        return dst_dir
            except OSError:
                pass
            tmp = f"{dst}.{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(data)
                f.flush()
                os.fsync(f.fileno())
            os.chmod(tmp, 0o755)
            os.replace(tmp, dst)
            return dst_dir
        except OSError as e:
            log.warning("isolated GPU sharing unavailable: cannot install %s (%s)", dst, e)
            return None

    def share_mounts(self) -> list[str]:
        """Every host path an Allocate may mount (the deploy manifest must declare hostPath
        volumes covering them; tests/unit/test_deploy_manifests.py checks it)."""
        return [os.path.join(self.cfg.state_dir, "lib"), os.path.join(self.cfg.state_dir, "share")]

    def _share_account(self, slots: list[str], limit: int, gpus: list[str]) -> str | None:
        """One HBM account per allocation, shared by every process of the container: 16 KiB,
        magic + per-GPU limit + the GPUs' HIP UUIDs (what the library matches each HSA agent
        against, so ranks with different ROCR_VISIBLE_DEVICES charge the same counter for the same
        GPU), zeroed counters, the slot ids as text. A slot belongs to one container at a time, so
        an earlier account naming any of these slots belongs to a container that is gone: it is
        deleted here (and by the sampler once the kubelet lists none of its slots). Returns the
        host path (None if the state directory is not writable: the budget is then per process)."""
        d = os.path.join(self.cfg.state_dir, "share")
        mine = set(slots)
        try:
            os.makedirs(d, exist_ok=True)
            for name in os.listdir(d):
                if not name.endswith(".acct"):
                    continue
                path = os.path.join(d, name)
                if mine & set(slotlib.account_slots(path) or ()):
                    for p in (path, path[:-len(".acct")] + ".limit"):
                        try:
                            os.unlink(p)
                        except FileNotFoundError:  # the sampler's GC got there first
                            pass
            with self.lock:
                uuids = [(self.by_uuid.get(u) or {}).get("hipUUID") or "" for u in gpus]
            if not all(uuids):
                # a GPU without a hipUUID (amd-smi CLI backend, empty serial) cannot be matched by
                # identity: a version-2 account would match no GPU and silently fall back to a
                # per-process budget. A version-1 account maps by enumeration order instead.
                log.warning("HBM account for %s: GPU(s) without hipUUID %s; ordinal mapping",
                            slots, [u for u, h in zip(gpus, uuids) if not h])
                uuids = []
            stem = os.path.join(d, uuid4().hex)
            path = stem + ".acct"
            fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o666)
            try:
                os.write(fd, slotlib.account_bytes(limit, slots, uuids))
                os.fchmod(fd, 0o666)  # pods may run as any user
            finally:
                os.close(fd)
            fd = os.open(stem + ".limit", os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644)
            try:
                os.write(fd, slotlib.limit_bytes(limit))
            finally:
                os.close(fd)
            return path
        except OSError as e:
            log.warning("HBM account for %s not created (%s): budget is per process", slots, e)
            return None

    def gc_share_accounts(self, now: float | None = None) -> list[str]:
        """Delete the HBM accounts of pods that are gone: no device ID the kubelet's last
        PodResources listing shows is one of the account's slots. Runs every sample period."""
        pod_ids = self._pod_ids
        if pod_ids is None:
            return []
        listed_at, live = pod_ids
        # an account made after that listing began may belong to a pod it could not show yet
        cutoff = min(listed_at, (now or time.time()) - self.cfg.share_acct_grace_s)
        gone = slotlib.gc_accounts(os.path.join(self.cfg.state_dir, "share"), live, cutoff)
        if gone:
            log.info("removed %d HBM account(s) of exited pods", len(gone))
        return gone

    def _slot_layout(self, uuid: str, rec: dict) -> dict:
        """The isolation a GPU's slots get under its pool's spec.sharing: per-slot CU-mask bits and
        layout, the enforced per-slot HBM budget. Memoised per (GPU, sharing policy, CU count,
        partition, HBM size): node views ask for it on every observe. Called under self.lock."""
        share = (rec.get("policy") or {}).get("sharing") or {}
        d = self.by_uuid.get(uuid) or {}
        key = (uuid, json.dumps(share, sort_keys=True), (d.get("asic") or {}).get("computeUnits"),
               json.dumps(d.get("partition") or {}, sort_keys=True), d.get("memTotalBytes"))
        hit = self._layouts.get(key)
        if hit is None:
            if len(self._layouts) > 4096:
                self._layouts.clear()
            hit = self._layouts[key] = self._compute_slot_layout(rec, share, d)
        return {k: (list(v) if isinstance(v, list) else v) for k, v in hit.items()}

    def _compute_slot_layout(self, rec: dict, share: dict, d: dict) -> dict:
        k = self._slots_of(rec)
        out: dict = {"replicasPerGPU": k}
        per_slot = int(share.get("hbmBytesPerSlot") or 0)
        if per_slot > 0:
            # never more than a fair share of what the agent leaves free, whatever the spec says
            # (claims of an overcommitted pool are refused; this covers a later spec edit)
            mem = int(d.get("memTotalBytes") or 0)
            if mem > 0:
                per_slot = min(per_slot, max(0, mem - self.cfg.hbm_reserve_bytes) // k)
            out["hbmBytesPerSlot"] = per_slot
        cu = int(share.get("cuPerSlot") or 0)
        if cu > 0:
            cus = int((d.get("asic") or {}).get("computeUnits") or 256)
            xcds = slotlib.xcd_count(d)
            masks, layout = [], "striped"
            for i in range(k):
                bits, layout = slotlib.slot_cus(i, k, cu, cus, xcds)
                masks.append(bits)
            out.update({"cuLayout": layout, "cuPerSlot": len(masks[0]), "xcds": xcds,
                        "masks": masks,
                        # per slot: its CU-mask bits and the XCDs they land on (node views)
                        "slotCUMasks": [_ranges(m) for m in masks],
                        "slotXcds": [_ranges(slotlib.slot_xcds(m, xcds)) for m in masks]})
        return out

    def _isolation_env(self, slots: list[str], mounts: list[dict]) -> dict[str, str]:
        """spec.sharing.hbmBytesPerSlot / cuPerSlot of the pool owning these slots: the ROCm
        runtime loads libgpupool_share.so (HSA_TOOLS_LIB) into the pod, which caps its HBM per
        GPU at (its slots on that GPU) x hbmBytesPerSlot and confines its queues to its slots'
        CUs — contiguous mask bits, disjoint from the other slots, the same number of CUs on every
        XCD (slots.py: why not whole XCDs). The library is mounted from its host copy under the
        state dir. Called under self.lock."""
        per_gpu: dict[str, list[int]] = {}
        for sid in slots:
            u, _, i = sid.partition(SLOT_SEP)
            per_gpu.setdefault(u, []).append(int(i or 0))
        hbm, cu_mask = 0, set()
        per_gpu_mask: dict[str, set[int]] = {}  # hipUUID -> the CUs of this pod's slots there
        for u, idx in per_gpu.items():
            lay = self._slot_layout(u, self.records.get(u) or {})
            if lay.get("hbmBytesPerSlot"):
                hbm = max(hbm, lay["hbmBytesPerSlot"] * len(idx))
            if "masks" in lay:
                hip = (self.by_uuid.get(u) or {}).get("hipUUID") or ""
                for i in idx:
                    bits = lay["masks"][i % len(lay["masks"])]
                    cu_mask.update(bits)
                    if hip:
                        per_gpu_mask.setdefault(hip, set()).update(bits)
        if not hbm and not cu_mask:
            return {}
        if not self.share_lib_dir:
            raise ValueError("isolated GPU sharing requested but libgpupool_share.so is not "
                             f"installed under {self.cfg.state_dir}/lib (see the agent log)")
        mounts.append({"container_path": self.SHARE_LIB_DIR, "host_path": self.share_lib_dir,
                       "read_only": True})
        env = {"HSA_TOOLS_LIB": f"{self.SHARE_LIB_DIR}/{self.SHARE_LIB}"}
        xcds = {lay.get("xcds") for lay in (self._slot_layout(u, self.records.get(u) or {})
                                             for u in per_gpu) if lay.get("xcds")}
        if cu_mask and xcds:  # a narrowed app mask must keep a CU on each XCD (share.cc)
            env["GPUPOOL_CU_XCDS"] = str(max(xcds))
        if hbm:  # allocate_spec adds the pod-wide account file (GPUPOOL_SHARE_ACCOUNT)
            env["GPUPOOL_HBM_LIMIT_BYTES"] = str(hbm)
        if cu_mask:
            # each GPU's own slot CUs, keyed by the UUID the library reads from the queue's agent: a
            # pod holding slot 0 of GPU A and slot 1 of GPU B must not get the union on both (it
            # overlaps the sibling tenants); the union stays as the fallback for a GPU not named
            env["GPUPOOL_CU_MASK"] = _ranges(sorted(cu_mask))
            env["GPUPOOL_CU_LAYOUT"] = "striped"
            if per_gpu_mask:
                env["GPUPOOL_CU_MASKS"] = ";".join(f"{h}={_ranges(sorted(b))}"
                                                   for h, b in sorted(per_gpu_mask.items()))
        return env

    # ================================================================ leader fencing
    MUTATING = {"/v1/claims", "/v1/release", "/v1/cordon", "/v1/policy", "/v1/maintenance"}

    def check_leader(self, method: str, path: str, headers: dict) -> tuple | None:
        """Fencing tokens (the manager's Lease, README.md:162->242's missing manager step): every
        mutating RPC of a leader-elected manager carries its identity, its epoch (the Lease's
        leaseTransitions) and the Lease's generation (creationTimestamp + uid: leaseTransitions
        starts again at 0 when the Lease is deleted and created anew). The newest token seen is
        persisted; tokens are ordered by (generation, epoch): an older one — a leader that was
        paused between its own fence check and the send while a successor took over, or a leader
        of a Lease that has since been recreated — is refused with 409 StaleLeader before anything
        is touched. A request without a token (leader election off, an admin's gpuctl) is not
        checked."""
        if method != "POST" or path not in self.MUTATING:
            return None
        raw = headers.get("x-gpupool-leader-epoch")
        if raw is None:
            return None
        from .rpc import json_reply
        try:
            epoch = int(raw)
        except ValueError:
            return json_reply({"reason": "BadRequest", "message": f"bad leader epoch {raw!r}"}, 400)
        holder = headers.get("x-gpupool-leader", "")
        lease = headers.get("x-gpupool-leader-lease")  # "<creationTimestamp> <uid>"
        created, _, uid = (lease or "").strip().partition(" ")
        with self._fence_mu:
            cur = self.leader_fence
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
                # a fence persisted before tokens carried the Lease generation: a Lease created
                # after that fence was recorded is a newer one (else its epoch, restarted at 0,
                # would be refused for good)
                newer_lease = created > str(cur.get("at", ""))
            stale = older_lease or (not newer_lease and (
                epoch < cur_e or (epoch == cur_e and cur_h and holder != cur_h)))
            if stale:
                self.stats["stale_leader_refused"] = self.stats.get("stale_leader_refused", 0) + 1
                log.warning("refused %s from stale leader %s (epoch %d, lease %s; newest seen %s "
                            "at %d, lease %s)", path, holder, epoch, created or "?", cur_h, cur_e,
                            cur_c or "?")
                return json_reply({"reason": "StaleLeader",
                                   "message": f"leader {holder} epoch {epoch} is stale: {cur_h} holds "
                                              f"epoch {cur_e}"
                                              + (" of a newer Lease" if older_lease else "")}, 409)
            if newer_lease or epoch > cur_e or not cur_h or (created and not cur_c):
                if newer_lease and cur_u:
                    retired = (retired + [cur_u])[-8:]
                self.leader_fence = {"holder": holder, "epoch": epoch, "at": now_rfc3339(),
                                     **({"leaseCreated": created, "leaseUID": uid,
                                         "retiredLeaseUIDs": retired} if created else {})}
                self.ledger.commit_leader(self.leader_fence)  # durable before acting on it
        return None

    # ================================================================ node registration
    def _node_conditions(self) -> dict[str, tuple[str, str, str]]:
        """The agent's own Node conditions (nodereg.OWN_CONDITIONS): type -> (status, reason,
        message)."""
        failed = {k: v["detail"] for k, v in self.preflight["checks"].items() if not v["ok"]}
        return {
            "GPUPoolAgentReady": ("True", "AgentRunning",
                                  f"{len(self.by_uuid)} GPU(s) via {self.backend}; probe "
                                  f"{self.probe_mode}"),
            "ROCmReady": ("True" if self.preflight["ready"] else "False",
                          "PreflightPassed" if self.preflight["ready"] else "PreflightFailed",
                          "; ".join(f"{k}: {v}" for k, v in failed.items()) or
                          "; ".join(v["detail"] for v in self.preflight["checks"].values()))}

    def node_registrar(self, client=None):
        """The Node registration / heartbeat writer (nodereg.py) for this agent."""
        from ..kube import Client
        from .nodereg import NodeRegistrar
        devs = self.snap["devices"]
        gfx = sorted({(d.get("asic") or {}).get("gfx", "") for d in devs} - {""})
        labels = {schema.LABEL_GFX: gfx[0] if gfx else "unknown",
                  "amd.com/gpu.count": str(len(devs)),
                  "amd.com/gpu.product": "MI355X",
                  "gpupool.amd.com/backend": self.backend}
        parts = sorted({(d.get("partition") or {}).get("compute", "") for d in devs} - {""})
        if parts:
            labels["amd.com/compute-partition"] = parts[0]
        c = client or Client.connect(self.cfg.apiserver, self.cfg.token or None,
                                     token_file=self.cfg.token_file or None)
        return NodeRegistrar(c, self.cfg.node, labels,
                             {schema.ANN_AGENT_ENDPOINT: self.endpoint()}, self._node_conditions)

    def register_node(self) -> None:
        if not self.cfg.apiserver:
            return
        self.registrar = self.node_registrar()
        if not self.registrar.heartbeat():
            log.info("node %s not registered by its kubelet yet: the heartbeat retries",
                     self.cfg.node)

    def _heartbeater(self) -> None:
        reg = self.registrar
        while not self._stop.wait(self.cfg.heartbeat_interval if reg.registered else 1.0):
            reg.heartbeat()

    def endpoint(self) -> str:
        if self.cfg.endpoint:
            return self.cfg.endpoint
        if self.cfg.socket:
            return "unix://" + os.path.abspath(self.cfg.socket)
        return f"{'https' if self.cfg.tls_cert else 'http'}://{self.cfg.listen}"

    # ================================================================ metrics
    def metrics_text(self) -> str:
        lines = []
        with self.lock:
            lines.append("# TYPE gpupool_device_healthy gauge")
            for u, d in self.by_uuid.items():
                rec = self.records.get(u) or {}
                lab = f'uuid="{u}",index="{d.get("index")}",node="{self.cfg.node}",' \
                      f'pool="{rec.get("pool", "")}"'
                v = self.verdicts.get(u, {})
                # utilisation (GPU调度平台搭建.md:800 "Prometheus + Grafana, GPU utilisation");
                # the pool label lets dashboards aggregate per pool / tenant
                tel = self._telemetry(d)
                for name, key in (("gpupool_device_gfx_activity_percent", "gfxActivity"),
                                  ("gpupool_device_umc_activity_percent", "umcActivity"),
                                  ("gpupool_device_power_watts", "powerW"),
                                  ("gpupool_device_vram_used_bytes", "memUsedBytes"),
                                  ("gpupool_device_vram_total_bytes", "memTotalBytes")):
                    if isinstance(tel.get(key), (int, float)):
                        lines.append(f"{name}{{{lab}}} {tel[key]}")
                ras = d.get("ras") or {}
                if ras.get("badPagesSupported"):
                    for t in ("retired", "pending", "unreservable"):
                        lines.append(f'gpupool_device_hbm_bad_pages{{{lab},state="{t}"}} '
                                     f"{ras.get(t + 'Pages', 0)}")
                lines.append(f"gpupool_device_healthy{{{lab}}} {1 if v.get('healthy') else 0}")
                lines.append(f"gpupool_device_claimed{{{lab}}} {1 if u in self.records else 0}")
                lines.append(f"gpupool_device_xgmi_links_up{{{lab}}} "
                             f"{(d.get('xgmi') or {}).get('up', 0)}")
                xs = self._xgmi_summary(u)
                if xs:  # peer-copy coverage of this GPU's pairs, and the pairs that failed
                    lines.append(f"gpupool_device_xgmi_pairs_covered{{{lab}}} {xs['pairsCovered']}")
                    lines.append(f"gpupool_device_xgmi_pairs_failed{{{lab}}} "
                                 f"{len(xs.get('failedPeers') or [])}")
                for t in ("correctable", "uncorrectable"):
                    lines.append(f'gpupool_device_ecc_errors_total{{{lab},type="{t}"}} '
                                 f"{(d.get('ecc') or {}).get(t, 0)}")
                for s, t in (d.get("temps") or {}).items():
                    if isinstance(t, dict) and t.get("current") is not None:
                        lines.append(f'gpupool_device_temperature_celsius{{{lab},sensor="{s}"}} '
                                     f"{t['current']}")
                cov = self.scrubber.coverage(u)
                if cov:
                    lines.append(f"gpupool_device_hbm_sweep_passes_total{{{lab}}} {cov.get('passes', 0)}")
                    lines.append(f"gpupool_device_hbm_sweep_fraction{{{lab}}} {cov.get('fraction', 0)}")
                pr = self.last_probe.get(u)
                if pr:  # last claim-time probe of this GPU (performance trend across claims)
                    lines.append(f"gpupool_device_probe_passed{{{lab}}} {1 if pr.get('passed') else 0}")
                    lines.append(f"gpupool_device_probe_hbm_gbps{{{lab}}} "
                                 f"{float((pr.get('hbm') or {}).get('GBps') or 0):.1f}")
                    lines.append(f"gpupool_device_probe_mfma_tflops{{{lab}}} "
                                 f"{float((pr.get('mfma') or {}).get('tflops') or 0):.1f}")
            lines.append("# TYPE gpupool_pod_vram_bytes gauge")
            for u, pods in self.pod_usage.items():
                d = self.by_uuid.get(u) or {}
                pool = (self.records.get(u) or {}).get("pool", "")
                for e in pods:
                    lab = f'uuid="{u}",index="{d.get("index")}",node="{self.cfg.node}",' \
                          f'pool="{pool}",namespace="{e["namespace"]}",pod="{e["pod"]}"'
                    lines.append(f"gpupool_pod_vram_bytes{{{lab}}} {e['vramBytes']}")
                    if e.get("slotBudgetBytes"):
                        lines.append(f"gpupool_pod_slot_budget_bytes{{{lab}}} {e['slotBudgetBytes']}")
                        lines.append(f"gpupool_pod_over_slot_budget{{{lab}}} "
                                     f"{1 if e.get('overBudget') else 0}")
                    if e.get("gfxBusy") is not None:
                        lines.append(f"gpupool_pod_gfx_busy_ratio{{{lab}}} {e['gfxBusy']}")
            for k, v in self.stats.items():
                lines.append(f"gpupool_agent_{k} {v}")
            if self.registrar is not None:  # Node registration / condition heartbeat (nodereg.py)
                for k, v in self.registrar.stats.items():
                    lines.append(f"gpupool_agent_node_{k} {v}")
            for src, ok in self.events_supported.items():
                lines.append(f'gpupool_agent_event_source_supported{{source="{src}"}} {1 if ok else 0}')
            for k, v in self.scrubber.stats.items():
                lines.append(f"gpupool_agent_hbm_scrub_{k}_total {v}")
            lines.append(f"gpupool_agent_gen {self.gen}")
            # the newest manager fencing token seen (-1: none): a takeover raises it
            lines.append(f"gpupool_agent_leader_epoch {int(self.leader_fence.get('epoch', -1))}")
            # GPUs the agent's probe helpers (or, inproc, the agent) hold a HIP context on
            lines.append(f"gpupool_agent_hip_devices {self.prober.hip_devices()}")
            lines.append(f"gpupool_agent_hip_init_ms {self.prober.init_ms:.1f}")
            if self.prober.helpers is not None:
                rss, pss = self.prober.helpers_mem()
                lines.append(f"gpupool_agent_probe_helpers_rss_bytes {rss}")
                lines.append(f"gpupool_agent_probe_helpers_pss_bytes {pss}")
                lines.append(f"gpupool_agent_probe_helpers {len(self.prober.helper_pids())}")
                fab = self.prober.helpers.snapshot().get("fabric") or {}
                if fab.get("warmMs") is not None:  # the xGMI fabric helper's all-pairs warm-up
                    warm = fab.get("warm") or {}
                    lines.append(f"gpupool_agent_probe_fabric_warm_ms {fab['warmMs']:.1f}")
                    lines.append(f"gpupool_agent_probe_fabric_warm_links {int(warm.get('links') or 0)}")
                    lines.append(f"gpupool_agent_probe_fabric_warm_passed {int(bool(warm.get('passed')))}")
                for k, v in self.prober.helpers.stats.items():
                    lines.append(f"gpupool_agent_probe_{k}_total {v}")
                for k, v in self.prober.helpers.snapshot().items():
                    idx = self.by_uuid.get(k, {}).get("index", k)
                    lines.append(f'gpupool_agent_probe_helper_up{{helper="{idx}",node="{self.cfg.node}"}} '
                                 f"{1 if v.get('alive') else 0}")
        lines += process_metrics()
        return "\n".join(lines) + "\n"

    # ================================================================ lifecycle
    def start_background(self) -> None:
        if self._podres is not None:
            try:
                self._refresh_pods()
            except Exception as e:  # kubelet not up yet: the sampler retries every period
                log.info("podresources not reachable yet: %s", e)
        # Plugins for the default resource and every resource in the ledger register now (as a
        # device plugin does at start-up), so a first claim never waits on plugin start, kubelet
        # registration and the first ListAndWatch (seconds once on a busy box, profiles/r2l).
        for res in {schema.DEFAULT_RESOURCE} | {r.get("resourceName", schema.DEFAULT_RESOURCE)
                                                 for r in self.records.values()}:
            self._ensure_plugin(res)
        loops = [(self._sampler, "sampler"), (self._device_event_watcher, "dev-events"),
                 (self._fault_watcher, "fault-watch")]
        if self.cfg.health_interval > 0:
            loops.append((self._health_poller, "health-poll"))
        if self._podres is not None and self.cfg.pod_watch_interval > 0:
            loops.append((self._pod_watcher, "pod-watch"))
        for fn, name in loops:
            t = threading.Thread(target=fn, daemon=True, name=name)
            t.start()
            self._threads.append(t)
        self.scrubber.start()
        if self.cfg.apiserver:
            self.register_node()
            t = threading.Thread(target=self._heartbeater, daemon=True, name="heartbeat")
            t.start()
            self._threads.append(t)

    def stop(self) -> None:
        self._stop.set()
        self.scrubber.stop()
        for p in list(self.plugins.values()):
            p.stop()
        self.prober.close()


# ==================================================================== RPC server
def build_routes(agent: Agent) -> dict:
    """The manager-facing RPC surface (served by ``rpc.RpcServer``, one thread per connection;
    every route but /healthz and /metrics requires the shared bearer token)."""
    from .rpc import json_reply, text_reply

    def body_json(body: bytes) -> dict:
        return json.loads(body or b"{}")

    def node(q, body):
        return json_reply(agent.node_view(q.get("pool", "")))

    def claims(q, body):
        req = body_json(body)
        if not req.get("poolUID") or int(req.get("count", 0)) <= 0:
            return json_reply({"reason": "BadRequest", "message": "poolUID and count>0 required"},
                              400)
        req["_t_in"] = time.perf_counter()
        pool = req["poolUID"]
        try:
            out = agent.claim(req, hold_events=True)
        except BaseException:
            agent.release_events(pool)
            raise
        tm = out.get("timingsMs")
        if tm is not None:  # reply serialisation (the claim ran on this connection's thread)
            tm["executorOut"] = round((time.perf_counter() - out.pop("_t_done")) * 1e3, 3)
        deferred = out.pop("_after", [])

        def after() -> None:  # the reply goes out first; then the deferred work and the events
            try:
                for fn in deferred:
                    fn()
            finally:
                agent.release_events(pool)
        return json_reply(out, after=after)

    def cordon(q, body):
        b = body_json(body)
        return json_reply(agent.cordon(b["poolUID"], b.get("uuids", [])))

    def release(q, body):
        b = body_json(body)
        out = agent.release(b["poolUID"], b.get("uuids", []))
        return json_reply(out, 200 if out.get("ok") else 409)

    def maintenance(q, body):
        b = body_json(body)
        out = agent.set_maintenance(str(b.get("gpu", "")), bool(b.get("on", True)),
                                    str(b.get("reason", "")))
        return json_reply(out, 200 if out.get("ok") else 404)

    def policy(q, body):
        b = body_json(body)
        return json_reply(agent.update_policy(b["poolUID"], b.get("policy") or {},
                                              b.get("resourceName")))

    def events(q, body):
        since = int(q.get("since", "-1"))
        timeout = min(float(q.get("timeoutSeconds", "30")), 300.0)
        gen, pools = agent.changed_since(since)
        if gen == since:
            with agent.gen_cv:
                agent.gen_cv.wait_for(lambda: agent.gen != since, timeout)
            gen, pools = agent.changed_since(since)
        return 200, "application/json", (json.dumps({"gen": gen, "pools": pools}) + "\n").encode(), None

    def sample(q, body):
        changed = agent.sample()
        return json_reply({"changed": sorted(changed), "gen": agent.gen})

    def scrub(q, body):
        """Synchronous HBM scrub of one free GPU (admin / tests): {"gpu": uuid|hipUUID|index,
        "windows": n}."""
        b = body_json(body)
        ref = str(b.get("gpu", ""))
        uuid = next((u for u, d in list(agent.by_uuid.items())
                     if ref in (u, d.get("hipUUID"), str(d.get("index")))), None)
        if uuid is None:
            return json_reply({"ok": False, "reason": "NotFound"}, 404)
        rec = agent.scrubber.scrub_device(uuid, int(b.get("windows") or 1), grace=False)
        return json_reply({"ok": True, "uuid": uuid, "coverage": agent.scrubber.coverage(uuid),
                           "record": rec})

    def xgmi_check(q, body):
        """Run the idle xGMI coverage ring now (admin / tests)."""
        return json_reply(agent.xgmi_recheck(True))

    def healthz(q, body):
        return text_reply("ok\n")

    def metrics(q, body):
        extra = agent.rpc.metrics_lines() if agent.rpc is not None else []
        return text_reply(agent.metrics_text() + "\n".join(extra) + ("\n" if extra else ""))

    return {("GET", "/v1/node"): node, ("POST", "/v1/claims"): claims,
            ("POST", "/v1/cordon"): cordon, ("POST", "/v1/release"): release,
            ("POST", "/v1/policy"): policy, ("POST", "/v1/maintenance"): maintenance,
            ("GET", "/v1/events"): events, ("POST", "/v1/sample"): sample,
            ("POST", "/v1/scrub"): scrub, ("POST", "/v1/xgmi-check"): xgmi_check,
            ("GET", "/healthz"): healthz, ("GET", "/metrics"): metrics}


def serve(agent: Agent, ready_file: str | None = None) -> None:
    """Start the RPC listeners and the agent's background loops; block until interrupted."""
    from .rpc import RpcServer
    srv = RpcServer(build_routes(agent), agent.cfg.auth_token, guard=agent.check_leader)
    agent.rpc = srv
    # the start-up heap (modules, gRPC/protobuf descriptors, the device model) lives for the whole
    # run: out of the collector's generations, a full collection walks only what came after — one
    # over the whole heap costs ~6-8 ms, which a claim that happened to trigger it would pay
    import gc
    gc.collect()
    gc.freeze()
    if agent.cfg.socket:
        srv.listen_unix(agent.cfg.socket)
    if agent.cfg.listen:
        host, port = agent.cfg.listen.rsplit(":", 1)
        ctx = None
        if agent.cfg.tls_cert:  # across nodes the RPC (and its bearer token) travels encrypted
            import ssl
            ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
            ctx.minimum_version = ssl.TLSVersion.TLSv1_2
            ctx.load_cert_chain(agent.cfg.tls_cert, agent.cfg.tls_key or None)
        srv.listen_tcp(host, int(port), ctx)
    agent.start_background()
    if ready_file:
        with open(ready_file + ".tmp", "w") as f:
            json.dump({"node": agent.cfg.node, "endpoint": agent.endpoint(),
                       "devices": len(agent.by_uuid), "probe": agent.probe_mode}, f)
        os.replace(ready_file + ".tmp", ready_file)
    print(f"gpupool-agent {agent.cfg.node} serving on {agent.endpoint()}", flush=True)
    try:
        while True:
            time.sleep(3600)
    finally:
        srv.close()

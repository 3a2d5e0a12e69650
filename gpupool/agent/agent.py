"""gpupool node agent: owns one node's MI355X GPUs.

Responsibilities (SURVEY.md §7.1 architecture), one module each:
  * discovery + telemetry through libmi355x_dev (amdsmi | cli | fake backend, fault overlay) and
    health verdicts under each owning pool's policy — health.py;
  * the claim ledger (all-or-nothing, topology-aware claims; cordon; release; quarantine) —
    claims.py, ledger.py; claim-time HIP probes in per-GPU helpers — prober.py, probehost.py;
  * xGMI link coverage rings — xgmi.py;
  * the ROCm device plugin endpoints (one per extended resource) — advertise.py, deviceplugin/;
    PodResources lookups — podview.py; per-pod accounting and slot budgets — accounting.py;
    isolated slot sharing — sharing.py;
  * Node registration + condition heartbeat — nodereg.py; leader fencing — fence.py;
  * an HTTP/JSON RPC surface for the manager (unix socket and/or TCP) with a long-poll event
    feed — routes.py, rpc.py.
This module holds the Agent's state, its views and its lifecycle.

Replaces what the reference's controller did through the Azure SDK (README.md:179-221) with a
node-local owner of physical devices.
"""
from __future__ import annotations

import logging
import os
import socket
import threading
import time
from dataclasses import dataclass, field
from typing import Any

from ..api import schema
from ..ops import devlib
from .accounting import AccountingMixin
from .advertise import AdvertiseMixin
from .claims import ClaimsMixin
from .common import SLOT_SEP, _ranges, gpu_of, now_rfc3339  # noqa: F401 (re-exported)
from .fence import LeaderFence, StaleLeader
from .health import HealthMixin
from .ledger import Ledger
from .podview import PodViewMixin
from .prober import Prober, default_mode
from .sharing import SharingMixin
from .xgmi import XgmiMixin

log = logging.getLogger("gpupool.agent")


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
    auth_token_file: str = ""        # ... from a file, re-read as it rotates (old one: grace)
    auth_grace_s: float = 300.0      # how long a rotated-out token stays valid
    manager_pubkeys: str = ""        # PEM bundle / dir of the manager's Ed25519 request keys
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


class Agent(HealthMixin, AccountingMixin, PodViewMixin, ClaimsMixin, XgmiMixin,
            AdvertiseMixin, SharingMixin):
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
        self.stats: dict[str, Any] = {}
        # the newest manager leader seen on a mutating RPC ({"holder", "epoch"}, ledger-persisted)
        self.fence = LeaderFence(self.ledger.leader_state(), self.ledger.commit_leader, self.stats)
        self.pod_usage: dict[str, list[dict]] = {}        # uuid -> per-pod VRAM / gfx time
        self._proc_prev: dict[tuple[str, int], list] = {}  # (uuid, pid) -> [(t, gfxNs)]
        self._pid_pods: dict[int, dict] = {}
        self._pid_miss: dict[int, float] = {}
        self._pods_by_uid: tuple[float, dict[str, dict]] = (0.0, {})
        self._xgmi_last = time.monotonic()
        self.stats.update({"claims": 0, "releases": 0, "probes": 0, "probe_failures": 0,
                           "rechecks": 0, "probe_ms_sum": 0.0, "samples": 0, "sample_ms_sum": 0.0,
                           "health_polls": 0, "health_poll_ms_sum": 0.0,
                           "device_events": 0, "fault_events": 0})
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
        self._api = None       # apiserver client (api())
        self._kx = None        # X25519 key of the per-node RPC MAC (kx)
        self._park_mu = threading.Lock()  # podview._sync_parking
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

    # ================================================================ views

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
        if uuid in self.prober.parked():  # no agent HIP context while a tenant holds it
            out["probeHelper"] = "Parked"
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

    # ================================================================ xGMI link coverage

    # ================================================================ device plugin glue

    # ================================================================ leader fencing
    @property
    def leader_fence(self) -> dict:
        return self.fence.state

    def check_leader(self, method: str, path: str, headers: dict) -> tuple | None:
        """The RPC server's guard: a mutating RPC from a stale manager leader is refused with
        409 StaleLeader before anything is touched (fence.py)."""
        try:
            self.fence.admit(method, path, headers)
        except StaleLeader as e:
            from .rpc import json_reply
            return json_reply({"reason": e.reason, "message": str(e)}, e.status)
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
        c = client or self.api()
        ann = {schema.ANN_AGENT_ENDPOINT: self.endpoint()}
        if self.kx is not None:  # the per-node MAC key's public half (edsig v2)
            ann[schema.ANN_AGENT_KX] = self.kx.annotation()
        return NodeRegistrar(c, self.cfg.node, labels, ann, self._node_conditions)

    def api(self):
        """The agent's apiserver client: one per process (per-thread keep-alive connections), its
        token re-read from ``token_file`` as it rotates (60 s, and at once after a 401)."""
        if self._api is None:
            from ..kube import Client
            self._api = Client.connect(self.cfg.apiserver, self.cfg.token or None,
                                       token_file=self.cfg.token_file or None)
            self._api.user_agent = "gpupool-agent/0.1"
        return self._api

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

    def rpc_auth(self):
        """The RPC's credentials (auth.py): manager signatures bound to this node, and/or the
        rotating shared token."""
        from ..utils import edsig
        from .auth import AgentAuth, TokenAuth
        ver = edsig.Verifier(self.cfg.manager_pubkeys, self.cfg.node, kx=self.kx) \
            if self.cfg.manager_pubkeys else None
        tok = None
        if self.cfg.auth_token_file or self.cfg.auth_token:
            tok = TokenAuth(self.cfg.auth_token, self.cfg.auth_token_file, self.cfg.auth_grace_s)
        return AgentAuth(ver, tok)

    @property
    def kx(self):
        """This agent's X25519 key (state dir; None without manager public keys)."""
        if self._kx is None and self.cfg.manager_pubkeys:
            from ..utils import edsig
            os.makedirs(self.cfg.state_dir, exist_ok=True)
            self._kx = edsig.AgentKx(os.path.join(self.cfg.state_dir, "agent-kx.key"))
        return self._kx

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


from .routes import build_routes, serve  # noqa: E402,F401 (re-exported)

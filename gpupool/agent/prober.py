"""Claim-time readiness probes (the MI355X replacement of `nvidia-smi` in a pod).

Modes:
  helper     — (default on real GPUs) the gfx950 probe runs in probe-helper child processes, one
               per GPU, each with a HIP context on its GPU only (probehost.py): a probe that faults
               kills its helper, not the agent; one that hangs is cut at spec.probe.timeoutSeconds.
               Helpers are warm (started with the agent), so a claim pays the kernels plus one
               pipe round trip. The xGMI peer ring runs in an on-demand fabric helper.
  helper-sim — the same helpers running the simulated kernels (fake backend on CPU): the whole
               isolation machinery — children, deadlines, crash replacement — without a GPU.
  inproc     — libmi355x_probe.so loaded in the agent itself. Kept only for A/B measurements of
               the helper's cost: a GPU fault in it takes the whole agent down.
  subprocess — `mi355x-probe --device N` per GPU (cold HIP init per probe).
  simulated  — for the fake backend on CPU-only hosts: a fixed latency and a result that fails
               only when the fault overlay sets ``probeFail``. Never used with real GPUs.
  off        — no probe (result passes with backend "off").

Probe failures the isolation produces (``error`` prefixes, surfaced on DeviceProbePassed):
  ProbeCrashed — the helper died while probing this GPU (e.g. HIP aborted on a memory fault);
  ProbeTimeout — the probe did not finish within spec.probe.timeoutSeconds; the helper was killed;
  ProbeUnavailable — the GPU's helper is being replaced after a crash (backoff) or never came up.
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import logging
import os
import subprocess
import threading
import time

from ..ops import native_path
from . import simprobe

log = logging.getLogger("gpupool.agent.prober")

HELPER_MODES = ("helper", "helper-sim")
DEFAULT_TIMEOUT_S = 10.0
# deadline of one xGMI ring (all its links at once: ~1 ms at 16 MiB per link on MI355X)
RING_TIMEOUT_S = float(os.environ.get("GPUPOOL_XGMI_RING_TIMEOUT_S", "3"))  # spec.probe.timeoutSeconds default (schema.py)


class Prober:
    def __init__(self, mode: str = "inproc", sim_ms: float = 20.0, gemm_n: int = 4096,
                 max_workers: int = 16, arena_idle_s: float = 10.0, overlap_gemm_n: int = 2048,
                 devices: list[dict] | None = None, fabric_idle_s: float = 0.0,
                 fabric_prewarm: bool = True):
        self.mode = mode
        self.sim_ms = sim_ms
        self.gemm_n = gemm_n                  # serial probe (pools with performance floors)
        # the claim-time probe's GEMM when it overlaps the HBM pattern test: the element check,
        # ABFT and the all-CU census run whatever its size, and a smaller GEMM takes less HBM
        # bandwidth from the pattern test (profiles/r4_probe_gemm_overlap_ab.json)
        self.overlap_gemm_n = overlap_gemm_n
        self.pool = cf.ThreadPoolExecutor(max_workers=max_workers, thread_name_prefix="probe")
        self.ordinals: dict[str, int] = {}
        self.helpers = None
        self.init_ms = 0.0
        t0 = time.perf_counter()
        if mode == "inproc":
            from ..ops import probe as hip_probe
            self._hip = hip_probe
            n = hip_probe.init()
            self.ordinals = hip_probe.hip_uuid_map()
            log.warning("HIP probe initialised IN the agent (%d device(s)): a GPU fault during a "
                        "probe takes the agent down; use --probe helper in production", n)
            # probe arenas stay allocated between back-to-back claims (scale-up bursts) and are
            # handed back to the GPU's workloads once idle for arena_idle_s
            self._trim_stop = threading.Event()
            self._trim_idle_ms = int(arena_idle_s * 1e3)
            threading.Thread(target=self._trim_loop, daemon=True, name="probe-trim").start()
        elif mode in HELPER_MODES:
            from .probehost import HelperPool
            # the xGMI fabric helper (2+ GPUs): resident (started with the GPU helpers, warmed
            # with one 1 MiB ring before it reports ready, replaced after an exit) unless it is
            # let go when idle (fabric_idle_s > 0) — then it starts on a ring's demand
            self.helpers = HelperPool("hip" if mode == "helper" else "sim", sim_ms=sim_ms,
                                      arena_idle_s=arena_idle_s, fabric_idle_s=fabric_idle_s,
                                      resident_fabric=fabric_prewarm and fabric_idle_s <= 0)
            ready = self.helpers.start(list(devices or []))
            ready.pop("fabric", None)  # not waited for: it warms in the background
            up = sorted(u for u, r in ready.items() if r.get("ok"))
            bad = {u: r.get("error") for u, r in ready.items() if not r.get("ok")}
            log.info("probe helpers up for %d/%d GPU(s)%s", len(up), len(ready),
                     f"; failed: {bad}" if bad else "")
        elif mode == "subprocess":
            out = subprocess.run([native_path("mi355x-probe"), "--list"], capture_output=True,
                                 text=True, timeout=120)
            for line in out.stdout.splitlines():
                info = json.loads(line)
                if info.get("hipUUID"):
                    self.ordinals[info["hipUUID"].lower()] = int(info["device"])
        elif mode not in ("simulated", "off"):
            raise ValueError(f"unknown probe mode {mode!r}")
        self.init_ms = (time.perf_counter() - t0) * 1e3

    # ------------------------------------------------------------ visibility
    def visible(self, dev: dict) -> bool:
        """Can this prober run kernels on ``dev``?"""
        if self.mode in HELPER_MODES:
            return self.helpers.alive(dev["uuid"])
        if self.mode in ("inproc", "subprocess"):
            return str(dev.get("hipUUID", "")).lower() in self.ordinals
        return True

    def can_probe(self, dev: dict) -> bool:
        """False while ``dev``'s probe helper is held back after an exit (respawn backoff): a
        claim then leaves the GPU out instead of failing it (and quarantining it) for a probe
        that cannot run."""
        return self.helpers is None or self.helpers.available(dev["uuid"])

    def warm(self, dev: dict) -> bool:
        """Would a probe of ``dev`` start at once (its helper is up), not after a HIP init?"""
        return self.helpers is None or self.helpers.alive(dev["uuid"])

    # ------------------------------------------------------------ parking (helper modes)
    def park(self, dev: dict) -> bool:
        """A tenant pod holds ``dev``: stop its probe helper (and take it out of the fabric
        helper's contexts), so the agent holds no HIP context, VRAM or process there."""
        return self.helpers is not None and self.helpers.park(dev["uuid"])

    def unpark(self, dev: dict, wait_s: float = 0.0) -> float | None:
        """``dev`` is pod-free again: restart its helper. With ``wait_s`` wait up to that long for
        it to come up; returns the ms waited (None: it was not parked)."""
        if self.helpers is None:
            return None
        t0 = time.perf_counter()
        h = self.helpers.unpark(dev["uuid"])
        if h is None:
            return None
        if wait_s > 0:
            h.ready.wait(wait_s)
        return (time.perf_counter() - t0) * 1e3

    def parked(self) -> set[str]:
        return self.helpers.parked() if self.helpers is not None else set()

    def restart_helper(self, dev: dict) -> None:
        """A fresh helper for ``dev`` (after a GPU reset its HIP context is stale)."""
        if self.helpers is not None:
            self.helpers.restart(dev["uuid"])

    def hip_devices(self) -> int:
        """GPUs this agent holds a HIP context on (in itself or its helpers)."""
        if self.mode == "helper":
            return sum(1 for k, v in self.helpers.snapshot().items() if k != "fabric" and v.get("alive"))
        return len(self.ordinals)  # helper-sim: no HIP anywhere (0)

    @property
    def fabric_warm_ms(self) -> float | None:
        """How long the fabric helper's warm ring took before it reported ready (None: no
        fabric helper up, or it did not warm)."""
        if self.helpers is None:
            return None
        return (self.helpers.snapshot().get("fabric") or {}).get("warmMs")

    PSS_TTL_S = 60.0

    def helpers_mem(self) -> tuple[int, int]:
        """(RSS, PSS) of the probe helpers together, bytes: the isolation's host-memory cost. RSS
        (``statm``: no page walk) is read on every call; PSS — shared pages split between the
        processes that map them, the fair share — needs ``smaps_rollup``, which walks the helper's
        page tables under its mmap lock (a probe allocating meanwhile would wait): at most once a
        minute, so a metrics scrape never stalls a claim."""
        page = os.sysconf("SC_PAGESIZE")
        rss = 0
        pids = self.helper_pids()
        for pid in pids:
            try:
                with open(f"/proc/{pid}/statm") as f:
                    rss += int(f.read().split()[1]) * page
            except (OSError, ValueError, IndexError):
                pass
        now = time.monotonic()
        cached = getattr(self, "_pss", None)
        if cached is None or now - cached[0] > self.PSS_TTL_S or cached[2] != pids:
            pss = 0
            for pid in pids:
                try:
                    with open(f"/proc/{pid}/smaps_rollup") as f:
                        for line in f:
                            if line.startswith("Pss:"):
                                pss += int(line.split()[1]) << 10
                                break
                except (OSError, ValueError, IndexError):
                    pass
            self._pss = cached = (now, pss, pids)
        return rss, cached[1]

    def prewake(self, devs: list[dict]) -> None:
        """The claim has chosen these GPUs and probes them in ~0.1-0.2 ms (ledger commit first):
        tell their helpers now, so each is running — not asleep in a blocking read — when its
        probe request arrives (probehost.SPIN_S)."""
        if self.helpers is None:
            return
        for d in devs:
            try:
                self.helpers.get(d["uuid"], d).notify("wake")
            except Exception:  # a helper being replaced: the probe reports it
                pass

    def helper_pids(self) -> set[int]:
        return self.helpers.pids() if self.helpers is not None else set()

    @staticmethod
    def _hooks(dev: dict) -> dict:
        """Fault-overlay hooks the helpers act out: probeCrash (the helper aborts, as HIP does on
        a GPU memory fault) and probeHang (the probe never returns)."""
        return {"crash": bool(simprobe.fault(dev, "probeCrash")),
                "hang": bool(simprobe.fault(dev, "probeHang"))}

    def _helper_call(self, dev: dict, op: str, args: dict, timeout: float) -> dict:
        """A probe-like request to ``dev``'s helper; failures of the helper itself come back as a
        failed result naming ProbeCrashed / ProbeTimeout / ProbeUnavailable."""
        from .probehost import HelperError, HelperTimeout
        idx = dev.get("index")
        try:
            h = self.helpers.get(dev["uuid"], dev)
            return h.call(op, args, timeout)
        except HelperTimeout:
            self.helpers.kill(dev["uuid"], f"{op} of GPU {idx} missed its {timeout:g} s deadline")
            return {"passed": False, "timedOut": True,
                    "error": f"ProbeTimeout: the {op} of GPU {idx} did not finish within "
                             f"{timeout:g} s (spec.probe.timeoutSeconds); its probe helper was "
                             f"killed"}
        except HelperError as e:
            return {"passed": False, "crashed": e.kind == "ProbeCrashed",
                    "error": f"{e.kind}: the probe helper of GPU {idx} {'died during the ' + op if e.kind == 'ProbeCrashed' else 'is unavailable'} ({e})"}
        except RuntimeError as e:  # the request itself raised in the helper
            return {"passed": False, "error": f"probe error: {e}"}

    def _one(self, dev: dict, opts: dict) -> dict:
        t0 = time.perf_counter()
        hbm = int(opts.get("hbmBytes", 1 << 30))
        mfma = bool(opts.get("mfma", True))
        if self.mode == "off" or not opts.get("enabled", True):
            return {"passed": True, "backend": "off", "ms": 0.0}
        if self.mode == "simulated":
            return simprobe.probe(dev, opts, self.sim_ms)
        # The HBM test and the MFMA phase normally overlap on two streams (~13 % shorter
        # probe). With performance floors the pool wants clean numbers: run them serially.
        floors = float(opts.get("minHbmGBps") or 0) > 0 or float(opts.get("minMfmaTflops") or 0) > 0
        if self.mode in HELPER_MODES:
            timeout = float(opts.get("timeoutSeconds") or DEFAULT_TIMEOUT_S)
            args = {"hipUUID": dev.get("hipUUID", ""), "hbmBytes": hbm, "mfma": mfma,
                    "gemmN": self.gemm_n if floors else self.overlap_gemm_n,
                    "overlap": 0 if floors else 1, "hooks": self._hooks(dev)}
            if self.mode == "helper-sim":
                args.update(dev=dev, opts=opts)
            res = self._helper_call(dev, "probe", args, timeout)
        else:
            ordinal = self.ordinals.get(str(dev.get("hipUUID", "")).lower())
            if ordinal is None:
                return {"passed": False, "backend": self.mode,
                        "error": f"device {dev.get('hipUUID')} not visible to HIP in this process",
                        "ms": 0.0}
            if self.mode == "inproc":
                res = self._hip.run(ordinal, hbm_bytes=hbm, mfma=mfma,
                                    gemm_n=self.gemm_n if floors else self.overlap_gemm_n,
                                    overlap=0 if floors else 1)
            else:
                cmd = [native_path("mi355x-probe"), "--device", str(ordinal), "--hbm-bytes",
                       str(hbm), "--gemm-n", str(self.gemm_n)] + ([] if mfma else ["--no-mfma"])
                p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
                try:
                    res = json.loads(p.stdout.strip().splitlines()[-1])
                except (ValueError, IndexError):
                    res = {"passed": False, "error": f"probe exited {p.returncode}: {p.stderr[-300:]}"}
        fault = simprobe.fault(dev, "probeFail")
        if fault and res.get("passed"):  # fault overlay also applies on top of real hardware
            res["passed"] = False
            res["error"] = "injected probe failure (fault overlay)"
        res["backend"] = self.mode
        res.setdefault("ms", (time.perf_counter() - t0) * 1e3)
        return res

    @staticmethod
    def apply_floors(res: dict, dev: dict, opts: dict) -> dict:
        """Performance floors (spec.probe.minHbmGBps / minMfmaTflops): a GPU that computes
        correctly but slowly (throttled clocks, degraded HBM stack, bad cooling) fails the probe.
        Fault overlay ``probeScale`` (0..1) scales the measured numbers to exercise this path."""
        scale = (dev.get("faults") or {}).get("probeScale") or dev.get("probeScale")
        hbm, mfma = res.get("hbm") or {}, res.get("mfma") or {}
        if scale:
            for part, key in ((hbm, "GBps"), (mfma, "tflops")):
                if isinstance(part.get(key), (int, float)):
                    part[key] = part[key] * float(scale)
        if not res.get("passed"):
            return res
        why = []
        floor_h = float(opts.get("minHbmGBps") or 0)
        if floor_h > 0 and float(hbm.get("GBps") or 0) < floor_h:
            why.append(f"HBM {float(hbm.get('GBps') or 0):.0f} GB/s < floor {floor_h:.0f}")
        floor_m = float(opts.get("minMfmaTflops") or 0)
        if floor_m > 0 and mfma.get("enabled", True) and float(mfma.get("tflops") or 0) < floor_m:
            why.append(f"MFMA {float(mfma.get('tflops') or 0):.0f} TFLOP/s < floor {floor_m:.0f}")
        if why:
            res["passed"] = False
            res["error"] = "PerformanceBelowFloor: " + "; ".join(why)
        return res

    @staticmethod
    def explain(res: dict) -> dict:
        """A failed probe names what failed (HBM bits, GEMM element/ABFT mismatches, CU census)."""
        if res.get("passed") or res.get("error"):
            return res
        why = []
        hbm, mfma, cus = res.get("hbm") or {}, res.get("mfma") or {}, res.get("cus") or {}
        if hbm.get("badBits"):
            why.append(f"HBMPatternMismatch: {hbm['badBits']} flipped bit(s), first at offset "
                       f"{hbm.get('firstBadOffset')}")
        if mfma.get("elementMismatches") or mfma.get("abftMismatches"):
            why.append(f"MFMAResultMismatch: {mfma.get('elementMismatches', 0)} element / "
                       f"{mfma.get('abftMismatches', 0)} ABFT mismatch(es)")
        if cus and not cus.get("ok", True):
            why.append(f"CUCensusFailed: {cus.get('mfmaVerified')}/{cus.get('expected')} CUs "
                       f"verified MFMA, per XCD {cus.get('perXcd')}, {cus.get('badWaves')} bad "
                       f"wave(s)")
        res["error"] = "; ".join(why) or "probe failed"
        return res

    def probe_many(self, devs: list[dict], opts: dict) -> list[dict]:
        def guarded(run):
            try:
                return run()
            except Exception as e:  # a probe must never take the agent down
                return {"passed": False, "backend": self.mode, "error": repr(e), "ms": 0.0}
        if len(devs) == 1:  # the caller is already off the event loop: no second thread hop
            return [self.apply_floors(self.explain(guarded(lambda: self._one(devs[0], opts))),
                                      devs[0], opts)]
        futs = [self.pool.submit(self._one, d, opts) for d in devs]
        return [self.apply_floors(self.explain(guarded(f.result)), d, opts)
                for d, f in zip(devs, futs)]

    def peer_ring(self, devs: list[dict], opts: dict) -> dict[str, dict]:
        """xGMI peer check in ring order (dev i -> dev i+1): for each sender uuid, the copy
        result {peer, GBps, passed[, error]}. Pairs run concurrently; the library serialises
        pairs that share a device. Empty when fewer than 2 GPUs or the mode cannot do it."""
        n = len(devs)
        if n < 2 or self.mode not in ("inproc", "simulated") + HELPER_MODES:
            return {}
        # 16 MiB per link: ~0.25 ms over one xGMI link, enough for a stable GB/s figure
        nbytes = int(opts.get("xgmiBytes") or (16 << 20))
        # a ring of 16 MiB links takes ~1 ms: a hung one is cut long before the probe's deadline
        timeout = min(float(opts.get("timeoutSeconds") or DEFAULT_TIMEOUT_S), RING_TIMEOUT_S)
        if self.mode in ("inproc",) + HELPER_MODES:
            ring = self._ring_whole(devs, nbytes, timeout)
            if ring is not None:
                return ring

        def one(i: int) -> tuple[str, dict]:
            src, dst = devs[i], devs[(i + 1) % n]
            faults = {**(src.get("faults") or {}), **src}
            # fault overlay on the sending GPU: xgmiPeerFail (every outgoing copy corrupted),
            # xgmiBadPeers [indices] (copies to those peers corrupted), xgmiPeerUnavailable (no
            # peer access: an infrastructure problem, not corruption)
            bad = bool(faults.get("xgmiPeerFail")) or \
                dst.get("index") in (faults.get("xgmiBadPeers") or [])
            if self.mode in ("simulated", "helper-sim") or bad or faults.get("xgmiPeerUnavailable"):
                r = simprobe.link(src, dst)
            elif self.mode == "helper":
                r = self._fabric_call(devs, "peer", {"src": src.get("hipUUID", ""),
                                                     "dst": dst.get("hipUUID", ""),
                                                     "bytes": nbytes}, timeout)
            else:
                a = self.ordinals.get(str(src.get("hipUUID", "")).lower())
                b = self.ordinals.get(str(dst.get("hipUUID", "")).lower())
                if a is None or b is None:
                    r = {"passed": False, "error": "peer device not visible to HIP"}
                else:
                    r = self._hip.peer(a, b, nbytes)
            r["peer"] = dst["uuid"]
            return src["uuid"], r
        out = {}
        for fut in [self.pool.submit(one, i) for i in range(n)]:
            try:
                u, r = fut.result()
                out[u] = r
            except Exception as e:  # never take the agent down
                log.warning("xGMI peer check failed: %r", e)
        return out

    def _fabric_call(self, devs: list[dict], op: str, args: dict, timeout: float) -> dict:
        """A request to the fabric helper. Its failure says nothing about any one link, so it
        comes back as a check that could not run (XGMIPeerCheckUnavailable, never a replace)."""
        from .probehost import HelperError, HelperTimeout
        try:
            h = self.helpers.fabric(devs)
            if self.helpers.resident_fabric and not h.ready.is_set():
                # the resident helper is (re)starting and warming its rings: this claim does not
                # wait for it — the check could not run; the next claim or idle recheck rings
                return {"passed": False, "error": "ProbeUnavailable: the xGMI fabric helper is "
                                                  "still starting"}
            return h.call(op, args, timeout)
        except HelperTimeout:
            self.helpers.kill("fabric", f"xGMI {op} missed its {timeout:g} s deadline")
            return {"passed": False, "error": f"ProbeTimeout: xGMI {op} did not finish within "
                                              f"{timeout:g} s; the fabric helper was killed"}
        except HelperError as e:
            return {"passed": False, "error": f"{e.kind}: fabric helper: {e}"}
        except RuntimeError as e:
            return {"passed": False, "error": f"xGMI {op} error: {e}"}

    def _ring_whole(self, devs: list[dict], nbytes: int, timeout: float) -> dict[str, dict] | None:
        """All links of the ring in one library call, concurrently (each GPU pair of an MI355X node
        has its own xGMI link): one copy time instead of n. None when a device is not visible to HIP
        or an injected link fault must be honoured — the pairwise path handles those."""
        for d in devs:
            f = {**(d.get("faults") or {}), **d}
            if f.get("xgmiPeerFail") or f.get("xgmiBadPeers") or f.get("xgmiPeerUnavailable"):
                return None
        if self.mode in HELPER_MODES:
            args = {"hipUUIDs": [d.get("hipUUID", "") for d in devs], "bytes": nbytes}
            if self.mode == "helper-sim":
                args["devs"] = devs
            r = self._fabric_call(devs, "peer_ring", args, timeout)
        else:
            if not hasattr(self._hip, "peer_ring"):
                return None
            ords = []
            for d in devs:
                o = self.ordinals.get(str(d.get("hipUUID", "")).lower())
                if o is None:
                    return None
                ords.append(o)
            r = self._hip.peer_ring(ords, nbytes)
        links = r.get("links")
        if not isinstance(links, list) or len(links) != len(devs):
            err = r.get("error") or "xGMI ring check returned no links"
            return {d["uuid"]: {"passed": False, "error": err, "peer": devs[(i + 1) % len(devs)]["uuid"]}
                    for i, d in enumerate(devs)}
        out = {}
        for i, (d, link) in enumerate(zip(devs, links)):
            link = dict(link)
            link["peer"] = devs[(i + 1) % len(devs)]["uuid"]
            out[d["uuid"]] = link
        return out

    # ------------------------------------------------------------ HBM scrubber kernels
    SWEEP_TIMEOUT_S = 60.0      # one window: ~3 ms at 4 GiB; seconds behind a driver clear
    SWEEP_MAP_TIMEOUT_S = 180.0  # mapping / freeing ~282 GiB: 0.2-6 s measured

    def sweep_window(self, dev: dict, offset: int, nbytes: int, reserve: int) -> dict:
        if self.mode == "simulated":
            return simprobe.sweep_window(dev, offset, nbytes, reserve)
        args = {"hipUUID": dev.get("hipUUID", ""), "offset": int(offset), "bytes": int(nbytes),
                "reserve": int(reserve), "keep": True}
        if self.mode in HELPER_MODES:
            if self.mode == "helper-sim":
                args["dev"] = dev
            return self._helper_call(dev, "sweep", args, self.SWEEP_TIMEOUT_S)
        o = self.ordinals.get(str(dev.get("hipUUID", "")).lower())
        if o is None:
            return {"passed": False, "error": "device not visible to HIP"}
        return self._hip.hbm_sweep(o, offset, nbytes, reserve, keep=True)

    def sweep_alloc(self, dev: dict, reserve: int) -> int:
        """The scrubber's big buffer: 1 allocated, 0 already held, < 0 failed."""
        if self.mode == "simulated":
            return 1
        if self.mode in HELPER_MODES:
            r = self._helper_call(dev, "sweep_alloc", {"hipUUID": dev.get("hipUUID", ""),
                                                       "reserve": int(reserve)},
                                  self.SWEEP_MAP_TIMEOUT_S)
            return r if isinstance(r, int) else -1
        o = self.ordinals.get(str(dev.get("hipUUID", "")).lower())
        return -1 if o is None else self._hip.sweep_alloc(o, reserve)

    def sweep_release(self, dev: dict) -> None:
        if self.mode == "simulated":
            return
        if self.mode in HELPER_MODES:
            # a helper that died meanwhile took the buffer with it: nothing left to free
            self._helper_call(dev, "sweep_release", {"hipUUID": dev.get("hipUUID", "")},
                              self.SWEEP_MAP_TIMEOUT_S)
            return
        o = self.ordinals.get(str(dev.get("hipUUID", "")).lower())
        if o is not None:
            self._hip.sweep_release(o)

    def warm_arena(self, dev: dict, hbm_bytes: int = 1 << 30) -> None:
        """Run one default-sized probe so the device's probe arena is allocated and kept (the
        library's trim skips it while an HBM sweep is held and for 30 s after its release)."""
        if self.mode == "inproc":
            o = self.ordinals.get(str(dev.get("hipUUID", "")).lower())
            if o is not None:
                self._hip.run(o, hbm_bytes=hbm_bytes, gemm_n=self.gemm_n)
        elif self.mode in HELPER_MODES:
            self._helper_call(dev, "warm", {"hipUUID": dev.get("hipUUID", ""),
                                            "hbmBytes": hbm_bytes, "gemmN": self.gemm_n},
                              self.SWEEP_TIMEOUT_S)

    def _trim_loop(self) -> None:
        period = max(0.05, min(1.0, self._trim_idle_ms / 4e3))
        while not self._trim_stop.wait(period):
            try:
                self._hip.trim(self._trim_idle_ms)
            except Exception as e:  # never let housekeeping kill the agent
                log.warning("probe arena trim failed: %s", e)

    def close(self) -> None:
        if self.mode == "inproc":
            self._trim_stop.set()
        if self.helpers is not None:
            self.helpers.stop()
        self.pool.shutdown(wait=False)


def default_mode(backend: str) -> str:
    env = os.environ.get("GPUPOOL_PROBE_MODE")
    if env:
        return env
    return "simulated" if backend == "fake" else "helper"

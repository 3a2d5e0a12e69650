"""Claim-time readiness probes (the MI355X replacement of `nvidia-smi` in a pod).

Modes:
  inproc     — libmi355x_probe.so loaded once in the agent; HIP contexts warmed at start so a
               claim pays only the kernels (HBM pattern fill/verify + bf16 MFMA GEMM checks);
               GPUs are probed concurrently (ctypes drops the GIL).
  subprocess — `mi355x-probe --device N` per GPU: process isolation (a faulting probe cannot take
               the agent down) at the cost of HIP initialisation per probe.
  simulated  — for the fake backend on CPU-only hosts: a fixed latency and a result that fails
               only when the fault overlay sets ``probeFail``. Never used with real GPUs.
  off        — no probe (result passes with backend "off").
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

log = logging.getLogger("gpupool.agent.prober")


class Prober:
    def __init__(self, mode: str = "inproc", sim_ms: float = 20.0, gemm_n: int = 4096,
                 max_workers: int = 16, arena_idle_s: float = 10.0, overlap_gemm_n: int = 2048):
        self.mode = mode
        self.sim_ms = sim_ms
        self.gemm_n = gemm_n                  # serial probe (pools with performance floors)
        # the claim-time probe's GEMM when it overlaps the HBM pattern test: the element check,
        # ABFT and the all-CU census run whatever its size, and a smaller GEMM takes less HBM
        # bandwidth from the pattern test (profiles/r4_probe_gemm_overlap_ab.json)
        self.overlap_gemm_n = overlap_gemm_n
        self.pool = cf.ThreadPoolExecutor(max_workers=max_workers, thread_name_prefix="probe")
        self.ordinals: dict[str, int] = {}
        self.init_ms = 0.0
        t0 = time.perf_counter()
        if mode == "inproc":
            from ..ops import probe as hip_probe
            self._hip = hip_probe
            n = hip_probe.init()
            self.ordinals = hip_probe.hip_uuid_map()
            log.info("HIP probe initialised: %d device(s) %s", n, sorted(self.ordinals))
            # probe arenas stay allocated between back-to-back claims (scale-up bursts) and are
            # handed back to the GPU's workloads once idle for arena_idle_s
            self._trim_stop = threading.Event()
            self._trim_idle_ms = int(arena_idle_s * 1e3)
            threading.Thread(target=self._trim_loop, daemon=True, name="probe-trim").start()
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

    def _one(self, dev: dict, opts: dict) -> dict:
        t0 = time.perf_counter()
        hbm = int(opts.get("hbmBytes", 1 << 30))
        mfma = bool(opts.get("mfma", True))
        if self.mode == "off" or not opts.get("enabled", True):
            return {"passed": True, "backend": "off", "ms": 0.0}
        if self.mode == "simulated":
            time.sleep(self.sim_ms / 1e3)
            fail = bool((dev.get("faults") or {}).get("probeFail")) or bool(dev.get("probeFail"))
            # nominal numbers = the measured MI355X probe (profiles/r1c_probe_gemm_ab_real.json)
            res = {"passed": not fail, "backend": "simulated",
                   "hbm": {"ok": not fail, "GBps": 4900.0, "bytes": hbm},
                   "mfma": {"ok": not fail, "tflops": 1200.0 if mfma else 0.0, "enabled": mfma}}
            if mfma:  # the CU census: every CU of this (partition of the) GPU proves its MFMA pipes
                cus = int((dev.get("asic") or {}).get("computeUnits") or 256)
                dead = int(dev.get("cuFault") or 0)
                res["cus"] = {"expected": cus, "mfmaVerified": cus - dead, "badWaves": dead * 8,
                              "ok": dead == 0}
                if dead and not fail:
                    res["passed"] = False
            if fail:
                res["error"] = "injected probe failure (fault overlay)"
            res["ms"] = (time.perf_counter() - t0) * 1e3
            return res
        ordinal = self.ordinals.get(str(dev.get("hipUUID", "")).lower())
        if ordinal is None:
            return {"passed": False, "backend": self.mode,
                    "error": f"device {dev.get('hipUUID')} not visible to HIP in this process",
                    "ms": 0.0}
        if self.mode == "inproc":
            # The HBM test and the MFMA phase normally overlap on two streams (~13 % shorter
            # probe). With performance floors the pool wants clean numbers: run them serially.
            floors = float(opts.get("minHbmGBps") or 0) > 0 or float(opts.get("minMfmaTflops") or 0) > 0
            res = self._hip.run(ordinal, hbm_bytes=hbm, mfma=mfma,
                                gemm_n=self.gemm_n if floors else self.overlap_gemm_n,
                                overlap=0 if floors else 1)
        else:
            cmd = [native_path("mi355x-probe"), "--device", str(ordinal), "--hbm-bytes", str(hbm),
                   "--gemm-n", str(self.gemm_n)] + ([] if mfma else ["--no-mfma"])
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            try:
                res = json.loads(p.stdout.strip().splitlines()[-1])
            except (ValueError, IndexError):
                res = {"passed": False, "error": f"probe exited {p.returncode}: {p.stderr[-300:]}"}
        fault = (dev.get("faults") or {}).get("probeFail") or dev.get("probeFail")
        if fault:  # fault overlay also applies on top of real hardware
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
        if n < 2 or self.mode not in ("inproc", "simulated"):
            return {}
        # 16 MiB per link: ~0.25 ms over one xGMI link, enough for a stable GB/s figure
        nbytes = int(opts.get("xgmiBytes") or (16 << 20))
        if self.mode == "inproc":
            ring = self._ring_inproc(devs, nbytes)
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
            if faults.get("xgmiPeerUnavailable"):
                r = {"passed": False, "canAccessPeer": False, "error": "hipDeviceCanAccessPeer=0"}
            elif self.mode == "simulated" or bad:
                r = {"passed": not bad, "canAccessPeer": True,
                     "GBps": 64.0 * float(faults.get("probeScale") or 1.0),
                     "badBits": 0 if not bad else 1}
                if bad:
                    r["error"] = "injected xGMI peer failure (fault overlay)"
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

    def _ring_inproc(self, devs: list[dict], nbytes: int) -> dict[str, dict] | None:
        """All links of the ring in one library call, concurrently (each GPU pair of an MI355X node
        has its own xGMI link): one copy time instead of n. None when a device is not visible to HIP
        or an injected link fault must be honoured — the pairwise path handles those."""
        if not hasattr(self._hip, "peer_ring"):
            return None
        ords = []
        for d in devs:
            o = self.ordinals.get(str(d.get("hipUUID", "")).lower())
            f = {**(d.get("faults") or {}), **d}
            if o is None or f.get("xgmiPeerFail") or f.get("xgmiBadPeers") or \
                    f.get("xgmiPeerUnavailable"):
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

    def warm_arena(self, ordinal: int, hbm_bytes: int = 1 << 30) -> None:
        """Run one default-sized probe so the device's probe arena is allocated and kept (the
        library's trim skips it while an HBM sweep is held and for 30 s after its release)."""
        if self.mode == "inproc":
            self._hip.run(ordinal, hbm_bytes=hbm_bytes, gemm_n=self.gemm_n)

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
        self.pool.shutdown(wait=False)


def default_mode(backend: str) -> str:
    env = os.environ.get("GPUPOOL_PROBE_MODE")
    if env:
        return env
    return "simulated" if backend == "fake" else "inproc"

"""Simulated probe kernels for the fake device backend on CPU-only hosts.

The same results the gfx950 kernels report (probe.hip), timed like them, failing only where the
fault overlay says so. Used by the agent's ``simulated`` probe mode (in process) and by the
``helper-sim`` probe helpers (probehost.py), so the helper machinery — child processes, deadlines,
crash handling — is exercised on CPU with the exact results the in-process simulation gives.
"""
from __future__ import annotations

import time

# nominal numbers = the measured MI355X probe (profiles/r1c_probe_gemm_ab_real.json)
SIM_HBM_GBPS = 4900.0
SIM_MFMA_TFLOPS = 1200.0
SIM_XGMI_GBPS = 64.0
SIM_SWEEP_GBPS = 6000.0


def fault(dev: dict, key: str):
    """A fault-overlay key of one device (the overlay merges device keys into the snapshot;
    older fixtures nest them under ``faults``)."""
    v = dev.get(key)
    return v if v is not None else (dev.get("faults") or {}).get(key)


def probe(dev: dict, opts: dict, sim_ms: float) -> dict:
    t0 = time.perf_counter()
    hbm = int(opts.get("hbmBytes", 1 << 30))
    mfma = bool(opts.get("mfma", True))
    time.sleep(sim_ms / 1e3)
    fail = bool(fault(dev, "probeFail"))
    res = {"passed": not fail, "backend": "simulated",
           "hbm": {"ok": not fail, "GBps": SIM_HBM_GBPS, "bytes": hbm},
           "mfma": {"ok": not fail, "tflops": SIM_MFMA_TFLOPS if mfma else 0.0, "enabled": mfma}}
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


def sweep_window(dev: dict, offset: int, window: int, reserve: int) -> dict:
    """One HBM scrub window: nominal timing of the real kernels (~6 TB/s over 4 passes); flipped
    bits where the overlay's ``hbmBadOffset`` (a byte offset) falls inside the window."""
    span = max(window, int(dev.get("memTotalBytes") or 288e9) - reserve)
    off = offset % span
    n = min(window, span - off)
    time.sleep(min(0.05, 4 * n / 6e12))
    bad_at = fault(dev, "hbmBadOffset")
    bad = 1 if bad_at is not None and off <= int(bad_at) < off + n else 0
    return {"passed": not bad, "offset": off, "bytes": n, "span": span, "badBits": bad,
            "firstBadOffset": int(bad_at) if bad else None, "GBps": SIM_SWEEP_GBPS, "ms": 0.0}


def link(src: dict, dst: dict) -> dict:
    """One simulated xGMI peer copy src -> dst (overlay: xgmiPeerFail, xgmiBadPeers [indices],
    xgmiPeerUnavailable, probeScale)."""
    faults = {**(src.get("faults") or {}), **src}
    bad = bool(faults.get("xgmiPeerFail")) or dst.get("index") in (faults.get("xgmiBadPeers") or [])
    if faults.get("xgmiPeerUnavailable"):
        return {"passed": False, "canAccessPeer": False, "error": "hipDeviceCanAccessPeer=0"}
    r = {"passed": not bad, "canAccessPeer": True,
         "GBps": SIM_XGMI_GBPS * float(faults.get("probeScale") or 1.0), "badBits": 0 if not bad else 1}
    if bad:
        r["error"] = "injected xGMI peer failure (fault overlay)"
    return r

#!/usr/bin/env python3
"""Claim-time probe after an idle gap vs back to back: the bench's claims come ~1.2 s apart (the
amd-smi ground-truth read sits between them) and measure the probe slower than an in-process loop.
Each round sleeps ``gap`` seconds, runs one probe (afterIdle) and then one more (warm), at the
agent's claim-time options (1 GiB, 2048^3 overlapped GEMM), rotating the probe variants between
rounds so none always follows another. Variants are probe options, e.g. zeroInKernel 1 (counters
reset inside the first kernels) vs 0 (memsets + a cross-stream event ahead of the first fill), or
hbmFirst 1 (MFMA phase enqueued after the whole HBM test) vs 2 (after the first fill).

    python scripts/probe_idle_gap_ab.py --rounds 24 --gap 1.2 \\
        --variant zeroInKernel=1 --variant zeroInKernel=0 > gpurun_out/probe_idle_gap_ab.json
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=24)
ap.add_argument("--gap", type=float, default=1.2)
ap.add_argument("--variant", action="append", default=[],
                help="comma-separated key=int probe options (repeat: one per variant)")
a = ap.parse_args()
variants = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in v.split(",") if kv)
            for v in (a.variant or ["zeroInKernel=1", "zeroInKernel=0"])]
names = [",".join(f"{k}={v}" for k, v in o.items()) for o in variants]
probe.init()


def timed_run(dev: int, hbm_bytes: int, gemm_n: int, **o: int) -> dict:
    """probe.run's steps (options JSON, the ctypes call, the reply JSON), each timed."""
    t0 = time.perf_counter()
    arg = probe._run_opts(hbm_bytes, True, gemm_n, 2, 1, 256, tuple(sorted(o.items())))
    t1 = time.perf_counter()
    p = probe.lib().mi355x_probe_run(dev, arg)
    t2 = time.perf_counter()
    r = json.loads(ctypes.string_at(p).decode())
    probe.lib().mi355x_probe_free(p)
    t3 = time.perf_counter()
    r["py"] = {"argMs": (t1 - t0) * 1e3, "callMs": (t2 - t1) * 1e3, "replyMs": (t3 - t2) * 1e3,
               "pyMs": (t3 - t0) * 1e3}
    return r

opts = dict(hbm_bytes=1 << 30, gemm_n=2048, overlap=1)
for o in variants:
    assert probe.run(0, **opts, **o)["passed"]
res: dict[str, list[dict]] = {}
for i in range(a.rounds):
    vi = (i + i // len(variants)) % len(variants)
    time.sleep(a.gap)
    r = timed_run(0, 1 << 30, 2048, overlap=1, **variants[vi])   # first probe after the idle gap
    w = timed_run(0, 1 << 30, 2048, overlap=1, **variants[vi])   # the next one, back to back
    for k, x in ((f"afterIdle {names[vi]}", r), (f"warm {names[vi]}", w)):
        assert x["passed"] and x["cus"]["ok"], x
        ph = x["phases"]
        res.setdefault(k, []).append({
            "ms": x["ms"], **x["py"], "reportMs": x.get("reportMs", 0.0), "hbmKernelMs": x["hbm"]["ms"], "writeGBps": x["hbm"]["writeGBps"],
            "readGBps": x["hbm"]["readGBps"], "launchMs": ph["launchMs"], "setupMs": ph["setupMs"],
            "allocMs": ph["allocMs"], "hbmWallMs": ph["hbmWallMs"], "mfmaWallMs": ph["mfmaWallMs"],
            "arenaReused": ph["arenaReused"]})
probe.trim(0)
print(json.dumps({"rounds": a.rounds, "gap_s": a.gap, "options": opts, "variants": names, "median": {
    k: {m: round(statistics.median(x[m] for x in rs), 4) for m in rs[0] if m != "arenaReused"}
    for k, rs in sorted(res.items())}, "samples": res}, indent=1))

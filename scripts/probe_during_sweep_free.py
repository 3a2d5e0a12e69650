#!/usr/bin/env python3
"""Does mapping / unmapping the scrubber's ~282 GiB sweep buffer stall a claim-time probe running
at the same time on the same GPU? Claim-time probes (1 GiB, 2048^3 overlapped), one every ~10 ms
(a burst of claims), alone, while another thread frees the sweep buffer (4 GiB chunks) and while it
allocates it again right after the free (the driver is still clearing the freed VRAM: the slow
case; sweep_alloc now gives up with -3 when a chunk maps slower than 20 ms). ``GPUPOOL_SWEEP_NO_YIELD=1``
turns off the chunk loop's yielding to running probes and that give-up (run the script once with,
once without).

    python scripts/probe_during_sweep_free.py > gpurun_out/probe_during_sweep_free.json
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

probe.init()
opts = dict(hbm_bytes=1 << 30, gemm_n=2048, overlap=1)
last_rc = None
assert probe.run(0, **opts)["passed"]


def probes_while(fn, gap_s: float = 0.01) -> tuple[list[float], float]:
    global last_rc
    out: list[float] = []
    box = {}

    def work():
        t = time.perf_counter()
        box["rc"] = fn()
        box["ms"] = (time.perf_counter() - t) * 1e3
    th = threading.Thread(target=work)
    th.start()
    while th.is_alive():
        t = time.perf_counter()
        r = probe.run(0, **opts)
        assert r["passed"], r
        out.append((time.perf_counter() - t) * 1e3)  # wall, incl. any wait for the device
        time.sleep(gap_s)
    th.join()
    last_rc = box["rc"]
    return out, box["ms"]


def stats(xs: list[float]) -> dict:
    return {"n": len(xs), "p50": round(statistics.median(xs), 3), "max": round(max(xs), 3),
            "over2ms": sum(1 for x in xs if x > 2.0)} if xs else {"n": 0}


res = {"yield": os.environ.get("GPUPOOL_SWEEP_NO_YIELD") is None,
       "alone": stats([probe.run(0, **opts)["ms"] for _ in range(100)])}
for rnd in range(2):
    t = time.perf_counter()
    rc = probe.sweep_alloc(0, 4 << 30)
    res[f"first_alloc_{rnd}"] = {"rc": rc, "ms": round((time.perf_counter() - t) * 1e3, 1)}
    if rc < 0:  # the driver is still clearing what an earlier process freed: wait and retry once
        time.sleep(10)
        rc = probe.sweep_alloc(0, 4 << 30)
        res[f"first_alloc_retry_{rnd}"] = {"rc": rc}
    assert rc >= 0, res
    d, ms = probes_while(lambda: probe.sweep_release(0))
    res[f"during_free_{rnd}"] = {**stats(d), "freeMs": round(ms, 1)}
    d, ms = probes_while(lambda: probe.sweep_alloc(0, 4 << 30))  # right after the free: clearing
    res[f"during_alloc_after_free_{rnd}"] = {**stats(d), "allocMs": round(ms, 1), "rc": last_rc}
    d, ms = probes_while(lambda: probe.sweep_release(0))
    res[f"during_free_b_{rnd}"] = {**stats(d), "freeMs": round(ms, 1)}
    time.sleep(8)  # the driver finishes clearing
    d, ms = probes_while(lambda: probe.sweep_alloc(0, 4 << 30))  # after the clear: the scrubber's case
    res[f"during_alloc_cleared_{rnd}"] = {**stats(d), "allocMs": round(ms, 1), "rc": last_rc}
    assert probe.sweep_release(0) >= 0
    time.sleep(8)
probe.trim(0)
print(json.dumps(res, indent=1))

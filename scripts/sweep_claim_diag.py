#!/usr/bin/env python3
"""Diagnose how the HBM scrubber's big sweep buffer interacts with a claim-time probe on one
MI355X: times sweep alloc / windows / free, then a probe issued (a) right after the free returned,
(b) while the free runs on another thread, (c) with the probe arena trimmed first; samples
hipMemGetInfo-visible free HBM (via a 1 MiB probe's report) over time after the free."""
from __future__ import annotations

import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402


def t(fn, *a, **k):
    t0 = time.perf_counter()
    r = fn(*a, **k)
    return r, round((time.perf_counter() - t0) * 1e3, 2)


def main() -> None:
    out: dict = {}
    probe.init()
    r, ms = t(probe.run, 0)
    out["probe_warm_ms"] = ms
    for case in ("after_free", "during_free", "trimmed_after_free", "during_alloc"):
        rec: dict = {}
        if case == "trimmed_after_free":
            probe.trim(0)
        if case == "during_alloc":
            th = threading.Thread(target=lambda: rec.__setitem__("alloc", t(probe.sweep_alloc, 0, 4 << 30)))
            th.start()
            time.sleep(0.05)
            r, ms = t(probe.run, 0)
            rec["probe_ms"], rec["probe_passed"] = ms, r.get("passed")
            th.join()
            rec["alloc_ms"] = rec.pop("alloc")[1]
            _, rec["free_ms"] = t(probe.sweep_release, 0)
            out[case] = rec
            print(case, rec, flush=True)
            continue
        _, rec["alloc_ms"] = t(probe.sweep_alloc, 0, 4 << 30)
        for i in range(2):
            w, ms = t(probe.hbm_sweep, 0, i * (16 << 30), 16 << 30, 4 << 30, keep=True)
            rec[f"window{i}_ms"] = ms
            rec[f"window{i}_GBps"] = w.get("GBps")
        if case == "during_free":
            th = threading.Thread(target=lambda: rec.__setitem__("free", t(probe.sweep_release, 0)))
            th.start()
            time.sleep(0.05)
            r, ms = t(probe.run, 0)
            rec["probe_ms"], rec["probe_passed"] = ms, r.get("passed")
            th.join()
            rec["free_ms"] = rec.pop("free")[1]
        else:
            _, rec["free_ms"] = t(probe.sweep_release, 0)
            r, ms = t(probe.run, 0)
            rec["probe_ms"], rec["probe_passed"] = ms, r.get("passed")
            rec["probe_detail"] = {k: r.get(k) for k in ("ms", "allocMs", "phases") if k in r}
        for j in range(3):
            r, ms = t(probe.run, 0)
            rec[f"probe_again{j}_ms"] = ms
        out[case] = rec
        print(case, rec, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Does the HBM pattern test read HBM or the 256 MiB Infinity Cache? The probe writes a pattern
over ``hbmBytes`` and reads it back in the same order; a buffer that fits the die-level cache
could be verified from the cache instead of the DRAM cells. The test's write+read bandwidth by
buffer size answers it: HBM tops out near 6.3 TB/s (MI355X_MICROARCH.md §HBM), so a size
reported well above that is (partly) served on-die. Median of ``--reps`` probes, HBM phase only.

    python scripts/hbm_cache_residency.py > gpurun_out/hbm_cache_residency.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=7)
args = ap.parse_args()
probe.init()
rows = {}
for mib in (32, 64, 128, 192, 256, 384, 512, 1024, 2048, 4096):
    gbps = []
    for _ in range(args.reps):
        r = probe.run(0, hbm_bytes=mib << 20, mfma=False, patterns=2)
        assert r["passed"], r
        gbps.append(r["hbm"]["GBps"])
    rows[str(mib)] = {"GBps_median": round(statistics.median(gbps), 1), "GBps_max": round(max(gbps), 1)}
    print(json.dumps({"MiB": mib, **rows[str(mib)]}), file=sys.stderr, flush=True)
probe.trim(0)
print(json.dumps({"reps": args.reps, "by_MiB": rows}, indent=1))

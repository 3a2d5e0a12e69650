"""In-process A/B (cdna_hip_programming.md §5.4 rule 24): the claim-time probe with its two streams
at equal priority vs. the HBM-test stream at the highest and the MFMA stream at the lowest queue
priority (``streamPriority``). The HBM test is the probe's critical path; the question is whether
the dispatcher, told so, gives the GEMM beside it less of the bandwidth.

    python scripts/probe_prio_ab.py [rounds] > gpurun_out/probe_prio_ab.json
"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 15
probe.init()
for p in (0, 1):
    assert probe.run(0, hbm_bytes=1 << 30, streamPriority=p)["passed"]
res: dict[str, list[dict]] = {}
for _ in range(rounds):
    for p in (0, 1):
        r = probe.run(0, hbm_bytes=1 << 30, streamPriority=p)
        assert r["passed"] and r["phases"]["arenaReused"], r
        res.setdefault(f"priority{p}", []).append(
            {"ms": r["ms"], "hbmWallMs": r["phases"]["hbmWallMs"], "mfmaWallMs": r["phases"]["mfmaWallMs"],
             "hbmGBps": r["hbm"]["GBps"], "tflops": r["mfma"]["tflops"]})
print(json.dumps({"rounds": rounds, "median": {
    k: {m: round(statistics.median(x[m] for x in rs), 3) for m in rs[0]} for k, rs in res.items()},
    "min_ms": {k: round(min(x["ms"] for x in rs), 3) for k, rs in res.items()}}, indent=1))

#!/usr/bin/env python3
"""HBM pattern-test kernel layout A/B (probe option ``hbmLayout``): grid-stride (0: each unrolled
access of a thread a whole grid apart) vs tiled (1: a workgroup's unrolled accesses cover one
contiguous 16 KiB tile), across (fill, verify) workgroups per CU; then the full claim-time probe
(2048^3 MFMA phase beside it) for each layout at the default grid. Interleaved rounds, one process.

    python scripts/probe_hbm_layout_ab.py [rounds] > gpurun_out/probe_hbm_layout_ab.json
"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
hbm = 1 << 30
grids = [(0, 1, 3), (1, 1, 3), (1, 2, 3), (1, 1, 4), (1, 2, 4), (1, 4, 4), (1, 1, 2), (0, 2, 4)]
probe.init()
res: dict[str, list[dict]] = {}
for layout, f, v in grids:  # warm every variant
    assert probe.run(0, hbm_bytes=hbm, mfma=False, hbmLayout=layout, hbmFillBlocksPerCU=f,
                     hbmVerifyBlocksPerCU=v)["passed"]
for r in range(rounds):
    order = grids if r % 2 == 0 else list(reversed(grids))
    for layout, f, v in order:
        x = probe.run(0, hbm_bytes=hbm, mfma=False, hbmLayout=layout, hbmFillBlocksPerCU=f,
                      hbmVerifyBlocksPerCU=v)
        assert x["passed"], x
        res.setdefault(f"layout{layout}_fill{f}_verify{v}", []).append(x["hbm"])
    for layout in ((0, 1) if r % 2 == 0 else (1, 0)):
        x = probe.run(0, hbm_bytes=hbm, gemm_n=2048, overlap=1, hbmLayout=layout)
        assert x["passed"], x
        res.setdefault(f"claimProbe_layout{layout}", []).append({"ms": x["ms"], **x["hbm"]})
out = {}
for k, rs in res.items():
    out[k] = {m: round(statistics.median(x[m] for x in rs), 3) for m in ("writeGBps", "readGBps", "GBps", "ms")
              if m in rs[0]}
probe.trim(0)
print(json.dumps({"rounds": rounds, "hbmBytes": hbm, "median": out}, indent=1))

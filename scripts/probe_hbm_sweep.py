"""HBM pattern-test grid sweep: (fill, verify) workgroups per CU, interleaved rounds in ONE
process (cdna_hip_programming.md §5.4 rule 24). Usage: probe_hbm_sweep.py "1:3,3:3,8:8" [rounds]"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

configs = [tuple(int(v) for v in c.split(":")) for c in
           (sys.argv[1] if len(sys.argv) > 1 else "1:3,3:3,8:8").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
probe.init()
res: dict[str, list[dict]] = {}
for _ in range(rounds):
    for f, v in configs:
        r = probe.run(0, hbm_bytes=1 << 30, mfma=False, hbmFillBlocksPerCU=f, hbmVerifyBlocksPerCU=v)
        assert r["passed"], r
        res.setdefault(f"fill{f}_verify{v}", []).append(r["hbm"])
print(json.dumps({k: {m: round(statistics.median(x[m] for x in rs), 1)
                      for m in ("writeGBps", "readGBps", "GBps")} for k, rs in res.items()}, indent=1))

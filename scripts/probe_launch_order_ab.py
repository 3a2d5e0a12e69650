#!/usr/bin/env python3
"""Claim-time probe A/B: enqueue the HBM test before or after the MFMA phase (probe option
``hbmFirst``). The HBM kernels are the probe's critical path; the MFMA phase is ~20 HIP API calls
of enqueue work. Interleaved rounds in one process at the agent's claim-time options (1 GiB,
2048^3 overlapped GEMM); reports total probe ms, the host enqueue time (phases.launchMs) and the
HBM kernels' own time.

    python scripts/probe_launch_order_ab.py [rounds] > gpurun_out/probe_launch_order_ab.json
"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 25
hbm = 1 << 30
probe.init()
res: dict[str, list[dict]] = {"hbmFirst": [], "mfmaFirst": []}
for hf in (1, 0):
    assert probe.run(0, hbm_bytes=hbm, gemm_n=2048, overlap=1, hbmFirst=hf)["passed"]
for i in range(rounds):
    for hf in ((1, 0) if i % 2 == 0 else (0, 1)):
        r = probe.run(0, hbm_bytes=hbm, gemm_n=2048, overlap=1, hbmFirst=hf)
        res["hbmFirst" if hf else "mfmaFirst"].append({
            "ms": r["ms"], "launchMs": r["phases"]["launchMs"], "hbmKernelMs": r["hbm"]["ms"],
            "hbmWallMs": r["phases"]["hbmWallMs"], "mfmaWallMs": r["phases"]["mfmaWallMs"],
            "passed": r["passed"], "cusOk": (r.get("cus") or {}).get("ok")})
probe.trim(0)
summary = {k: {m: round(statistics.median(x[m] for x in rs), 4)
               for m in ("ms", "launchMs", "hbmKernelMs", "hbmWallMs", "mfmaWallMs")}
           | {"all_passed": all(x["passed"] and x["cusOk"] for x in rs)}
           for k, rs in res.items()}
print(json.dumps({"rounds": rounds, "hbmBytes": hbm, "gemmN": 2048, "summary": summary,
                  "samples": res}, indent=1))

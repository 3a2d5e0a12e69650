#!/usr/bin/env python3
"""Claim-time probe A/B: the MFMA phase's GEMM size when it overlaps the HBM pattern test.

The claim-time probe runs the 1 GiB HBM pattern test and the MFMA phase on two streams. The GEMM
competes with the pattern test for HBM (profiles/r3x_probe_size_sweep.json: 5.38 TB/s beside a
4096^3 GEMM, 5.94 TB/s beside 2048^3). What the MFMA phase must prove does not depend on the GEMM
size: the 256^3 element-exact check, the ABFT-checked big GEMM and the CU census (every CU runs
MFMA waves, its own kernel) all run either way. So the question is only the probe's wall time —
and that coverage really is unchanged. Interleaved rounds, one process, the agent's options.

    python scripts/probe_gemm_overlap_ab.py [rounds] > gpurun_out/probe_gemm_overlap_ab.json
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
res: dict[str, list[dict]] = {"gemm2048": [], "gemm4096": []}
for g in (2048, 4096):  # warm both code paths and the arena
    assert probe.run(0, hbm_bytes=hbm, gemm_n=g, overlap=1)["passed"]
for i in range(rounds):
    for g in ((2048, 4096) if i % 2 == 0 else (4096, 2048)):
        r = probe.run(0, hbm_bytes=hbm, gemm_n=g, overlap=1)
        cus = r.get("cus") or {}
        res[f"gemm{g}"].append({
            "ms": r["ms"], "hbmGBps": r["hbm"]["GBps"], "tflops": r["mfma"]["tflops"],
            "passed": r["passed"], "cusVerified": cus.get("mfmaVerified"),
            "cusExpected": cus.get("expected"), "gemmTiles": cus.get("gemmTiles"),
            "abftMismatches": r["mfma"].get("abftMismatches"),
            "elementMismatches": r["mfma"].get("elementMismatches")})
probe.trim(0)
summary = {}
for k, rs in res.items():
    summary[k] = {m: round(statistics.median(x[m] for x in rs), 3) for m in ("ms", "hbmGBps", "tflops")}
    summary[k]["ms_p90"] = round(sorted(x["ms"] for x in rs)[int(0.9 * (len(rs) - 1))], 3)
    summary[k]["all_passed"] = all(x["passed"] for x in rs)
    summary[k]["all_cus_verified"] = all(x["cusVerified"] == x["cusExpected"] for x in rs)
    summary[k]["gemm_tiles"] = rs[0]["gemmTiles"]
print(json.dumps({"rounds": rounds, "hbmBytes": hbm, "overlap": True, "summary": summary,
                  "samples": res}, indent=1))

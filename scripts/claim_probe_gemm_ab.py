#!/usr/bin/env python3
"""The claim-time probe (1 GiB x 2 patterns of HBM test beside the 2048^3 MFMA phase, two streams)
with each GEMM K-loop, interleaved in one process: does the loop change the probe's length, and what
does each cost beside the HBM stream? Prints medians of the probe's ms, its HBM GB/s and the GEMM's
TFLOP/s per ``gemmPipe``.

    python scripts/claim_probe_gemm_ab.py [rounds] [pipes] > gpurun_out/claim_probe_gemm_ab.json
"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 30
pipes = [int(p) for p in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "2"])]
probe.init()
for p in pipes:  # warm each variant's code object and the arena
    probe.run(0, hbm_bytes=1 << 30, gemm_n=2048, overlap=1, gemmPipe=p)
res: dict[str, dict[str, list[float]]] = {}
for r in range(rounds):
    for p in (pipes if r % 2 == 0 else pipes[::-1]):
        out = probe.run(0, hbm_bytes=1 << 30, gemm_n=2048, overlap=1, gemmPipe=p)
        assert out["passed"], out
        d = res.setdefault(f"pipe{p}", {"ms": [], "hbm_GBps": [], "gemm_tflops": []})
        d["ms"].append(out["ms"])
        d["hbm_GBps"].append(out["hbm"]["GBps"])
        d["gemm_tflops"].append(out["mfma"]["tflops"])
probe.trim(0)
print(json.dumps({"rounds": rounds, "summary": {k: {m: round(statistics.median(v), 3) for m, v in d.items()}
                                               for k, d in res.items()}}, indent=1))

#!/usr/bin/env python3
"""K-loop variants of the probe's 256x256 GEMM, interleaved in one process (§5.4 rule 24), with two
timing-only ablations that bound where the time goes:

  pipe 0   the 2-phase loop (gemm_bf16_mfma_256)
  pipe 1   half-tile pipeline (gemm_bf16_mfma_256p<false>)
  pipe 2   half-tile pipeline, wave groups staggered by a barrier (gemm_bf16_mfma_256p<true>)
  pipe 11  pipe 2 without the DMA inside the K-loop (compute + LDS reads + barriers only)
  pipe 12  pipe 2 without the MFMAs (DMA + LDS reads + barriers only)

The ablations compute a wrong C (the probe reports failed); only their time is used.

    python scripts/gemm_kloop_ab.py [rounds] [variants, e.g. 0,2,2g8] [sizes] > gpurun_out/gemm_kloop_ab.json
"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
# a variant is "<pipe>" or "<pipe>g<group_m>" (tile-row group size of the tile order, default 4)
variants = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2", "3", "11", "12"]
sizes = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [2048, 4096, 8192]
probe.init()
res: dict[str, list[float]] = {}
for n in sizes:
    for r in range(rounds):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            pipe, _, group = v.partition("g")
            out = probe.run(0, hbm_bytes=1 << 20, patterns=1, gemm_n=n, gemm_reps=10, overlap=0,
                            gemmPipe=int(pipe), gemmGroupM=int(group or 4))
            if int(pipe) < 10:
                assert out["passed"], out
            res.setdefault(f"{n}:pipe{v}", []).append(round(out["mfma"]["tflops"], 1))
probe.trim(0)
print(json.dumps({"rounds": rounds, "summary": {k: statistics.median(v) for k, v in res.items()},
                  "samples": res}, indent=1))

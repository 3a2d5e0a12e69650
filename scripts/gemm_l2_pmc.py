#!/usr/bin/env python3
"""One serial probe GEMM run at N^3 with a given tile order (and K-loop, ``gemmPipe`` 0/1/2), for a
rocprofv3 --pmc pass over it (L2 hit / miss of gemm_bf16_mfma_256 with row-major vs grouped tile
order; SQ counters of the K-loop variants):

    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d D -o g4 -- \\
        python3 scripts/gemm_l2_pmc.py 8192 4
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
group = int(sys.argv[2]) if len(sys.argv) > 2 else 4
pipe = int(sys.argv[3]) if len(sys.argv) > 3 else 0
probe.init()
r = probe.run(0, hbm_bytes=1 << 20, patterns=1, gemm_n=n, gemm_reps=3, overlap=0, gemmGroupM=group,
              gemmPipe=pipe)
assert r["passed"], r
print({"n": n, "group": group, "pipe": pipe, "tflops": r["mfma"]["tflops"]})
probe.trim(0)

#!/usr/bin/env python3
"""Claim-time probes in-process, for rocprofv3 --pmc passes over them: the HBM traffic of each
probe kernel as the memory system counts it (TCC FETCH_SIZE / WRITE_SIZE, KiB), against what the
kernel is meant to move (hbm_fill writes 1 GiB, hbm_verify reads 1 GiB). One counter group per
run (FETCH_SIZE takes 3 of the 4 TCC counters, WRITE_SIZE 2):

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d D -o fetch -- python3 scripts/probe_hbm_pmc.py 5
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
probe.init()
for _ in range(n):  # the claim-time shape: 1 GiB x 2 patterns beside the 2048^3 MFMA phase
    r = probe.run(0, hbm_bytes=1 << 30, gemm_n=2048, overlap=1)
    assert r["passed"], r
print({"probes": n, "ms": r.get("ms")})
probe.trim(0)

"""Claim-time probe cost vs. what it covers: spec.probe.hbmBytes x the GEMM size, in ONE process,
at the agent's probe configuration (two-stream: HBM pattern test beside the MFMA phase). The table behind the hbmBytes guidance in
docs/ARCHITECTURE.md §3: the pattern test is HBM-bound (2 writes + 2 reads of every byte), so
its time scales with the bytes covered; the rest of the HBM is walked by the idle scrubber.

    python scripts/probe_size_sweep.py [rounds] > gpurun_out/probe_size_sweep.json
"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

MiB = 1 << 20
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
configs = [(h, g) for h in (64 * MiB, 256 * MiB, 512 * MiB, 1024 * MiB, 4096 * MiB) for g in (4096,)] + \
    [(1024 * MiB, 2048), (1024 * MiB, 8192)]
probe.init()
res: dict[str, list[dict]] = {}
# The probe keeps its arena between runs unless the size changes by more than 2x (as the agent's
# claims do: one size per pool), so each size runs its rounds back to back after one warm run;
# two passes over the sizes expose drift.
for _ in range(2):
    for h, g in configs:
        assert probe.run(0, hbm_bytes=h, gemm_n=g)["passed"]
        for _ in range(rounds):
            r = probe.run(0, hbm_bytes=h, gemm_n=g)
            assert r["passed"] and r["phases"]["arenaReused"], r
            res.setdefault(f"hbm{h // MiB}MiB_gemm{g}", []).append(
                {"ms": r["ms"], "hbmGBps": r["hbm"]["GBps"], "tflops": r["mfma"]["tflops"]})
probe.trim(0)
print(json.dumps({"rounds": rounds, "median": {
    k: {m: round(statistics.median(x[m] for x in rs), 3) for m in ("ms", "hbmGBps", "tflops")}
    for k, rs in res.items()}}, indent=1))

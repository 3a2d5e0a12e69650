#!/usr/bin/env python3
"""Tile order of the probe's 256x256 MFMA GEMM inside each XCD (probe option ``gemmGroupM``): 0 =
row-major over the XCD's contiguous tile range, g > 1 = groups of g tile rows walked column-major
(the tiles an XCD runs at once then share A and B panels in its L2). Interleaved rounds in one
process, serial probe (no HBM test beside it), 10 GEMM reps per timing; every run's exact ABFT
checksums and element check must pass.

    python scripts/probe_gemm_group_ab.py [rounds] > gpurun_out/probe_gemm_group_ab.json
"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
# variants: "gN" = gemmGroupM N; "pN" = that with s_setprio around the MFMA block; "vN" = that
# with the transposed MFMA and 16-byte C stores
variants = tuple(os.environ.get("GROUP_AB_VARIANTS", "g0,g2,g4,g8,g16").split(","))


def opts_of(v: str) -> dict:
    return {"gemmGroupM": int(v[1:]), "gemmPrio": int(v[0] == "p"), "gemmVecC": int(v[0] == "v")}
probe.init()
res: dict[str, list[float]] = {}
sizes = tuple(int(x) for x in os.environ.get("GROUP_AB_SIZES", "4096,8192").split(","))
for n in sizes:
    for g in variants:  # warm every variant once
        assert probe.run(0, hbm_bytes=1 << 20, patterns=1, gemm_n=n, overlap=0, **opts_of(g))["passed"]
    for r in range(rounds):
        order = variants if r % 2 == 0 else tuple(reversed(variants))
        for g in order:
            out = probe.run(0, hbm_bytes=1 << 20, patterns=1, gemm_n=n, gemm_reps=10, overlap=0,
                            **opts_of(g))
            assert out["passed"] and out["mfma"]["abftMismatches"] == 0, (n, g, out)
            res.setdefault(f"{n}:{g}", []).append(round(out["mfma"]["tflops"], 1))
probe.trim(0)
summary = {k: {"median": statistics.median(v), "min": min(v), "max": max(v)} for k, v in res.items()}
print(json.dumps({"rounds": rounds, "summary": summary, "samples": res}, indent=1))

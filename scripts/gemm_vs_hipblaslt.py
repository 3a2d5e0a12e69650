#!/usr/bin/env python3
"""The probe's hand-written MFMA GEMMs (gemm_bf16_mfma_256, 256x256x64 glds tile, 2-phase loop;
gemm_bf16_mfma_256p, the same tile with the half-tile pipeline, "probe_pipe"; "probe_pipe2" with
the two wave groups one barrier apart) against the vendor
library on the same box: torch.matmul (hipBLASLt) on bf16 A[N,K] @ B[N,K]^T with fp32 accumulate,
interleaved rounds in one process. The probe's operands are small integers in [-2, 2] (exact
checks need them); data changes the clock the chip holds (cdna_hip_programming.md §5.4 rule 25),
so the library is timed on the same small-integer data and on full-range random normal data.

    python scripts/gemm_vs_hipblaslt.py [rounds] > gpurun_out/gemm_vs_hipblaslt.json
"""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
res: dict[str, list[float]] = {}
probe.init()
dev = torch.device("cuda:0")
for n in (2048, 4096, 8192):
    flop = 2.0 * n ** 3
    small_a = torch.randint(-2, 3, (n, n), device=dev).to(torch.bfloat16)
    small_b = torch.randint(-2, 3, (n, n), device=dev).to(torch.bfloat16)
    rnd_a = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    rnd_b = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def lib(a, b, reps=10):
        torch.matmul(a, b.t())
        ev0.record()
        for _ in range(reps):
            torch.matmul(a, b.t())
        ev1.record()
        torch.cuda.synchronize()
        return flop * reps / (ev0.elapsed_time(ev1) * 1e-3) / 1e12

    for r in range(rounds):
        order = ("probe", "probe_pipe", "probe_pipe2", "lib_small", "lib_random")
        for what in (order if r % 2 == 0 else order[::-1]):
            if what.startswith("probe"):
                out = probe.run(0, hbm_bytes=1 << 20, patterns=1, gemm_n=n, gemm_reps=10, overlap=0,
                                gemmPipe={"probe": 0, "probe_pipe": 1}.get(what, 2))
                assert out["passed"], out
                tf = out["mfma"]["tflops"]
            elif what == "lib_small":
                tf = lib(small_a, small_b)
            else:
                tf = lib(rnd_a, rnd_b)
            res.setdefault(f"{n}:{what}", []).append(round(tf, 1))
    del small_a, small_b, rnd_a, rnd_b
    torch.cuda.empty_cache()
probe.trim(0)
summary = {k: {"median_tflops": statistics.median(v), "max_tflops": max(v)} for k, v in res.items()}
for n in (2048, 4096, 8192):
    ls = summary[f"{n}:lib_small"]["median_tflops"]
    for what in ("probe", "probe_pipe", "probe_pipe2"):
        summary[f"{n}:{what}_vs_lib_same_data"] = round(summary[f"{n}:{what}"]["median_tflops"] / ls, 3)
print(json.dumps({"rounds": rounds, "note": "torch.matmul bf16 (hipBLASLt) vs the probe's MFMA GEMM; "
                  "fp32 accumulate; peak bf16 dense ~2500 TFLOP/s", "summary": summary,
                  "samples": res}, indent=1))

"""Interleaved in-process A/B of the probe's two GEMM kernels (cdna_hip_programming.md §5.4 rule 24:
N variants x M rounds in ONE process) plus the probe wall-time phases.

    python scripts/probe_ab.py --rounds 5 > gpurun_out/probe_ab.json

Every run must pass (bit-exact VALU 256^3 check + ABFT on N^3); the summary reports median/min
TFLOP/s per (tile, N) and the median probe phases at the agent's default config (1 GiB, N=4096).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpupool.ops import probe  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sizes", default="4096,8192")
    ap.add_argument("--tiles", default="128,256",
                    help="gemmTile kinds to compare: 128 (register-staged) and 256 (glds)")
    ap.add_argument("--stress", type=int, default=0,
                    help="extra exactness runs per tile at 512..4096 (race screen)")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    n_dev = probe.init()
    assert n_dev >= 1, "no HIP device"
    sizes = [int(x) for x in a.sizes.split(",")]
    tiles = [int(x) for x in a.tiles.split(",")]
    runs: dict[str, list[dict]] = {}
    failures = []
    for r in range(a.rounds):
        for n in sizes:
            for tile in tiles:
                res = probe.run(a.device, hbm_bytes=1 << 28, gemm_n=n, gemm_tile=tile)
                if not res.get("passed"):
                    failures.append(res)
                runs.setdefault(f"tile{tile}_n{n}", []).append(res)
        # the agent's default probe (1 GiB HBM, N=4096, 256 tile, HBM test and MFMA phase
        # overlapped on two streams) vs the same work serialised on one stream
        runs.setdefault("default_1GiB", []).append(probe.run(a.device))
        runs.setdefault("serial_1GiB", []).append(probe.run(a.device, overlap=0))
    stress = {}
    for i in range(a.stress):
        for tile in tiles:
            n = (512, 1024, 2048, 4096)[i % 4]
            res = probe.run(a.device, hbm_bytes=1 << 24, gemm_n=n, gemm_tile=tile)
            stress[tile] = stress.get(tile, 0) + 1
            if not res.get("passed"):
                failures.append(res)
    summary = {"stress_runs": stress}
    for key, rs in runs.items():
        tf = [x["mfma"]["tflops"] for x in rs]
        summary[key] = {"tflops_median": round(statistics.median(tf), 1), "tflops_min": round(min(tf), 1),
                        "tflops_max": round(max(tf), 1), "gemm_ms_median": round(statistics.median(
                            x["mfma"]["ms"] for x in rs), 4),
                        "probe_ms_median": round(statistics.median(x["ms"] for x in rs), 3),
                        "passed": all(x.get("passed") for x in rs)}
        if key in ("default_1GiB", "serial_1GiB"):
            for ph in rs[0].get("phases", {}):
                summary[key][ph + "_median"] = round(statistics.median(x["phases"][ph] for x in rs), 4)
            summary[key]["hbm_GBps_median"] = round(statistics.median(x["hbm"]["GBps"] for x in rs), 1)
    print(json.dumps({"summary": summary, "failures": failures[:3], "example": runs["default_1GiB"][-1]},
                     indent=1))
    return 0 if not failures else 1


if __name__ == "__main__":
    sys.exit(main())

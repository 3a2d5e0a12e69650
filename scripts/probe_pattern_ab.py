"""HBM pattern A/B: the per-word mix (hbmPattern 0) against the one-multiply-per-16-B pattern
(hbmPattern 1), interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24), both the
HBM test alone and the claim-time probe (HBM test beside the MFMA phase). Every run must pass.
Usage: probe_pattern_ab.py [rounds]"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.ops import probe  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
probe.init()
for pat in (0, 1):  # warm both kernels
    probe.run(0, hbm_bytes=1 << 30, hbmPattern=pat)
res: dict[str, list[dict]] = {}
for _ in range(rounds):
    for pat in (0, 1):
        r = probe.run(0, hbm_bytes=1 << 30, mfma=False, hbmPattern=pat)
        assert r["passed"], r
        res.setdefault(f"hbm_only_pattern{pat}", []).append({**r["hbm"], "hbmMs": r["hbm"]["ms"], "totalMs": r["ms"]})
        r = probe.run(0, hbm_bytes=1 << 30, hbmPattern=pat)
        assert r["passed"], r
        res.setdefault(f"claim_probe_pattern{pat}", []).append({**r["hbm"], "hbmMs": r["hbm"]["ms"], "totalMs": r["ms"]})
    # a corrupted word is still found, with its address, under the new pattern
    r = probe.run(0, hbm_bytes=1 << 30, mfma=False, hbmPattern=1, injectBitFlips=3)
    assert not r["passed"] and r["hbm"].get("badBits", 0) >= 3, r
out = {k: {m: round(statistics.median(x[m] for x in rs), 3)
           for m in ("writeGBps", "readGBps", "GBps", "hbmMs", "totalMs")} for k, rs in res.items()}
print(json.dumps({"rounds": rounds, "median": out}, indent=1))

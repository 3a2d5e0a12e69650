#!/usr/bin/env python3
"""Which queue CU masks does an SPX MI355X accept, and where do their waves land?

For each candidate mask a child process loads libgpupool_share.so (HSA_TOOLS_LIB, debug on: the
status hsa_amd_queue_cu_set_mask returned for every queue) and runs the probe's CU census (every CU
that ran an MFMA wave, per XCD). Used to decide the slot layout of gpupool/agent/slots.py:

  striped        bits 0-63 (contiguous)              -> 8 CUs on each XCD (profiles/r3b)
  xcd01          bits b%8 in {0,1}                    -> XCDs 0,1 whole, the other six empty
  xcd01+1each    xcd01 plus one CU on every other XCD -> does a non-empty XCD mask make it legal?
  skip-xcd7      every CU except those of XCD 7
  half-xcds      bits b%8 in {0..3}

    python scripts/cu_mask_layouts.py --out gpurun_out/cu_mask_layouts.json
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gpupool.agent.agent import _ranges  # noqa: E402

LIB = os.path.join(ROOT, "build", "native", "libgpupool_share.so")
CENSUS = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from gpupool.ops import probe
probe.init()
r = probe.run(0, hbm_bytes=64 << 20, mfma=True, gemm_n=1024, cuKeys=1)
print(json.dumps({"cus": len(r["cus"]["cuKeys"]), "perXcd": r["cus"]["perXcd"],
                  "mfmaOk": r["mfma"]["elementMismatches"] == 0}), flush=True)
"""


def masks() -> dict[str, list[int]]:
    xcd01 = [b for b in range(256) if b % 8 in (0, 1)]
    one_each = [b for b in range(256) if b % 8 >= 2 and b < 8]  # bits 2..7: one CU on XCDs 2..7
    return {
        "striped": list(range(64)),
        "xcd01": xcd01,
        "xcd01+1each": sorted(set(xcd01) | set(one_each)),
        "skip-xcd7": [b for b in range(256) if b % 8 != 7],
        "half-xcds": [b for b in range(256) if b % 8 < 4],
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/cu_mask_layouts.json")
    a = ap.parse_args()
    res = {}
    for name, bits in masks().items():
        env = dict(os.environ, PYTHONPATH=ROOT, HSA_TOOLS_LIB=LIB, GPUPOOL_CU_MASK=_ranges(bits),
                   GPUPOOL_SHARE_DEBUG="1")
        r = subprocess.run([sys.executable, "-c", CENSUS, ROOT], env=env, capture_output=True,
                           text=True, timeout=120)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        row = json.loads(lines[-1]) if lines else {"error": r.stderr[-800:]}
        row["maskBits"] = len(bits)
        row["mask"] = _ranges(bits)
        row["queueStatus"] = sorted({ln.rsplit("status", 1)[-1].strip() for ln in r.stderr.splitlines()
                                     if "CU mask" in ln and "status" in ln})
        row["rc"] = r.returncode
        res[name] = row
        print(name, json.dumps({k: row.get(k) for k in ("cus", "perXcd", "queueStatus", "rc")}),
              flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Where a probe helper's start-up goes (the HIP init a claim waits for when it must take a GPU
whose helper was parked under a tenant moments ago): fresh processes, each timing

  runtime   hipGetDeviceCount (HIP runtime + ROCr + driver open)
  context   hipSetDevice + hipFree(0) (the device context: queues, their context-save areas)
  warm      mi355x_probe_init's small warm probe (code object load, first launches, arena)

under the runtime settings that might move them. Prints one JSON line per setting (medians over
``--reps`` fresh processes). GPU only."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, json, os, sys, time
t0 = time.perf_counter()
hip = ctypes.CDLL("libamdhip64.so")
n = ctypes.c_int(0)
assert hip.hipGetDeviceCount(ctypes.byref(n)) == 0
t1 = time.perf_counter()
assert hip.hipSetDevice(0) == 0
hip.hipFree(ctypes.c_void_p(0))
t2 = time.perf_counter()
sys.path.insert(0, sys.argv[1])
from gpupool.ops import probe as hp
hp.init()
t3 = time.perf_counter()
print(json.dumps({"runtime": (t1 - t0) * 1e3, "context": (t2 - t1) * 1e3, "warm": (t3 - t2) * 1e3,
                  "total": (t3 - t0) * 1e3}))
"""

SETTINGS = {
    "default": {},
    "hw_queues_2": {"GPU_MAX_HW_QUEUES": "2"},
    "deferred_loading_off": {"HIP_ENABLE_DEFERRED_LOADING": "0"},
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    env0 = dict(os.environ)
    env0["ROCR_VISIBLE_DEVICES"] = env0.get("ROCR_VISIBLE_DEVICES", "0")
    for name, extra in SETTINGS.items():
        rows = []
        for _ in range(args.reps):
            p = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True,
                               timeout=120, env={**env0, **extra})
            if p.returncode != 0:
                print(json.dumps({"setting": name, "error": p.stderr[-400:]}), flush=True)
                break
            rows.append(json.loads(p.stdout.strip().splitlines()[-1]))
            time.sleep(0.2)
        if rows:
            print(json.dumps({"setting": name, "env": extra, "n": len(rows), "median_ms": {
                k: round(statistics.median(r[k] for r in rows), 1) for k in rows[0]}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

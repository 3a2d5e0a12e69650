#!/usr/bin/env python3
"""What the ~610 MiB of host memory a HIP context costs is made of, and whether anything in the
helper's control gives it back: each variant is a fresh child process that initialises the probe
library (HIP on this box's GPU) under an environment override, reports smaps_rollup and its
largest anonymous regions, then calls glibc's malloc_trim(0) and reports again.

    python scripts/hip_host_memory.py
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

VARIANTS = {
    "default": {},
    "hw_queues_1": {"GPU_MAX_HW_QUEUES": "1"},
    "hw_queues_2": {"GPU_MAX_HW_QUEUES": "2"},
    "hw_queues_3": {"GPU_MAX_HW_QUEUES": "3"},
}


def rollup() -> dict:
    out = {}
    with open("/proc/self/smaps_rollup") as f:
        for line in f:
            k, _, v = line.partition(":")
            if k in ("Rss", "Pss", "Private_Clean", "Private_Dirty", "Anonymous", "Locked"):
                out[k] = round(int(v.split()[0]) / 1024, 1)
    return out


def big_anon(min_mib: float = 8.0) -> list[dict]:
    head = re.compile(r"^([0-9a-f]+)-([0-9a-f]+) (\S+) \S+ \S+ \S+\s*(.*)$")
    rows, cur = [], None
    with open("/proc/self/smaps") as f:
        for line in f:
            m = head.match(line)
            if m:
                size = (int(m.group(2), 16) - int(m.group(1), 16)) / 2**20
                cur = {"sizeMiB": round(size, 1), "perm": m.group(3),
                       "name": m.group(4).strip() or "[anon]"}
                rows.append(cur)
            elif cur is not None:
                k, _, v = line.partition(":")
                if k in ("Rss", "Private_Clean", "Private_Dirty", "Locked"):
                    cur[k] = round(int(v.split()[0]) / 1024, 1)
                elif k == "VmFlags":
                    cur["flags"] = v.strip()
    rows = [r for r in rows if r["name"] in ("[anon]", "/dev/zero (deleted)")
            or r["name"].startswith("/dev/")]
    rows = [r for r in rows if r.get("Rss", 0) >= min_mib or r["name"].startswith("/dev/kfd")]
    return sorted(rows, key=lambda r: -r.get("Rss", 0))[:12]


def child() -> None:
    sys.path.insert(0, ROOT)
    out = {"before": rollup()}
    from gpupool.ops import probe
    probe.init()
    out["after_init"] = rollup()
    # the claim-time probe (HBM test beside the MFMA phase on two streams): does the queue cap
    # cost the overlap?
    times = []
    for _ in range(7):
        r = probe.run(0, hbm_bytes=1 << 30, mfma=True, gemm_n=2048, overlap=1)
        times.append(float(r.get("ms", 0.0)))
    out["probe_ms"] = sorted(times)[len(times) // 2]
    out["after_probe"] = rollup()
    out["regions"] = big_anon()
    import ctypes
    ctypes.CDLL("libc.so.6").malloc_trim(0)
    out["after_malloc_trim"] = rollup()
    print(json.dumps(out))


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        return 0
    res = {}
    for name, env in VARIANTS.items():
        r = subprocess.run(["timeout", "-k", "5", "60", sys.executable, __file__, "--child"],
                           capture_output=True, text=True, env={**os.environ, **env})
        try:
            res[name] = json.loads(r.stdout.strip().splitlines()[-1])
        except (IndexError, ValueError):
            res[name] = {"error": f"exit {r.returncode}: {r.stderr[-400:]}"}
        print(name, json.dumps({k: v for k, v in res[name].items() if k != "regions"}),
              file=sys.stderr, flush=True)
    tool = os.path.join(ROOT, "build", "native", "queue_mem")
    for name, env in (("queue_mem_default", {}), ("queue_mem_hwq1", {"GPU_MAX_HW_QUEUES": "1"}),
                      ("queue_mem_hwq2", {"GPU_MAX_HW_QUEUES": "2"})):
        r = subprocess.run(["timeout", "-k", "5", "60", tool, "3"], capture_output=True, text=True,
                           env={**os.environ, **env})
        res[name] = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")] or \
            {"error": f"exit {r.returncode}: {r.stderr[-300:]}"}
        print(name, json.dumps(res[name]), file=sys.stderr, flush=True)
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

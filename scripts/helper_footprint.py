#!/usr/bin/env python3
"""Host memory of the probe helpers (what ``--probe helper`` costs a node in RAM): N helpers on
this box's GPU (as on an N-GPU node, one per GPU), their RSS and PSS together after HIP init and
after one claim-size probe each, and what one helper's memory is made of (its largest mappings by
private + shared pages, from /proc/<pid>/smaps). PSS splits the pages the helpers share (the HIP
runtime's libraries) between them, so it is the fair per-node figure.

    python scripts/helper_footprint.py [N]      # default 8
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def mem(pid: int) -> dict:
    out = {}
    with open(f"/proc/{pid}/smaps_rollup") as f:
        for line in f:
            k, _, v = line.partition(":")
            if k in ("Rss", "Pss", "Private_Clean", "Private_Dirty", "Shared_Clean", "Anonymous"):
                out[k] = int(v.split()[0]) << 10
    return out


def top_mappings(pid: int, n: int = 12) -> list[dict]:
    """Largest mappings of ``pid`` by RSS, grouped by what is mapped (file or [anon])."""
    import re
    head = re.compile(r"^[0-9a-f]+-[0-9a-f]+ ")
    groups: dict[str, dict] = {}
    cur = None
    with open(f"/proc/{pid}/smaps") as f:
        for line in f:
            parts = line.split()
            if head.match(line):
                name = os.path.basename(parts[5]) if len(parts) >= 6 else "[anon]"
                cur = groups.setdefault(name or "[anon]", {"rss": 0, "pss": 0, "private": 0})
            elif cur is not None and line.startswith("Rss:"):
                cur["rss"] += int(parts[1]) << 10
            elif cur is not None and line.startswith("Pss:"):
                cur["pss"] += int(parts[1]) << 10
            elif cur is not None and line.startswith(("Private_Clean:", "Private_Dirty:")):
                cur["private"] += int(parts[1]) << 10
    rows = sorted(({"mapping": k, **{x: round(v / 2**20, 1) for x, v in d.items()}}
                   for k, d in groups.items()), key=lambda r: -r["rss"])
    return rows[:n]


def totals(pids: list[int]) -> dict:
    ms = [mem(p) for p in pids]
    return {k: round(sum(m.get(k, 0) for m in ms) / 2**20, 1)
            for k in ("Rss", "Pss", "Private_Clean", "Private_Dirty", "Shared_Clean", "Anonymous")}


def main() -> int:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    from gpupool.agent.probehost import HelperPool, start_spawner
    start_spawner()
    from gpupool.ops import devlib
    dev = devlib.DeviceLib("amdsmi", node="t", events=False).snapshot()["devices"][0]
    devs = [{"uuid": f"helper-{i}", "index": dev["index"], "hipUUID": dev.get("hipUUID", "")}
            for i in range(n)]
    out: dict = {"helpers": n, "gpu": dev.get("hipUUID"), "self_rss_mib": round(mem(os.getpid())["Rss"] / 2**20, 1)}
    pool = HelperPool("hip", arena_idle_s=0)
    try:
        t0 = time.perf_counter()
        ready = pool.start(devs)
        out["start_s"] = round(time.perf_counter() - t0, 2)
        out["ready"] = sum(1 for r in ready.values() if r.get("ok"))
        pids = sorted(pool.pids())
        time.sleep(0.5)
        out["after_init"] = totals(pids)
        args = {"hipUUID": dev.get("hipUUID", ""), "hbmBytes": 1 << 30, "mfma": True,
                "gemmN": 2048, "overlap": 1}
        for d in devs:  # one claim-size probe each, one at a time (one GPU here)
            pool.get(d["uuid"], d).call("probe", args, 60)
        time.sleep(0.5)
        out["after_probe"] = totals(pids)
        out["per_helper_after_probe_mib"] = {k: round(v / n, 1) for k, v in out["after_probe"].items()}
        out["one_helper_top_mappings"] = top_mappings(pids[0])
    finally:
        pool.stop()
    # the fabric helper (HIP on every GPU it rings; one here) with the runtime's default hardware
    # queues per GPU and with the one it is started with (probehost.FABRIC_HW_QUEUES)
    from gpupool.agent import probehost
    out["fabric"] = {}
    for cap in (0, 1):
        probehost.FABRIC_HW_QUEUES = cap
        fp = HelperPool("hip", arena_idle_s=0)
        try:
            h = fp.fabric([devs[0], devs[0]])
            if not h.wait_ready(60):
                out["fabric"][f"hwq{cap}"] = {"error": h.ready_error or "not ready"}
                continue
            ring = {"hipUUIDs": [dev.get("hipUUID", "")] * 2, "bytes": 16 << 20}
            h.call("peer_ring", ring, 30)  # first ring allocates the windows
            t = []
            for _ in range(5):
                t0 = time.perf_counter()
                h.call("peer_ring", ring, 30)
                t.append((time.perf_counter() - t0) * 1e3)
            time.sleep(0.3)
            m = mem(h.pid)
            out["fabric"][f"hwq{cap}"] = {"RssMiB": round(m["Rss"] / 2**20, 1),
                                          "PssMiB": round(m["Pss"] / 2**20, 1),
                                          "ring_ms_p50": round(sorted(t)[2], 3)}
        finally:
            fp.stop()
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

#!/usr/bin/env python3
"""Memory the node agent keeps on a GPU it shares with workload pods: VRAM in
use on device 0 (amdsmi, whole device) and this process's RSS at each stage of the agent's probe
lifecycle — before HIP is touched, after the HIP context + warm-up probe (probe.init), with the
~1.2 GiB claim-time arena kept after a default probe, and after the idle trim frees it."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rss_mib() -> float:
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024.0
    return 0.0


def main() -> None:
    from gpupool.ops import devlib
    dev = devlib.DeviceLib("amdsmi", node="t", events=False)

    def vram() -> int:
        time.sleep(0.3)  # let the driver's accounting settle
        return int(dev.snapshot()["devices"][0].get("memUsedBytes") or 0)

    out = {"stages": []}

    def stage(name: str) -> None:
        out["stages"].append({"stage": name, "vramUsedMiB": round(vram() / 2**20, 1),
                              "rssMiB": round(rss_mib(), 1)})
    stage("before HIP (amdsmi only)")
    from gpupool.ops import probe
    probe.init()  # HIP context on every visible GPU + 1 MiB warm-up probe (arena not kept)
    stage("HIP context + warm-up (agent idle)")
    r = probe.run(0, hbm_bytes=1 << 30)
    stage("after a claim-time probe (1 GiB arena kept)")
    freed = probe.trim(0)
    stage(f"after idle trim (freed {freed} arena)")
    base = out["stages"][0]["vramUsedMiB"]
    out["contextMiB"] = round(out["stages"][1]["vramUsedMiB"] - base, 1)
    out["arenaMiB"] = round(out["stages"][2]["vramUsedMiB"] - out["stages"][1]["vramUsedMiB"], 1)
    out["probePassed"] = r.get("passed")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

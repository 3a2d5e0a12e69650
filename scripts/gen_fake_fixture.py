#!/usr/bin/env python3
"""Generate tests/fixtures/node_8x_mi355x.json: an 8x MI355X OAM node for the fake backend.

Every per-device field is modelled on the real capture in tests/fixtures/real_mi355x/
(amd-smi + amdsmi Python on a gfx950 box): uuid/hipUUID formats, 7 of 8 xGMI links UP (one
'X' = disabled), hotspot/VRAM thermals with device critical/emergency limits (edge is N/A on
MI355X), SPX/NPS1 partitioning, 288 GB (294896 MiB) HBM3E. Topology: every GPU pair one xGMI hop
(weight 15, the amdsmi link weight of a direct xGMI link); GPUs 0-3 on NUMA 0, 4-7 on NUMA 1.
"""
from __future__ import annotations

import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BDFS = ["0000:05:00.0", "0000:15:00.0", "0000:65:00.0", "0000:75:00.0",
        "0000:85:00.0", "0000:95:00.0", "0000:e5:00.0", "0000:f5:00.0"]


def device(i: int) -> dict:
    serial = f"be28{i:02x}b252f0d03{i:01x}"
    return {
        "index": i,
        "uuid": f"beff75a3-0000-1000-80{i:02x}-8b252f0d03{i:02x}",
        "hipUUID": f"GPU-{serial}",
        "bdf": BDFS[i],
        "renderMinor": 128 + 8 * i,
        "renderNode": f"/dev/dri/renderD{128 + 8 * i}",
        "cardIndex": 8 + i,
        "kfdNode": 2 + i,
        "kfdId": 23660 + 1000 * i,
        "hipId": i,
        "numa": 0 if i < 4 else 1,
        "asic": {"marketName": "AMD Instinct MI355 OAM", "deviceId": "0x75a3", "gfx": "gfx950",
                 "computeUnits": 256, "serial": "0x" + serial.upper(), "oamId": i},
        "memTotalBytes": 309220868096,
        "partition": {"compute": "SPX", "memory": "NPS1"},
        "ecc": {"correctable": 0, "uncorrectable": 0, "deferred": 0},
        "xgmi": {"links": ["X", "U", "U", "U", "U", "U", "U", "U"], "up": 7, "down": 0},
        "temps": {"hotspot": {"current": 46 + i, "critical": 100, "emergency": 112},
                  "vram": {"current": 33 + i, "critical": 115, "emergency": 125}},
        "power": {"socketW": 262, "limitW": 1400},
        "activity": {"gfx": 0, "umc": 0},
        "present": True,
    }


def main() -> None:
    n = 8
    snap = {
        "backend": "fake",
        "node": "mi355x-node-0",
        "devices": [device(i) for i in range(n)],
        "topology": {
            "weights": [[0 if i == j else 15 for j in range(n)] for i in range(n)],
            "types": [["SELF" if i == j else "XGMI" for j in range(n)] for i in range(n)],
        },
    }
    path = os.path.join(ROOT, "tests", "fixtures", "node_8x_mi355x.json")
    with open(path, "w") as f:
        json.dump(snap, f, indent=1)
        f.write("\n")
    print(f"wrote {path}")


if __name__ == "__main__":
    main()

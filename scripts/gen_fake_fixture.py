#!/usr/bin/env python3
"""Generate the fake-backend node fixtures:

* ``tests/fixtures/node_8x_mi355x.json`` — an 8x MI355X OAM node in SPX/NPS1 (one logical GPU per
  ASIC, 256 CUs, 288 GB).
* ``tests/fixtures/node_8x_mi355x_cpx.json`` — the same node in CPX/NPS2: every ASIC exposes 8
  logical GPUs (one per XCD: 32 CUs, 36 GB, its own render/KFD node and PCI function), 64 in all.
  This is the MI355X's spatial-partitioning analogue of HAMi/MIG GPU sharing
  (/root/reference/GPU调度平台搭建.md:289-298).

Every per-device field is modelled on the real capture in tests/fixtures/real_mi355x/
(amd-smi + amdsmi Python on a gfx950 box): uuid/hipUUID formats, 7 of 8 xGMI links UP (one
'X' = disabled), hotspot/VRAM thermals with device critical/emergency limits (edge is N/A on
MI355X), 288 GB (294896 MiB) HBM3E, bad-page (RAS) counts, VRAM in use. Topology: every GPU pair
one xGMI hop (weight 15, the amdsmi link weight of a direct xGMI link); GPUs 0-3 on NUMA 0, 4-7 on
NUMA 1; partitions of one ASIC are closer than any xGMI peer (weight 5, type "SAMEASIC").
"""
from __future__ import annotations

import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BDFS = ["0000:05:00.0", "0000:15:00.0", "0000:65:00.0", "0000:75:00.0",
        "0000:85:00.0", "0000:95:00.0", "0000:e5:00.0", "0000:f5:00.0"]
HBM_BYTES = 309220868096
CUS = 256
XCDS = 8


def device(i: int, part: int | None = None) -> dict:
    """ASIC ``i``; ``part`` = partition (XCD) index in CPX mode, None in SPX."""
    serial = f"be28{i:02x}b252f0d03{i:01x}"
    p = part or 0
    idx = i if part is None else i * XCDS + p
    tag = f"{i:02x}" if part is None else f"{i:01x}{p:01x}"
    d = {
        "index": idx,
        "uuid": f"beff75a3-0000-1000-80{i:02x}-8b252f0d03{tag}",
        "hipUUID": f"GPU-{serial}" if part is None else f"GPU-{serial[:-1]}{p:01x}",
        "bdf": BDFS[i] if part is None else BDFS[i][:-1] + str(p),
        "renderMinor": 128 + 8 * i + p,
        "renderNode": f"/dev/dri/renderD{128 + 8 * i + p}",
        "cardIndex": 8 + 8 * i + p if part is not None else 8 + i,
        "kfdNode": 2 + (i if part is None else idx),
        "kfdId": 23660 + 1000 * i + p,
        "hipId": idx,
        "numa": 0 if i < 4 else 1,
        "asic": {"marketName": "AMD Instinct MI355 OAM", "deviceId": "0x75a3", "gfx": "gfx950",
                 "computeUnits": CUS if part is None else CUS // XCDS,
                 "serial": "0x" + serial.upper(), "oamId": i},
        "memTotalBytes": HBM_BYTES if part is None else HBM_BYTES // XCDS,
        "memUsedBytes": 298844160 if part is None else 298844160 // XCDS,
        "partition": {"compute": "SPX", "memory": "NPS1"} if part is None else
                     {"compute": "CPX", "memory": "NPS2", "id": p},
        "ecc": {"correctable": 0, "uncorrectable": 0, "deferred": 0},
        "ras": {"badPagesSupported": True, "retiredPages": 0, "pendingPages": 0,
                "unreservablePages": 0},
        "xgmi": {"links": ["X", "U", "U", "U", "U", "U", "U", "U"], "up": 7, "down": 0},
        "temps": {"hotspot": {"current": 46 + i, "critical": 100, "emergency": 112},
                  "vram": {"current": 33 + i, "critical": 115, "emergency": 125}},
        "power": {"socketW": 262, "limitW": 1400},
        "activity": {"gfx": 0, "umc": 0},
        "present": True,
    }
    return d


def node(cpx: bool) -> dict:
    devs = [device(i, p) for i in range(8) for p in range(XCDS)] if cpx else \
        [device(i) for i in range(8)]
    n = len(devs)
    asic = [d["asic"]["serial"] for d in devs]

    def w(a: int, b: int) -> int:
        return 0 if a == b else 5 if asic[a] == asic[b] else 15

    def t(a: int, b: int) -> str:
        return "SELF" if a == b else "SAMEASIC" if asic[a] == asic[b] else "XGMI"
    return {
        "backend": "fake",
        "node": "mi355x-node-0",
        "devices": devs,
        "topology": {"weights": [[w(a, b) for b in range(n)] for a in range(n)],
                     "types": [[t(a, b) for b in range(n)] for a in range(n)]},
    }


def main() -> None:
    for cpx, name in ((False, "node_8x_mi355x.json"), (True, "node_8x_mi355x_cpx.json")):
        path = os.path.join(ROOT, "tests", "fixtures", name)
        with open(path, "w") as f:
            json.dump(node(cpx), f, indent=1 if not cpx else None)
            f.write("\n")
        print(f"wrote {path}")


if __name__ == "__main__":
    main()

"""Helpers shared by the agent's modules."""
from __future__ import annotations

import datetime as _dt
import logging

SLOT_SEP = "::"  # device-plugin ID of a time-sliced slot: "<uuid>::<slot>"

log = logging.getLogger("gpupool.agent")


def gpu_of(device_id: str) -> str:
    """The GPU uuid behind a device-plugin ID (a plain uuid, or a shared GPU's slot)."""
    return device_id.split(SLOT_SEP, 1)[0]


def now_rfc3339() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _ranges(bits: list[int]) -> str:
    """[0, 1, 2, 5, 6] -> "0-2,5-6" (the CU-mask syntax libgpupool_share.so reads)."""
    out, start, prev = [], None, None
    for b in bits:
        if start is None:
            start = prev = b
        elif b == prev + 1:
            prev = b
        else:
            out.append(f"{start}-{prev}")
            start = prev = b
    if start is not None:
        out.append(f"{start}-{prev}")
    return ",".join(out)

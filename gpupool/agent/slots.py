"""Slot isolation on a shared MI355X (spec.sharing; the HAMi layer of the reference platform,
GPU调度平台搭建.md:289-298): which CUs a slot's queues may use, whether a pool's HBM budgets fit
the GPU, and the pod-wide HBM account file libgpupool_share.so charges (native/src/share/share.cc).

CU layout. ROCr's queue CU mask interleaves its bits over the XCDs: on an SPX MI355X (8 XCDs x 32
CUs) bit b is a CU of XCD b mod 8. And the dispatcher deals a kernel's workgroups round-robin over
all 8 XCDs whatever the mask, so a queue needs CUs on every XCD. Measured on the MI355X
(profiles/r4b_cu_mask_layouts.json, probe CU census per XCD):

  * a mask that leaves any XCD empty is NOT applied — silently: ROCr reports success and the
    queue runs on all 256 CUs (XCDs {0,1} only, XCDs {0..3}, every XCD but 7: all 256 CUs);
  * with at least one CU on every XCD the mask holds (XCDs 0,1 whole + 1 CU on each other XCD:
    exactly those 70 CUs) — but the round-robin then queues 6/8 of the workgroups on 6 single CUs.

So an SPX slot cannot own whole XCDs (nor an L2 of its own: every slot runs on every XCD), and the
balanced layout is the right one: slot i takes the contiguous bits [i*c, (i+1)*c), which land c/8
CUs on each XCD ("striped"). A slot of fewer CUs than the partition has XCDs would leave XCDs empty
and so run unconfined: such a pool is refused (``cu_floor``). L2 isolation between tenants comes
from compute partitions instead (spec.partition.compute DPX/QPX/CPX: each logical GPU has XCDs and
L2s of its own), with slots subdividing a partition.
"""
from __future__ import annotations

import os
import struct
import time

# XCDs per logical GPU by compute partition (MI355X: 8 XCDs per package)
XCDS_BY_PARTITION = {"SPX": 8, "DPX": 4, "QPX": 2, "CPX": 1}
CUS_PER_XCD = 32  # MI355X: 256 CUs on 8 XCDs


def xcd_count(dev: dict) -> int:
    part = str(((dev or {}).get("partition") or {}).get("compute") or "").upper()
    if part in XCDS_BY_PARTITION:
        return XCDS_BY_PARTITION[part]
    cus = int(((dev or {}).get("asic") or {}).get("computeUnits") or 256)
    return max(1, cus // CUS_PER_XCD)


def slot_cus(slot: int, slots: int, cu_per_slot: int, cus: int, xcds: int) -> tuple[list[int], str]:
    """CU-mask bits of ``slot`` (of ``slots`` on the GPU) and the layout ("striped": contiguous
    bits, cu/xcds CUs on every XCD). ``cu_per_slot`` is narrowed to the GPU's own share
    (cus // slots)."""
    cus, slots = max(1, cus), max(1, slots)
    cu = max(1, min(cu_per_slot, cus // slots))
    return list(range(slot * cu, (slot + 1) * cu)), "striped"


def slot_xcds(bits: list[int], xcds: int) -> list[int]:
    """The XCDs a mask's bits land on (the interleave above)."""
    return sorted({b % max(1, xcds) for b in bits})


def cu_floor(sharing: dict, dev: dict) -> str:
    """Why a pool's cuPerSlot cannot be confined on this GPU (fewer CUs per slot than the
    partition has XCDs: some XCD would get none, and the hardware would ignore the whole mask),
    or "" when it can."""
    cu = int((sharing or {}).get("cuPerSlot") or 0)
    if cu <= 0:
        return ""
    k = max(1, int((sharing or {}).get("replicasPerGPU") or 1))
    cus = int(((dev or {}).get("asic") or {}).get("computeUnits") or 256)
    xcds = xcd_count(dev)
    bits, _ = slot_cus(0, k, cu, cus, xcds)
    if len(slot_xcds(bits, xcds)) >= xcds:
        return ""
    return (f"cuPerSlot {cu} (x replicasPerGPU {k} on {cus} CUs) leaves XCDs of this "
            f"{xcds}-XCD GPU without CUs: the hardware would not apply the mask — use at least "
            f"{xcds} CUs per slot")


def overcommit(sharing: dict, mem_total: int, reserve: int) -> str:
    """Why a pool's slot budgets do not fit a GPU of ``mem_total`` bytes with ``reserve`` bytes kept
    for the agent's own use of it (HIP context + probe arena), or "" when they fit."""
    per_slot = int((sharing or {}).get("hbmBytesPerSlot") or 0)
    k = max(1, int((sharing or {}).get("replicasPerGPU") or 1))
    if per_slot <= 0 or mem_total <= 0:
        return ""
    usable = mem_total - max(0, reserve)
    if k * per_slot <= usable:
        return ""
    return (f"replicasPerGPU {k} x hbmBytesPerSlot {per_slot} = {k * per_slot} B exceeds the GPU's "
            f"{mem_total} B HBM minus the agent's {reserve} B reserve ({usable} B)")


# ---- the pod-wide HBM account (layout: native/src/share/share.cc) ----
ACCT_BYTES = 16384
ACCT_UUIDS_AT = 8192   # version 2: 8 x 32-byte GPU identities (HSA agent UUID = amdsmi hip_uuid)
ACCT_UUID_BYTES = 32
ACCT_IDS_AT_V1 = 8192  # the slot ids as text (agent bookkeeping)
ACCT_IDS_AT_V2 = ACCT_UUIDS_AT + 8 * ACCT_UUID_BYTES


def account_bytes(limit: int, slots: list[str], gpu_uuids: list[str],
                  created: float | None = None) -> bytes:
    """A fresh version-2 account: magic, per-GPU limit, the GPUs' identities (account index g is
    the g-th of ``gpu_uuids``), its creation time (header pad, ignored by the library: the file's
    mtime moves with every charge), zeroed counters, the slot ids as text."""
    buf = bytearray(ACCT_BYTES)
    ids = list(gpu_uuids)[:8]
    # no identities: version 1 (ordinal mapping); its slot-id text sits where v2 keeps the UUIDs
    version = 2 if ids else 1
    buf[0:32] = b"GPSHARE1" + struct.pack("<QIId", int(limit), version, len(ids) or 1,
                                          time.time() if created is None else created)
    for g, u in enumerate(ids):
        raw = u.encode()[:ACCT_UUID_BYTES - 1]
        at = ACCT_UUIDS_AT + g * ACCT_UUID_BYTES
        buf[at:at + len(raw)] = raw
    at = ACCT_IDS_AT_V2 if version >= 2 else ACCT_IDS_AT_V1
    text = ",".join(slots).encode()[: ACCT_BYTES - at - 1]
    buf[at:at + len(text)] = text
    return bytes(buf)


def limit_bytes(limit: int) -> bytes:
    """The read-only limit file beside an account (share.cc read_limit_file)."""
    return f"GPLIMIT1 {int(limit)}\n".encode()


def read_account(path: str) -> dict | None:
    """An account file's header and slot ids (None if unreadable / not an account)."""
    try:
        with open(path, "rb") as f:
            head = f.read(32)
            if len(head) < 32 or head[:8] != b"GPSHARE1":
                return None
            limit, version, ngpus, created = struct.unpack("<QIId", head[8:32])
            f.seek(ACCT_IDS_AT_V2 if version >= 2 else ACCT_IDS_AT_V1)
            text = f.read().split(b"\0", 1)[0].decode(errors="replace")
    except OSError:
        return None
    # (version 1 files of earlier agents kept no creation time: 0.0 there)
    return {"limit": limit, "version": version, "ngpus": ngpus, "created": created,
            "slots": [s for s in text.split(",") if s]}


def account_slots(path: str) -> list[str] | None:
    """The slot ids an account file was made for (None if unreadable / not an account)."""
    a = read_account(path)
    return None if a is None else a["slots"]


def gc_accounts(directory: str, live_ids: set[str], older_than: float) -> list[str]:
    """Delete the account files none of whose slots a pod holds any more (``live_ids``: the device
    IDs the kubelet's PodResources lists) and that were created before ``older_than`` (wall clock)
    — an Allocate can precede the listing that shows its pod. Returns the deleted paths."""
    gone = []
    try:
        names = os.listdir(directory)
    except OSError:
        return gone
    for name in names:
        if not name.endswith(".acct"):
            continue
        path = os.path.join(directory, name)
        acct = read_account(path)
        if acct is None or acct["created"] >= older_than or set(acct["slots"]) & live_ids:
            continue
        try:
            os.unlink(path)
            gone.append(path)
        except OSError:
            pass
        try:  # its read-only limit file goes with it
            os.unlink(path[:-len(".acct")] + ".limit")
        except OSError:
            pass
    return gone

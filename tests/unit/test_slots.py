"""Slot isolation helpers (gpupool/agent/slots.py): CU-mask layout per slot, the per-XCD floor,
HBM overcommit against the agent's reserve, and the HBM account file format + GC."""
from __future__ import annotations

import os
import time

from gpupool.agent import slots as sl

SPX = {"asic": {"computeUnits": 256}, "partition": {"compute": "SPX"}, "memTotalBytes": 309220868096}
CPX = {"asic": {"computeUnits": 32}, "partition": {"compute": "CPX"}}


def test_xcd_count_by_partition_and_cu_count():
    assert sl.xcd_count(SPX) == 8 and sl.xcd_count(CPX) == 1
    assert sl.xcd_count({"partition": {"compute": "DPX"}}) == 4
    assert sl.xcd_count({"asic": {"computeUnits": 64}}) == 2  # no partition info: CUs / 32


def test_slots_are_contiguous_disjoint_and_span_every_xcd():
    masks = [sl.slot_cus(i, 4, 64, 256, 8)[0] for i in range(4)]
    assert [m[0] for m in masks] == [0, 64, 128, 192] and all(len(m) == 64 for m in masks)
    assert sorted(b for m in masks for b in m) == list(range(256))
    assert all(sl.slot_xcds(m, 8) == list(range(8)) for m in masks)
    # narrowed to the GPU's share: 4 slots can never take more than 64 CUs each
    assert len(sl.slot_cus(3, 4, 128, 256, 8)[0]) == 64


def test_cu_floor_refuses_slots_that_would_leave_an_xcd_empty():
    assert sl.cu_floor({"replicasPerGPU": 4, "cuPerSlot": 4}, SPX)
    assert sl.cu_floor({"replicasPerGPU": 2, "cuPerSlot": 7}, SPX)
    assert not sl.cu_floor({"replicasPerGPU": 32, "cuPerSlot": 8}, SPX)
    assert not sl.cu_floor({"replicasPerGPU": 8, "cuPerSlot": 4}, CPX)  # one XCD: any size
    assert not sl.cu_floor({"replicasPerGPU": 4}, SPX)  # no CU share asked


def test_overcommit_against_the_agents_reserve():
    why = sl.overcommit({"replicasPerGPU": 4, "hbmBytesPerSlot": 100 << 30},
                        SPX["memTotalBytes"], 2 << 30)
    assert "exceeds" in why and "reserve" in why
    assert not sl.overcommit({"replicasPerGPU": 4, "hbmBytesPerSlot": 64 << 30},
                             SPX["memTotalBytes"], 2 << 30)
    # exactly the usable HBM fits; one byte more does not
    usable = SPX["memTotalBytes"] - (2 << 30)
    assert not sl.overcommit({"replicasPerGPU": 1, "hbmBytesPerSlot": usable}, SPX["memTotalBytes"], 2 << 30)
    assert sl.overcommit({"replicasPerGPU": 1, "hbmBytesPerSlot": usable + 1}, SPX["memTotalBytes"], 2 << 30)


def test_account_round_trip_and_gc(tmp_path):
    d = tmp_path / "share"
    d.mkdir()
    old = d / "old.acct"
    old.write_bytes(sl.account_bytes(8 << 30, ["g1::0", "g1::1"], ["GPU-aa", "GPU-bb"], created=100.0))
    a = sl.read_account(str(old))
    assert a == {"limit": 8 << 30, "version": 2, "ngpus": 2, "created": 100.0, "slots": ["g1::0", "g1::1"]}
    raw = old.read_bytes()
    assert raw[8192:8198] == b"GPU-aa" and raw[8224:8230] == b"GPU-bb" and not any(raw[64:8192])
    live = d / "live.acct"
    live.write_bytes(sl.account_bytes(8 << 30, ["g2::0"], ["GPU-cc"], created=100.0))
    young = d / "young.acct"
    young.write_bytes(sl.account_bytes(8 << 30, ["g3::0"], ["GPU-dd"]))
    (d / "other.txt").write_text("not an account")
    gone = sl.gc_accounts(str(d), {"g2::0"}, older_than=time.time() - 10)
    assert gone == [str(old)], gone  # live slot kept, young account kept, non-accounts untouched
    assert sorted(os.listdir(d)) == ["live.acct", "other.txt", "young.acct"]

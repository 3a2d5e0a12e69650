"""The claim ledger's hand-over commits (gpupool/agent/ledger.py): a claim passes its live claim
map and its lock to the writer (``commit(lock=...)``) and probes while the writer encodes and
fsyncs it; ``flush(seq)`` still returns only once that state is on disk, and owners that flush
while holding their lock never deadlock with the writer encoding under it."""
from __future__ import annotations

import json
import os
import threading
import time

from gpupool.agent.ledger import Ledger, read_claims


def _on_disk(d: str) -> dict:
    with open(os.path.join(d, "ledger.json")) as f:
        return json.load(f)["claims"]


def test_handed_over_map_is_durable_after_flush(tmp_path):
    led = Ledger(str(tmp_path), fsync=True)
    lock = threading.RLock()
    recs = {"gpu-a": {"uuid": "gpu-a", "poolUID": "p", "state": "Probing"}}
    with lock:
        seq = led.commit(recs, durable=False, lock=lock)
    with lock:  # the owner keeps mutating under its lock (Probing -> Claimed)
        recs["gpu-a"]["state"] = "Claimed"
    led.flush(seq)
    assert _on_disk(str(tmp_path))["gpu-a"]["state"] in ("Probing", "Claimed")
    led.flush()
    assert read_claims(str(tmp_path))["gpu-a"]["state"] == "Claimed"


def test_eager_commit_after_hand_over_wins(tmp_path):
    led = Ledger(str(tmp_path), fsync=False)
    lock = threading.RLock()
    led.commit({"a": {"uuid": "a"}}, durable=False, lock=lock)
    led.commit({"b": {"uuid": "b"}})  # durable, encoded now: the newer state
    led.flush()
    assert set(_on_disk(str(tmp_path))) == {"b"}


def test_owner_flushing_under_its_lock_never_deadlocks_with_the_writer(tmp_path):
    """Owners commit durably while holding their lock (lock -> writer mutex); the background
    writer encodes handed-over maps under the same lock, before it takes the writer mutex."""
    led = Ledger(str(tmp_path), fsync=False)
    lock = threading.RLock()
    recs: dict[str, dict] = {}
    stop = time.monotonic() + 2.0
    errors: list[BaseException] = []

    def claimer(k: int) -> None:
        try:
            i = 0
            while time.monotonic() < stop:
                with lock:
                    recs[f"g{k}-{i}"] = {"uuid": f"g{k}-{i}"}
                    seq = led.commit(recs, durable=False, lock=lock)
                led.flush(seq)
                i += 1
        except BaseException as e:  # pragma: no cover - reported below
            errors.append(e)

    def durable_owner() -> None:
        try:
            while time.monotonic() < stop:
                with lock:
                    led.commit(recs)  # durable, under the lock
        except BaseException as e:  # pragma: no cover
            errors.append(e)

    ts = [threading.Thread(target=claimer, args=(k,)) for k in range(3)] + \
        [threading.Thread(target=durable_owner)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    assert not any(t.is_alive() for t in ts), "ledger writer deadlocked with an owner"
    assert not errors, errors
    led.flush()
    with lock:
        assert set(_on_disk(str(tmp_path))) == set(recs)

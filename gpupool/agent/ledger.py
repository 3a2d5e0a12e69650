"""Claim ledger: the node agent's durable record of which GPU belongs to which pool.

One JSON file per claimed device (``<state>/claims/<uuid>.json``) written atomically
(write temp -> fsync -> rename -> fsync dir), plus ``<state>/quarantine/<uuid>.json`` for GPUs that
failed a probe. Together with ``status.devices`` on the pool and the device labels this is what
makes the operator stateless across restarts (SURVEY.md §5 checkpoint/resume row): on start the
agent reloads the ledger, and the manager's orphan sweep releases claims whose pool UID is gone.
"""
from __future__ import annotations

import json
import os
import threading
import time


def _atomic_write(path: str, data: dict) -> None:
    d = os.path.dirname(path)
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp.{os.getpid()}.{threading.get_ident()}"
    with open(tmp, "w") as f:
        json.dump(data, f, sort_keys=True)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    try:
        fd = os.open(d, os.O_RDONLY)
        try:
            os.fsync(fd)
        finally:
            os.close(fd)
    except OSError:
        pass


def _safe(uuid: str) -> str:
    return "".join(c if c.isalnum() or c in "-_." else "_" for c in uuid)


class Ledger:
    def __init__(self, state_dir: str, fsync: bool = True):
        self.dir = state_dir
        self.claims_dir = os.path.join(state_dir, "claims")
        self.quar_dir = os.path.join(state_dir, "quarantine")
        os.makedirs(self.claims_dir, exist_ok=True)
        os.makedirs(self.quar_dir, exist_ok=True)
        self.fsync = fsync

    # ---------------------------------------------------------------- claims
    def load(self) -> dict[str, dict]:
        out = {}
        for name in sorted(os.listdir(self.claims_dir)):
            if not name.endswith(".json"):
                continue
            try:
                with open(os.path.join(self.claims_dir, name)) as f:
                    rec = json.load(f)
                out[rec["uuid"]] = rec
            except (OSError, ValueError, KeyError):
                continue  # torn/partial files cannot exist (atomic rename); ignore stray junk
        return out

    def put(self, rec: dict) -> None:
        path = os.path.join(self.claims_dir, _safe(rec["uuid"]) + ".json")
        if self.fsync:
            _atomic_write(path, rec)
        else:
            tmp = path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(rec, f, sort_keys=True)
            os.replace(tmp, path)

    def delete(self, uuid: str) -> None:
        try:
            os.remove(os.path.join(self.claims_dir, _safe(uuid) + ".json"))
        except FileNotFoundError:
            pass

    # ---------------------------------------------------------------- quarantine
    def quarantine(self, uuid: str, seconds: float, reason: str) -> None:
        _atomic_write(os.path.join(self.quar_dir, _safe(uuid) + ".json"),
                      {"uuid": uuid, "until": time.time() + seconds, "reason": reason})

    def quarantined(self) -> dict[str, dict]:
        out, now = {}, time.time()
        for name in os.listdir(self.quar_dir):
            p = os.path.join(self.quar_dir, name)
            try:
                with open(p) as f:
                    rec = json.load(f)
            except (OSError, ValueError):
                continue
            if rec.get("until", 0) > now:
                out[rec["uuid"]] = rec
            else:
                try:
                    os.remove(p)
                except OSError:
                    pass
        return out

    def clear_quarantine(self, uuid: str) -> None:
        try:
            os.remove(os.path.join(self.quar_dir, _safe(uuid) + ".json"))
        except FileNotFoundError:
            pass

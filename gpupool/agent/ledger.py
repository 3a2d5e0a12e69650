"""Claim ledger: the node agent's durable record of which GPU belongs to which pool.

All claims live in one JSON document (``<state>/ledger.json``: ``{"version": 1, "claims": {uuid:
record}, "hbmSweep": {uuid: scrubber cursor/coverage}, "xgmiPairs": {"uA|uB": last peer check}}``) that is replaced atomically (write temp
-> fsync -> rename -> fsync dir), so a claim of 8 GPUs costs one fsync, not eight, and a crash can
never leave a half-written batch. Commits that must be durable before the agent acts on them
(claim, release) are flushed synchronously — the claim's while its probe runs; transitions a crash
may safely lose (Probing -> Claimed) go through a coalescing background writer. GPUs that failed a probe are recorded in ``<state>/quarantine/<uuid>.json``.
Together with ``status.devices`` on the pool this makes the operator stateless across restarts
(SURVEY.md §5 checkpoint/resume row): on start the agent reloads the ledger, and the manager's
orphan sweep releases claims whose pool UID is gone.
"""
from __future__ import annotations

import json
import os
import threading
import time

VERSION = 1


def _fsync_dir(d: str) -> None:
    try:
        fd = os.open(d, os.O_RDONLY)
        try:
            os.fsync(fd)
        finally:
            os.close(fd)
    except OSError:
        pass


def _atomic_write_text(path: str, text: str, fsync: bool = True) -> None:
    d = os.path.dirname(path)
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp.{os.getpid()}.{threading.get_ident()}"
    with open(tmp, "w") as f:
        f.write(text)
        if fsync:
            f.flush()
            os.fsync(f.fileno())
    os.replace(tmp, path)
    if fsync:
        _fsync_dir(d)


def _safe(uuid: str) -> str:
    return "".join(c if c.isalnum() or c in "-_." else "_" for c in uuid)


def read_claims(state_dir: str) -> dict[str, dict]:
    """Parse a ledger directory without an agent (used by the bench's independent ground truth)."""
    path = os.path.join(state_dir, "ledger.json")
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return {}
    return dict(doc.get("claims") or {})


class Ledger:
    def __init__(self, state_dir: str, fsync: bool = True):
        self.dir = state_dir
        self.path = os.path.join(state_dir, "ledger.json")
        self.quar_dir = os.path.join(state_dir, "quarantine")
        os.makedirs(self.quar_dir, exist_ok=True)
        self.fsync = fsync
        self._mu = threading.Lock()      # guards the serialised sections + sequence numbers
        self._wmu = threading.Lock()     # one writer at a time; the newest state wins
        self._seq = 0                    # bumped by every commit
        self._written = 0                # newest seq known to be on disk
        self._lazy = threading.Event()
        self._lazy_thread: threading.Thread | None = None
        self.writes = 0
        # quarantine entries cached in memory (this process is the only writer): claims and node
        # views consult them per GPU and must not rescan the directory each time
        self._quar: dict[str, dict] = {}
        for name in os.listdir(self.quar_dir):
            try:
                with open(os.path.join(self.quar_dir, name)) as f:
                    rec = json.load(f)
                self._quar[rec["uuid"]] = rec
            except (OSError, ValueError, KeyError):
                continue
        # serialised sections: each is rendered by its writer's thread (the claim map under the
        # agent lock), so a scrubber write never iterates a claim map another thread is editing
        self._claims_text = "{}"
        self._claims_src: tuple | None = None  # (claims, lock) handed over by commit(lock=...)
        self._src_seq = 0                      # the sequence number of that hand-over
        self._sweep: dict[str, dict] = {}
        self._xgmi: dict[str, dict] = {}
        self._leader: dict = {}
        try:
            with open(self.path) as f:
                doc = json.load(f) or {}
            self._sweep = dict(doc.get("hbmSweep") or {})
            self._xgmi = dict(doc.get("xgmiPairs") or {})
            self._leader = dict(doc.get("leaderFence") or {})
        except (OSError, ValueError):
            pass

    # ---------------------------------------------------------------- claims
    def load(self) -> dict[str, dict]:
        claims = read_claims(self.dir)
        self._claims_text = json.dumps(claims, sort_keys=True)
        legacy = os.path.join(self.dir, "claims")  # per-device files of earlier versions
        if os.path.isdir(legacy):
            for name in sorted(os.listdir(legacy)):
                if name.endswith(".json"):
                    try:
                        with open(os.path.join(legacy, name)) as f:
                            rec = json.load(f)
                        claims.setdefault(rec["uuid"], rec)
                    except (OSError, ValueError, KeyError):
                        continue
        return claims

    def commit(self, claims: dict[str, dict], durable: bool = True,
               lock: threading.RLock | None = None) -> int:
        """Record the full claim map; returns its sequence number. ``durable``: written and
        fsync'ed before returning (one write per agent operation, atomically replaced). Otherwise
        the write is left to a background writer (coalesced) — for transitions a crash may lose
        safely, e.g. Probing -> Claimed: a restarted agent probes a 'Probing' record's GPU again
        (kept if it passes, replaced by its pool if not) — or made durable later by
        ``flush(seq)``. With ``lock`` (the caller's lock guarding ``claims``; not durable) the map
        is serialised by the writer too, under that lock: a claim hands its record over and probes
        while the writer encodes and fsyncs it."""
        with self._mu:
            # encoded and numbered together: two commits racing (callers normally serialise them
            # under the agent's lock) can never number the older map after the newer one
            text = None if lock is not None and not durable else json.dumps(claims, sort_keys=True)
            self._seq += 1
            seq = self._seq
            if text is None:
                self._claims_src, self._src_seq = (claims, lock), seq
            else:
                self._claims_text, self._claims_src = text, None
        if durable:
            self.flush(seq)
        else:
            self._kick_lazy()
        return seq

    def flush(self, upto: int | None = None) -> None:
        """Make everything up to sequence ``upto`` (default: all committed so far) durable."""
        with self._mu:
            want = self._seq if upto is None else upto
        while True:
            with self._mu:  # already on disk: do not queue behind a writer busy with a newer state
                if self._written >= want:
                    return
                src = self._claims_src
            if src is not None:
                # encode a handed-over claim map under its owner's lock — before taking _wmu:
                # owners hold their lock while they flush (lock -> _wmu), never the reverse
                claims, lock = src
                with lock:
                    text = json.dumps(claims, sort_keys=True)
                with self._mu:
                    if self._claims_src is src:  # a newer commit replaced it otherwise
                        self._claims_text, self._claims_src = text, None
            with self._wmu:
                with self._mu:
                    if self._written >= want:
                        return
                    seq = self._seq
                    if self._claims_src is not None:  # handed over after the encode: next turn
                        seq = self._src_seq - 1
                    text = '{"version": %d, "claims": %s, "hbmSweep": %s, "xgmiPairs": %s, ' \
                        '"leaderFence": %s}' % (
                            VERSION, self._claims_text, json.dumps(self._sweep, sort_keys=True),
                            json.dumps(self._xgmi, sort_keys=True),
                            json.dumps(self._leader, sort_keys=True))
                if seq > self._written:
                    _atomic_write_text(self.path, text, self.fsync)
                    self.writes += 1
                    with self._mu:
                        self._written = max(self._written, seq)

    def _kick_lazy(self) -> None:
        if self._lazy_thread is None:
            self._lazy_thread = threading.Thread(target=self._lazy_loop, daemon=True,
                                                 name="ledger-writer")
            self._lazy_thread.start()
        self._lazy.set()

    def _lazy_loop(self) -> None:
        while True:
            self._lazy.wait()
            self._lazy.clear()
            try:
                self.flush()
            except OSError:
                time.sleep(0.1)
                self._lazy.set()

    def commit_sweep(self, sweep: dict[str, dict]) -> None:
        """Persist the HBM scrubber's per-device cursors/coverage (same document, same atomicity)."""
        with self._mu:
            self._sweep = {u: dict(r) for u, r in sweep.items()}
            self._seq += 1
            seq = self._seq
        self.flush(seq)

    def commit_xgmi(self, pairs: dict[str, dict], durable: bool = False) -> None:
        """Persist the per-GPU-pair xGMI peer-check results (``"uuidA|uuidB"`` -> last result and
        time), so link coverage survives agent restarts."""
        with self._mu:
            self._xgmi = {k: dict(r) for k, r in pairs.items()}
            self._seq += 1
            seq = self._seq
        if durable:
            self.flush(seq)
        else:
            self._kick_lazy()

    def commit_leader(self, fence: dict) -> None:
        """Persist the highest leader fencing token seen (durable: a restarted agent must still
        refuse an older leader)."""
        with self._mu:
            self._leader = dict(fence)
            self._seq += 1
            seq = self._seq
        self.flush(seq)

    def leader_state(self) -> dict:
        with self._mu:
            return dict(self._leader)

    def xgmi_state(self) -> dict[str, dict]:
        with self._mu:
            return {k: dict(r) for k, r in self._xgmi.items()}

    def sweep_state(self) -> dict[str, dict]:
        with self._mu:
            return {u: dict(r) for u, r in self._sweep.items()}

    # ---------------------------------------------------------------- quarantine
    def quarantine(self, uuid: str, seconds: float, reason: str, maintenance: bool = False,
                   write: bool = True) -> dict:
        """Quarantine ``uuid`` (in memory at once). ``write=False`` leaves the durable file to
        ``persist_quarantine`` — for callers holding a lock that fsyncs must not run under."""
        rec = {"uuid": uuid, "until": time.time() + seconds, "reason": reason,
               "maintenance": maintenance}
        with self._mu:
            self._quar[uuid] = rec
        if write:
            self.persist_quarantine(rec)
        return rec

    def persist_quarantine(self, rec: dict) -> None:
        _atomic_write_text(os.path.join(self.quar_dir, _safe(rec["uuid"]) + ".json"),
                           json.dumps(rec), self.fsync)

    def quarantined(self) -> dict[str, dict]:
        now = time.time()
        with self._mu:
            expired = [u for u, r in self._quar.items() if r.get("until", 0) <= now]
            for u in expired:
                del self._quar[u]
            out = dict(self._quar)
        for u in expired:
            try:
                os.remove(os.path.join(self.quar_dir, _safe(u) + ".json"))
            except OSError:
                pass
        return out

    def clear_quarantine(self, uuid: str) -> None:
        with self._mu:
            self._quar.pop(uuid, None)
        try:
            os.remove(os.path.join(self.quar_dir, _safe(uuid) + ".json"))
        except FileNotFoundError:
            pass

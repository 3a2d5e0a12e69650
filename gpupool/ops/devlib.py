"""ctypes binding for libmi355x_dev.so (native/include/mi355x/dev.h)."""
from __future__ import annotations

import ctypes
import json
import threading
from typing import Any

from . import native_path

_lib = None
_lock = threading.Lock()


def lib() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            l = ctypes.CDLL(native_path("libmi355x_dev.so"))
            l.mi355x_dev_open.restype = ctypes.c_void_p
            l.mi355x_dev_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                          ctypes.c_size_t]
            l.mi355x_dev_close.argtypes = [ctypes.c_void_p]
            for fn in ("mi355x_dev_snapshot", "mi355x_dev_health_snapshot"):
                getattr(l, fn).restype = ctypes.c_void_p
                getattr(l, fn).argtypes = [ctypes.c_void_p]
            for fn in ("mi355x_dev_wait_events", "mi355x_dev_wait_faults"):
                getattr(l, fn).restype = ctypes.c_void_p
                getattr(l, fn).argtypes = [ctypes.c_void_p, ctypes.c_int]
            l.mi355x_dev_evaluate.restype = ctypes.c_void_p
            l.mi355x_dev_evaluate.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
            l.mi355x_dev_evaluate_batch.restype = ctypes.c_void_p
            l.mi355x_dev_evaluate_batch.argtypes = [ctypes.c_char_p]
            l.mi355x_dev_select.restype = ctypes.c_void_p
            l.mi355x_dev_select.argtypes = [ctypes.c_char_p]
            l.mi355x_free.argtypes = [ctypes.c_void_p]
            l.mi355x_dev_version.restype = ctypes.c_char_p
            _lib = l
    return _lib


def _take(p: int | None) -> Any:
    if not p:
        raise RuntimeError("libmi355x_dev returned NULL")
    try:
        return json.loads(ctypes.string_at(p).decode())
    finally:
        lib().mi355x_free(p)


class DeviceLib:
    """One backend instance: ``DeviceLib("fake", fixture=..., faults=..., node=...)``."""

    def __init__(self, backend: str = "auto", **cfg: Any):
        err = ctypes.create_string_buffer(1024)
        self._h = lib().mi355x_dev_open(backend.encode(), json.dumps(cfg).encode(), err, len(err))
        if not self._h:
            raise RuntimeError(f"mi355x_dev_open({backend}): {err.value.decode()}")
        self.backend = backend
        self._mu = threading.Lock()

    def snapshot(self) -> dict:
        with self._mu:
            out = _take(lib().mi355x_dev_snapshot(self._h))
        if "error" in out:
            raise RuntimeError(out["error"])
        return out

    def health_snapshot(self) -> dict:
        """ECC / xGMI / temperatures / presence only (the fields verdicts use), for a fast poll."""
        with self._mu:
            out = _take(lib().mi355x_dev_health_snapshot(self._h))
        if "error" in out:
            raise RuntimeError(out["error"])
        return out

    def wait_events(self, timeout_ms: int = 500) -> dict:
        """Block (GIL released) up to ``timeout_ms`` for amdsmi device events:
        {"supported", "events": [{"index", "type", "message"}]}."""
        return _take(lib().mi355x_dev_wait_events(self._h, int(timeout_ms)))

    def wait_faults(self, timeout_ms: int = 500) -> dict:
        """Block up to ``timeout_ms`` for the fault-overlay file to change: {"supported", "changed"}."""
        return _take(lib().mi355x_dev_wait_faults(self._h, int(timeout_ms)))

    def close(self) -> None:
        if self._h:
            lib().mi355x_dev_close(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def evaluate(device: dict, baseline: dict | None, policy: dict | None) -> dict:
    return _take(lib().mi355x_dev_evaluate(json.dumps(device).encode(),
                                           json.dumps(baseline or {}).encode(),
                                           json.dumps(policy or {}).encode()))


def evaluate_batch(items: list[tuple[dict, dict | None, dict | None]]) -> list[dict]:
    """[(device, baseline or None, policy or None)] -> verdicts, in one native call."""
    if not items:
        return []
    out = _take(lib().mi355x_dev_evaluate_batch(json.dumps(
        [{"device": d, "baseline": b, "policy": p or {}} for d, b, p in items]).encode()))
    if isinstance(out, dict) and "error" in out:
        raise RuntimeError(out["error"])
    return out


def select(count: int, candidates: list[int], owned: list[int], policy: str,
           weights: list, numa: list) -> list[int]:
    out = _take(lib().mi355x_dev_select(json.dumps({
        "count": count, "candidates": candidates, "owned": owned, "policy": policy,
        "weights": weights, "numa": numa}).encode()))
    return list(out.get("selected", []))


def version() -> str:
    return lib().mi355x_dev_version().decode()

"""Bindings to the native MI355X libraries (built by ``make native`` into build/native/).

* :mod:`gpupool.ops.devlib` — libmi355x_dev.so: discovery, telemetry, health verdicts, selection.
* :mod:`gpupool.ops.probe`  — libmi355x_probe.so: the gfx950 HIP readiness probe kernels.

Both fail loudly (:class:`NativeLibraryMissing`) when the shared object is absent: there is no
silent Python fallback for the device path.
"""
from __future__ import annotations

import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class NativeLibraryMissing(RuntimeError):
    pass


def native_dir() -> str:
    return os.environ.get("GPUPOOL_NATIVE_DIR") or os.path.join(ROOT, "build", "native")


def native_path(name: str) -> str:
    p = os.path.join(native_dir(), name)
    if not os.path.exists(p):
        raise NativeLibraryMissing(f"{p} not found: run `make native` (or __graft_entry__.build())")
    return p

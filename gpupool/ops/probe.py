"""ctypes binding for libmi355x_probe.so — the gfx950 HIP readiness probe (probe.hip).

``init()`` warms every HIP context once (done by the long-lived node agent at start-up), so a
claim-time ``run()`` pays only its kernels. ``run()`` releases the GIL (ctypes does), so probes of
different GPUs run concurrently from a thread pool.
"""
from __future__ import annotations

import ctypes
import functools
import json
import threading

from . import native_path

_lib = None
_lock = threading.Lock()
_count: int | None = None


def lib() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            l = ctypes.CDLL(native_path("libmi355x_probe.so"))
            l.mi355x_probe_init.restype = ctypes.c_int
            l.mi355x_probe_init.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
            l.mi355x_probe_device_count.restype = ctypes.c_int
            l.mi355x_probe_identify.restype = ctypes.c_void_p
            l.mi355x_probe_identify.argtypes = [ctypes.c_int]
            l.mi355x_probe_run.restype = ctypes.c_void_p
            l.mi355x_probe_run.argtypes = [ctypes.c_int, ctypes.c_char_p]
            l.mi355x_probe_free.argtypes = [ctypes.c_void_p]
            l.mi355x_probe_peer.restype = ctypes.c_void_p
            l.mi355x_probe_peer.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p]
            if hasattr(l, "mi355x_probe_peer_ring"):  # absent from a library built before it
                l.mi355x_probe_peer_ring.restype = ctypes.c_void_p
                l.mi355x_probe_peer_ring.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                                     ctypes.c_char_p]
            l.mi355x_probe_trim.restype = ctypes.c_int
            l.mi355x_probe_trim.argtypes = [ctypes.c_int]
            l.mi355x_probe_hbm_sweep.restype = ctypes.c_void_p
            l.mi355x_probe_hbm_sweep.argtypes = [ctypes.c_int, ctypes.c_char_p]
            l.mi355x_probe_sweep_alloc.restype = ctypes.c_int
            l.mi355x_probe_sweep_alloc.argtypes = [ctypes.c_int, ctypes.c_longlong]
            l.mi355x_probe_sweep_release.restype = ctypes.c_int
            l.mi355x_probe_sweep_release.argtypes = [ctypes.c_int]
            l.mi355x_probe_gemm_bf16.restype = ctypes.c_int
            l.mi355x_probe_gemm_bf16.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int]
            _lib = l
    return _lib


def _take(p) -> dict:
    if not p:
        raise RuntimeError("libmi355x_probe returned NULL")
    try:
        return json.loads(ctypes.string_at(p).decode())
    finally:
        lib().mi355x_probe_free(p)


def init() -> int:
    """Initialise HIP + warm all visible devices. Returns the HIP device count."""
    global _count
    if _count is not None:
        return _count
    err = ctypes.create_string_buffer(512)
    n = lib().mi355x_probe_init(err, len(err))
    if n < 0:
        raise RuntimeError(f"HIP probe init failed: {err.value.decode()}")
    _count = n
    return n


def identify(dev: int) -> dict:
    return _take(lib().mi355x_probe_identify(dev))


def run(dev: int, hbm_bytes: int = 1 << 30, mfma: bool = True, gemm_n: int = 4096,
        patterns: int = 2, gemm_reps: int = 1, gemm_tile: int = 256, **test_hooks: int) -> dict:
    """Probe HIP device ``dev``. ``gemm_tile`` 256 (default, the glds 256x256 kernel) or 128 (the
    older register-staged kernel, for A/B). ``test_hooks``: injectBitFlips=N / injectGemmFault=1
    corrupt the device buffers between compute and check so tests can prove the checkers catch
    faults."""
    opts = _run_opts(int(hbm_bytes), bool(mfma), int(gemm_n), int(patterns), int(gemm_reps),
                     int(gemm_tile), tuple(sorted((k, int(v)) for k, v in test_hooks.items())))
    return _take(lib().mi355x_probe_run(dev, opts))


@functools.lru_cache(maxsize=64)
def _run_opts(hbm_bytes: int, mfma: bool, gemm_n: int, patterns: int, gemm_reps: int,
              gemm_tile: int, hooks: tuple) -> bytes:
    # An agent probes with a handful of option sets: encode each once. Encoding it per claim cost
    # 0.05 ms on a CPU woken from idle (profiles/r4n_probe_idle_binding.json).
    return json.dumps({"hbmBytes": hbm_bytes, "mfma": mfma, "gemmN": gemm_n, "patterns": patterns,
                       "gemmReps": gemm_reps, "gemmTile": gemm_tile, **dict(hooks)}).encode()


def peer(src: int, dst: int, nbytes: int = 64 << 20) -> dict:
    """xGMI peer check src -> dst: pattern written on src, hipMemcpyPeer over the link, every bit
    verified on dst; reports GB/s. ``src == dst`` exercises the same path as a local copy."""
    opts = json.dumps({"bytes": int(nbytes)})
    return _take(lib().mi355x_probe_peer(src, dst, opts.encode()))


def peer_ring(ordinals: list[int], nbytes: int = 64 << 20) -> dict:
    """The xGMI ring in one call: link i copies ordinals[i] -> ordinals[i+1] (wrapping), every link
    concurrently, then each receiver verifies every bit. -> {"links": [...], "passed"}."""
    n = len(ordinals)
    if n < 2:
        raise ValueError("a ring needs at least 2 entries")
    if not hasattr(lib(), "mi355x_probe_peer_ring"):
        raise RuntimeError("libmi355x_probe.so predates the ring check: rebuild it")
    arr = (ctypes.c_int * n)(*[int(o) for o in ordinals])
    opts = json.dumps({"bytes": int(nbytes)})
    return _take(lib().mi355x_probe_peer_ring(arr, n, opts.encode()))


def hip_uuid_map() -> dict[str, int]:
    """hipUUID ("GPU-<serial>") -> HIP ordinal for every visible device."""
    n = init()
    out = {}
    for d in range(n):
        info = identify(d)
        if info.get("hipUUID"):
            out[info["hipUUID"].lower()] = d
    return out


def trim(idle_ms: int = 0) -> int:
    """Free the probe arenas (kept between probes to skip a ~1.2 GiB hipMalloc) that have been idle
    for at least ``idle_ms``; returns how many were freed."""
    return int(lib().mi355x_probe_trim(int(idle_ms)))


def hbm_sweep(dev: int, offset: int, nbytes: int = 16 << 30, reserve: int = 4 << 30,
              keep: bool = False, **test_hooks: int) -> dict:
    """Pattern-test HBM window [offset, offset+nbytes) of a buffer spanning all free HBM minus
    ``reserve`` (the rotating sweep that covers the whole 288 GB over successive calls). With
    ``keep`` the big buffer stays allocated for the next window (free it with sweep_release)."""
    opts = json.dumps({"offset": int(offset), "bytes": int(nbytes), "reserve": int(reserve),
                       "keep": bool(keep), **{k: int(v) for k, v in test_hooks.items()}})
    return _take(lib().mi355x_probe_hbm_sweep(dev, opts.encode()))


def sweep_alloc(dev: int, reserve: int = 4 << 30) -> int:
    """Allocate the sweep buffer (all free HBM minus ``reserve``) without blocking probes: 1
    allocated, 0 already held, < 0 error."""
    return int(lib().mi355x_probe_sweep_alloc(dev, int(reserve)))


def sweep_release(dev: int) -> int:
    """Free the sweep buffer (seconds for ~280 GB; probes of the device are not blocked)."""
    return int(lib().mi355x_probe_sweep_release(dev))


def gemm_bf16(dev: int, a_ptr: int, bt_ptr: int, c_ptr: int, m: int, n: int, k: int) -> None:
    """The probe's production MFMA GEMM on caller HOST buffers (C fp32 [m,n] = A bf16 [m,k] x
    Bt bf16 [n,k]^T; e.g. CPU torch tensors' ``data_ptr()``), for independent numerics checks."""
    rc = lib().mi355x_probe_gemm_bf16(dev, a_ptr, bt_ptr, c_ptr, m, n, k)
    if rc != 0:
        raise ValueError(f"mi355x_probe_gemm_bf16 failed (rc={rc}): m,n % 256 and k % 64 must be "
                         f"0 and the device index valid")

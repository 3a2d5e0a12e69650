"""A/B: what the probe helper (gpupool/agent/probehost.py) adds to one claim-time probe over the
in-process library call, on a CPU coming out of idle (the claim path's situation).

Variants: inproc (libmi355x_probe.so in this process), helper with no spinning, helper with a
"wake" sent ~0.15 ms ahead (as the claim path does after selecting its GPUs) and the helper polling
its pipe for 3 ms after a message, and the same plus the caller polling for the reply. Each
iteration idles ``--idle-ms`` first. Prints one JSON line; run on the GPU box:
    python scripts/helper_overhead_ab.py > gpurun_out/helper_ab.json
With ``--backend sim`` it runs the simulated kernels (CPU dry run)."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def stats(xs: list[float]) -> dict:
    xs = sorted(xs)
    return {"p50": round(statistics.median(xs), 4), "p90": round(xs[int(len(xs) * 0.9)], 4),
            "n": len(xs)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="hip", choices=["hip", "sim"])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--idle-ms", type=float, default=20.0)
    ap.add_argument("--gap-ms", type=float, default=0.15, help="wake -> probe request gap")
    a = ap.parse_args()
    sys.setswitchinterval(0.00005)  # the agent's setting
    from gpupool.agent import probehost
    probehost.start_spawner()  # before anything touches the GPU
    devs = [{"uuid": "gpu0", "index": 0, "hipUUID": ""}]
    out: dict = {"backend": a.backend, "iters": a.iters, "idle_ms": a.idle_ms}
    args = {"hipUUID": "", "hbmBytes": 1 << 30, "mfma": True, "gemmN": 2048, "overlap": 1,
            "hooks": {}, "dev": {"uuid": "gpu0"}, "opts": {}}
    for name, child_spin, caller_spin, wake in (("helper_nospin", 0, 0, False),
                                                ("helper_wake_childspin", 3, 0, True),
                                                ("helper_wake_bothspin", 3, 2, True)):
        probehost.Helper.CALLER_SPIN_S = caller_spin / 1e3
        pool = probehost.HelperPool(a.backend, sim_ms=0.85, fabric_idle_s=0)
        orig = pool._gpu_spec
        pool._gpu_spec = lambda d, f=orig, s=child_spin: {**f(d), "spinS": s / 1e3}
        pool.start(devs)
        h = pool.get("gpu0")
        wall, over = [], []
        for i in range(a.iters + 5):
            time.sleep(a.idle_ms / 1e3)
            t0 = time.perf_counter()
            if wake:
                h.notify("wake")
            t1 = time.perf_counter()
            while time.perf_counter() - t1 < a.gap_ms / 1e3:
                pass
            t2 = time.perf_counter()
            r = h.call("probe", args, 10)
            dt = (time.perf_counter() - t2) * 1e3
            if i >= 5:
                wall.append(dt)
                over.append(dt - float(r.get("ms") or 0))
        out[name] = {"call_ms": stats(wall), "overhead_ms": stats(over)}
        pool.stop()
    if a.backend == "hip":
        from gpupool.ops import probe as hp
        hp.init()
        wall, over = [], []
        for i in range(a.iters + 5):
            time.sleep(a.idle_ms / 1e3)
            t0 = time.perf_counter()
            r = hp.run(0, hbm_bytes=1 << 30, gemm_n=2048, overlap=1)
            dt = (time.perf_counter() - t0) * 1e3
            if i >= 5:
                wall.append(dt)
                over.append(dt - float(r.get("ms") or 0))
        out["inproc"] = {"call_ms": stats(wall), "overhead_ms": stats(over)}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

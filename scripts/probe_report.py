"""Print one default claim-time probe result and a few HBM sweep windows (real MI355X)."""
import json
import sys
import time

sys.path.insert(0, ".")
from gpupool.ops import probe  # noqa: E402

probe.init()
out = {"probe": probe.run(0, hbm_bytes=1 << 30)}
t0 = time.perf_counter()
w = [probe.hbm_sweep(0, i * (16 << 30), 16 << 30, keep=True) for i in range(4)]
out["sweep_windows"] = w
out["sweep_4x16GiB_wall_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
t0 = time.perf_counter()
probe.sweep_release(0)
out["sweep_release_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
t0 = time.perf_counter()
full = []
off = 0
span = w[0]["span"]
while off < span:
    r = probe.hbm_sweep(0, off, 32 << 30, keep=True)
    full.append(r)
    off += r["bytes"]
probe.sweep_release(0)
out["full_sweep"] = {"windows": len(full), "span": span, "wall_ms": round((time.perf_counter() - t0) * 1e3, 2),
                     "all_passed": all(r["passed"] for r in full),
                     "min_GBps": min(r["GBps"] for r in full)}
out["probe_after_sweep"] = probe.run(0, hbm_bytes=1 << 30)
print(json.dumps(out, indent=1))

"""Host-side overhead of one claim-time probe call (ctypes + JSON result) on the agent's path:
Python wall time of gpupool.ops.probe.run vs the library's own ``ms`` (hipSetDevice -> result
written), median over interleaved rounds, alone and with a Python thread competing for the GIL."""
from __future__ import annotations

import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpupool.agent.prober import Prober  # noqa: E402
from gpupool.ops import probe  # noqa: E402


def main() -> int:
    sys.setswitchinterval(0.0005)  # the agent's setting (gpupool/agent/__main__.py)
    probe.init()
    probe.run(0)  # warm: arena allocated, kernels loaded
    out = {}
    for label, busy, sw in (("alone", False, 0.0005), ("gil_contended_500us", True, 0.0005),
                            ("gil_contended_100us", True, 0.0001),
                            ("gil_contended_50us", True, 0.00005)):
        sys.setswitchinterval(sw)
        stop = threading.Event()

        def spin():
            x = 0
            while not stop.is_set():
                x += 1
        t = threading.Thread(target=spin, daemon=True)
        if busy:
            t.start()
        walls, libs = [], []
        for _ in range(40):
            t0 = time.perf_counter()
            r = probe.run(0)
            walls.append((time.perf_counter() - t0) * 1e3)
            libs.append(r["ms"])
            assert r["passed"], r
        stop.set()
        out[label] = {"wall_ms": round(statistics.median(walls), 3),
                      "lib_ms": round(statistics.median(libs), 3),
                      "overhead_ms": round(statistics.median(w - m for w, m in zip(walls, libs)), 3),
                      "switch_interval_s": sys.getswitchinterval()}
    sys.setswitchinterval(0.0005)
    # the agent's wrapper (explain + floors) around the same call
    pr = Prober("inproc")
    dev = {"uuid": "gpu0", "hipUUID": probe.identify(0).get("hipUUID", ""), "index": 0}
    walls = []
    for _ in range(40):
        t0 = time.perf_counter()
        r = pr.probe_many([dev], {"enabled": True, "hbmBytes": 1 << 30})[0]
        walls.append((time.perf_counter() - t0) * 1e3)
    out["agent_prober"] = {"wall_ms": round(statistics.median(walls), 3), "passed": r.get("passed")}
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())

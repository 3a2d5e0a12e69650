"""Where the claim RPC's time goes outside the agent's own claim phases.

Starts one fake (or, with --backend amdsmi, real) node agent without a manager, then repeats
claim -> release of one GPU through the agent's RPC socket, timing each round trip on the client
and comparing it with the phases the agent reports (``timingsMs``). The difference is the RPC
cost: HTTP parse, executor hop, JSON encode, socket. Also times trivial requests (/healthz,
/v1/node?pool=) for the floor of one round trip.

    python scripts/agent_rpc_overhead.py [--n 50] [--backend fake|amdsmi] [--out F]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpupool.testing.cluster import Cluster, NodeSpec  # noqa: E402


def p50(xs):
    return round(statistics.median(xs), 3) if xs else None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50)
    ap.add_argument("--backend", default="fake")
    ap.add_argument("--out")
    ap.add_argument("--agent-arg", action="append", default=[], help="extra agent flag (repeat)")
    a = ap.parse_args()
    wd = tempfile.mkdtemp(prefix="rpcov")
    node = NodeSpec("n0", backend=a.backend, count=1 if a.backend != "fake" else -1,
                    extra_args=list(a.agent_arg))
    c = Cluster(wd, nodes=[node], manager=False, kinds="mi355x")
    c.start()
    try:
        from gpupool.kube import Client
        cl = Client("unix://" + c.agent_socket("n0"), c.agent_token)
        rt, inner, probe, ex_in, ex_out = [], [], [], [], []
        phases: dict[str, list[float]] = {}
        health, view = [], []
        for i in range(a.n + 3):
            t0 = time.perf_counter()
            r = cl.request("POST", "/v1/claims", {"poolUID": "bench-uid", "pool": "default/b",
                                                  "count": 1, "probe": {"enabled": True,
                                                                        "hbmBytes": 1 << 30}})
            dt = (time.perf_counter() - t0) * 1e3
            assert r["ok"], r
            uu = [d["uuid"] for d in r["devices"]]
            t1 = time.perf_counter()
            cl.request("GET", "/v1/node?pool=bench-uid")
            dv = (time.perf_counter() - t1) * 1e3
            t2 = time.perf_counter()
            cl.request("GET", "/healthz")
            dh = (time.perf_counter() - t2) * 1e3
            cl.request("POST", "/v1/release", {"poolUID": "bench-uid", "uuids": uu})
            if i < 3:
                continue
            rt.append(dt)
            inner.append(sum(r["timingsMs"].values()))
            probe.append(r["timingsMs"].get("probe", 0.0))
            for k, v in r["timingsMs"].items():
                phases.setdefault(k, []).append(v)
            ex_in.append(r["timingsMs"].get("executorIn", 0.0))
            ex_out.append(r["timingsMs"].get("executorOut", 0.0))
            view.append(dv)
            health.append(dh)
            time.sleep(0.02)
        out = {"backend": a.backend, "n": a.n, "claim_rtt_p50_ms": p50(rt),
               "claim_phases_p50_ms": p50(inner), "probe_p50_ms": p50(probe),
               "rpc_overhead_p50_ms": p50([x - y for x, y in zip(rt, inner)]),
               "executor_in_p50_ms": p50(ex_in), "executor_out_p50_ms": p50(ex_out),
               "pool_view_rtt_p50_ms": p50(view), "healthz_rtt_p50_ms": p50(health),
               "agent_args": a.agent_arg, "phases_p50_ms": {k: p50(v) for k, v in phases.items()}}
        print(json.dumps(out), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(out, f, indent=1)
    finally:
        c.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

"""Control-plane scale: many fake 8x MI355X nodes, many pools at once.

The headline bench times one pool on one node. A production cluster has many nodes, each with its
own agent (one manager long-poll feed and one view cache entry per node), and pools created in
bursts. This starts N fake nodes (agent + fake kubelet each, launched in parallel), then creates P
pools of R GPUs without a nodeName (the manager places them) all at once and times:

* create-to-Ready per pool (p50 / p90 / max) and until the last pool is Ready,
* scale-to-zero of all pools (release) the same way,
* the manager's CPU seconds and RSS over the run, and the agents' RPC counts.

    python scripts/scale_bench.py [--nodes 16] [--pools 48] [--replicas 2] [--out F]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpupool.kube import MI355XPOOLS  # noqa: E402
from gpupool.testing.cluster import Cluster, NodeSpec  # noqa: E402


def pstats(xs: list[float]) -> dict:
    xs = sorted(xs)
    if not xs:
        return {}
    return {"n": len(xs), "p50_s": round(statistics.median(xs), 4),
            "p90_s": round(xs[min(len(xs) - 1, int(0.9 * len(xs)))], 4), "max_s": round(xs[-1], 4)}


def proc_usage(pid: int) -> dict:
    with open(f"/proc/{pid}/stat") as f:
        fields = f.read().rsplit(")", 1)[1].split()
    tick = os.sysconf("SC_CLK_TCK")
    cpu = (int(fields[11]) + int(fields[12])) / tick
    rss = 0
    with open(f"/proc/{pid}/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                rss = int(line.split()[1]) * 1024
    return {"cpu_s": round(cpu, 3), "rss_mib": round(rss / 2**20, 1)}


def wait_all(k, names: list[str], pred, t0: float, timeout: float) -> dict[str, float]:
    """Time at which each pool first satisfied ``pred``, from a watch stream (polling lists of
    every pool would load the apiserver-sim more than the operator does). A watch that ends early
    (the server closes it, or its resourceVersion is too old) is resumed from a fresh list."""
    done: dict[str, float] = {}
    want = set(names)
    deadline = time.monotonic() + timeout
    while len(done) < len(want) and time.monotonic() < deadline:
        lst = k.list(MI355XPOOLS, "default")
        for o in lst["items"]:
            n = o["metadata"]["name"]
            if n in want and n not in done and pred(o):
                done[n] = time.perf_counter() - t0
        if len(done) == len(want):
            break
        stop = threading.Event()
        timer = threading.Timer(max(0.1, deadline - time.monotonic()), stop.set)
        timer.start()
        try:
            for ev in k.watch(MI355XPOOLS, "default",
                              resource_version=lst["metadata"]["resourceVersion"],
                              timeout_seconds=int(deadline - time.monotonic()) + 1, stop=stop):
                o = ev.get("object") or {}
                n = (o.get("metadata") or {}).get("name")
                if ev.get("type") in ("ADDED", "MODIFIED") and n in want and n not in done \
                        and pred(o):
                    done[n] = time.perf_counter() - t0
                if len(done) == len(want):
                    break
        except Exception:  # a broken stream: list and watch again
            time.sleep(0.05)
        finally:
            stop.set()
            timer.cancel()
    return done


def ready(r: int):
    def pred(o):
        st = o.get("status") or {}
        c = {x["type"]: x for x in st.get("conditions", [])}
        return st.get("observedGeneration") == o["metadata"].get("generation") and \
            st.get("readyReplicas") == r and len(st.get("devices", [])) == r and \
            c.get("Ready", {}).get("status") == "True"
    return pred


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=16)
    ap.add_argument("--pools", type=int, default=48)
    ap.add_argument("--replicas", type=int, default=2)
    ap.add_argument("--workers", type=int, default=8, help="manager reconcile workers")
    ap.add_argument("--timeout", type=float, default=180.0)
    ap.add_argument("--out")
    a = ap.parse_args()
    assert a.pools * a.replicas <= a.nodes * 8, "more GPUs requested than the nodes have"
    wd = tempfile.mkdtemp(prefix="scale")
    nodes = [NodeSpec(f"node-{i:03d}") for i in range(a.nodes)]
    c = Cluster(wd, nodes=nodes, manager=False, sample_interval=2.0,
                manager_args=["--workers", str(a.workers)])
    t_start = time.perf_counter()
    c.start_apiserver()
    errs: list[BaseException] = []

    def up(n: NodeSpec) -> None:
        try:
            c.start_kubelet(n)
            c.start_agent(n)
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append(e)

    ts = [threading.Thread(target=up, args=(n,)) for n in nodes]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        c.stop()
        raise errs[0]
    c.start_manager()
    startup = time.perf_counter() - t_start
    k = c.client
    try:
        names = [f"pool-{i:03d}" for i in range(a.pools)]
        mgr = c.procs["manager"].pid
        u0 = proc_usage(mgr)
        t0 = time.perf_counter()
        for n in names:
            k.create(MI355XPOOLS, {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xPool",
                                   "metadata": {"name": n},
                                   "spec": {"replicas": a.replicas,
                                            "probe": {"enabled": True, "hbmBytes": 1 << 30}}},
                     "default")
        created = time.perf_counter() - t0
        up_t = wait_all(k, names, ready(a.replicas), t0, a.timeout)
        u1 = proc_usage(mgr)
        placed: dict[str, int] = {}
        stuck = []
        for o in k.list(MI355XPOOLS, "default")["items"]:
            if o["metadata"]["name"] not in up_t and len(stuck) < 5:  # diagnostics
                st = o.get("status") or {}
                entry = {"pool": o["metadata"]["name"],
                         "conditions": {x["type"]: [x["status"], x.get("reason"),
                                                    (x.get("message") or "")[:200]]
                                        for x in st.get("conditions", [])},
                         "status_devices": st.get("devices")}
                node = st.get("nodeName")
                if node:
                    try:
                        view = c.agent_request(node, "GET", "/v1/node")
                        entry["agent_devices"] = [d for d in view.get("devices", [])
                                                  if d.get("poolUID") == o["metadata"]["uid"]]
                        entry["agent_gen"] = view.get("gen")
                        m = c.agent_request(node, "GET", "/metrics")
                        entry["agent_metrics"] = [ln for ln in m.splitlines()
                                                  if "plugin" in ln or "stream" in ln
                                                  or "advert" in ln][:20]
                    except Exception as e:  # noqa: BLE001 - diagnostics only
                        entry["agent_error"] = repr(e)
                stuck.append(entry)
            for d in (o.get("status") or {}).get("devices", []):
                placed[d["node"]] = placed.get(d["node"], 0) + 1
        t1 = time.perf_counter()
        for n in names:
            k.patch(MI355XPOOLS, n, {"spec": {"replicas": 0}}, "default")
        down_t = wait_all(k, names, ready(0), t1, a.timeout)
        u2 = proc_usage(mgr)
        metrics: dict[str, float] = {}
        for line in c.manager_metrics().splitlines():
            if line.startswith("#") or " " not in line:
                continue
            name = line.split("{", 1)[0].split(" ", 1)[0]
            if name in ("gpupool_reconcile_span_seconds_sum", "gpupool_reconcile_span_seconds_count"):
                span = line.split('span="', 1)[1].split('"', 1)[0] if 'span="' in line else "?"
                key = ("span_s_" if name.endswith("_sum") else "span_n_") + span
                metrics[key] = metrics.get(key, 0.0) + float(line.rsplit(" ", 1)[1])
            if name == "gpupool_reconcile_total":  # by result as well
                res = line.split('result="', 1)[1].split('"', 1)[0] if 'result="' in line else "?"
                metrics["reconcile_" + res] = metrics.get("reconcile_" + res, 0.0) + \
                    float(line.rsplit(" ", 1)[1])
            if name in ("gpupool_reconcile_total", "gpupool_agent_view_cache_hits_total",
                        "gpupool_reconcile_duration_seconds_sum",
                        "gpupool_reconcile_duration_seconds_count"):
                metrics[name] = metrics.get(name, 0.0) + float(line.rsplit(" ", 1)[1])
        out = {"nodes": a.nodes, "pools": a.pools, "replicas": a.replicas,
               "gpus_claimed": a.pools * a.replicas, "manager_workers": a.workers,
               "startup_s": round(startup, 2), "create_requests_s": round(created, 3),
               "ready": {**pstats(list(up_t.values())), "all_ready": len(up_t) == a.pools,
                         "last_s": round(max(up_t.values()), 4) if up_t else None},
               "scale_to_zero": {**pstats(list(down_t.values())), "all_done": len(down_t) == a.pools,
                                 "last_s": round(max(down_t.values()), 4) if down_t else None},
               "not_ready": stuck,
               "gpus_per_node_used": {"min": min(placed.values()) if placed else 0,
                                      "max": max(placed.values()) if placed else 0,
                                      "nodes_used": len(placed)},
               "manager": {"cpu_s_scale_up": round(u1["cpu_s"] - u0["cpu_s"], 3),
                           "cpu_s_scale_down": round(u2["cpu_s"] - u1["cpu_s"], 3),
                           "rss_mib": u2["rss_mib"],
                           "reconciles": int(metrics.get("gpupool_reconcile_total", 0)),
                           "reconcile_s_avg": round(metrics.get("gpupool_reconcile_duration_seconds_sum", 0)
                                                    / max(1, metrics.get(
                                                        "gpupool_reconcile_duration_seconds_count", 0)), 4),
                           "view_cache_hits": int(metrics.get("gpupool_agent_view_cache_hits_total", 0)),
                           "reconciles_by_result": {k2[len("reconcile_"):]: int(v) for k2, v in
                                                    metrics.items() if k2.startswith("reconcile_")},
                           # where the passes spent their time: span -> [count, total s]
                           "spans": {k2[len("span_s_"):]: [int(metrics.get("span_n_" + k2[7:], 0)),
                                                           round(v, 3)]
                                     for k2, v in metrics.items() if k2.startswith("span_s_")}},
               "host_cpus": os.cpu_count()}
        print(json.dumps(out), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(out, f, indent=1)
    finally:
        c.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

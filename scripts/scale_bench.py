"""Control-plane scale: many fake 8x MI355X nodes, many pools at once.

The headline bench times one pool on one node. A production cluster has many nodes, each with its
own agent (one manager long-poll feed and one view cache entry per node), and pools created in
bursts. This starts N fake nodes (agent + fake kubelet each, launched in parallel), then creates P
pools of R GPUs without a nodeName (the manager places them) all at once and times:

* create-to-Ready per pool (p50 / p90 / max) and until the last pool is Ready,
* scale-to-zero of all pools (release) the same way,
* the manager's CPU seconds and RSS over the run, and the agents' RPC counts.

    python scripts/scale_bench.py [--nodes 16] [--pools 48] [--replicas 2] [--out F]

``--mode jobs`` measures the Mi355xJob gang scheduler and the manager's pod cache instead: N Node
objects (allocatable 8 GPUs each, kubelet-style heartbeats every 10 s), F filler pods (one GPU pod
per node, the rest CPU-only), then G gangs submitted at once. It reports the time to place every
gang, apiserver LIST counts (total and after the caches synced, per minute), node events by
whether a placement fact changed, and the manager's CPU and RSS:

    python scripts/scale_bench.py --mode jobs --nodes 64 --filler-pods 5000 --gangs 200
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


def wait_all(k, names: list[str], pred, t0: float, timeout: float, res=MI355XPOOLS) -> dict[str, float]:
    """Time at which each pool first satisfied ``pred``, from a watch stream (polling lists of
    every pool would load the apiserver-sim more than the operator does). A watch that ends early
    (the server closes it, or its resourceVersion is too old) is resumed from a fresh list."""
    done: dict[str, float] = {}
    want = set(names)
    deadline = time.monotonic() + timeout
    while len(done) < len(want) and time.monotonic() < deadline:
        lst = k.list(res, "default")
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
            for ev in k.watch(res, "default",
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


def _metrics(text: str) -> dict[str, float]:
    out: dict[str, float] = {}
    for line in text.splitlines():
        if line.startswith("#") or " " not in line:
            continue
        key, _, val = line.rpartition(" ")
        try:
            out[key] = out.get(key, 0.0) + float(val)
        except ValueError:
            pass
    return out


def _sum(m: dict[str, float], prefix: str) -> float:
    return sum(v for k, v in m.items() if k.startswith(prefix))


def jobs_mode(a) -> int:
    """Gang placement and the pod cache at cluster scale (no agents: jobs place on Node
    allocatable; their pods stay Pending, as nothing runs them — placement is what is timed)."""
    from gpupool.kube import MI355XJOBS, NODES, PODS, Client
    wd = tempfile.mkdtemp(prefix="scalejobs")
    c = Cluster(wd, nodes=[], kinds="job", manager_bin=a.manager_bin, agent_auth="token",
                manager_args=["--workers", str(a.workers), "--resync", "10s"])
    c.start_apiserver()
    k = c.client
    t_setup = time.perf_counter()
    names = [f"gpu-{i:03d}" for i in range(a.nodes)]
    for n in names:
        k.create(NODES, {"apiVersion": "v1", "kind": "Node",
                         "metadata": {"name": n, "labels": {"kubernetes.io/hostname": n}}})
        k.patch(NODES, n, {"status": {"capacity": {"amd.com/gpu": "8", "cpu": "192"},
                                      "allocatable": {"amd.com/gpu": "8", "cpu": "192"},
                                      "conditions": [{"type": "Ready", "status": "True",
                                                      "lastHeartbeatTime": "t0"}]}},
                sub="status", ptype="strategic")
    # filler pods: one 1-GPU pod per node (GPUs in use), the rest CPU-only, all Running
    cl = [Client(c.url) for _ in range(8)]

    def fill(w: int) -> None:
        for i in range(w, a.filler_pods, 8):
            gpu = i < a.nodes
            pod = {"apiVersion": "v1", "kind": "Pod",
                   "metadata": {"name": f"filler-{i:05d}", "labels": {"app": "filler"}},
                   "spec": {"nodeName": names[i % a.nodes], "containers": [{
                       "name": "c", "image": "x", "resources": {"limits": {
                           **({"amd.com/gpu": "1"} if gpu else {}), "cpu": "1"}}}]},
                   "status": {"phase": "Running", "podIP": f"10.{i // 65536}.{i // 256 % 256}.{i % 256}"}}
            cl[w].create(PODS, pod, f"team-{i % 20}")
    ts = [threading.Thread(target=fill, args=(w,)) for w in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    setup_s = time.perf_counter() - t_setup
    stop = threading.Event()

    def heartbeats() -> None:  # what every kubelet does every 10 s (node-status-update-frequency)
        hb = Client(c.url)
        n = 0
        while not stop.wait(10.0 / max(1, a.nodes)):
            node = names[n % a.nodes]
            n += 1
            hb.patch(NODES, node, {"status": {"conditions": [{"type": "Ready", "status": "True",
                                                              "lastHeartbeatTime": f"t{n}"}]}},
                     sub="status", ptype="strategic")
    threading.Thread(target=heartbeats, daemon=True).start()

    def runner() -> None:  # the kubelets' part for gang pods: each one starts (Running, a pod IP)
        r = Client(c.url)
        rv = r.list(PODS, None, label_selector="gpupool.amd.com/job-name")["metadata"]["resourceVersion"]
        n = 0
        while not stop.is_set():
            try:
                for ev in r.watch(PODS, None, resource_version=rv, stop=stop, timeout_seconds=30,
                                  label_selector="gpupool.amd.com/job-name"):
                    o = ev.get("object") or {}
                    rv = (o.get("metadata") or {}).get("resourceVersion", rv)
                    if ev.get("type") == "ADDED" and not (o.get("status") or {}).get("podIP"):
                        n += 1
                        r.patch(PODS, o["metadata"]["name"], {"status": {
                            "phase": "Running", "podIP": f"10.200.{n // 256 % 256}.{n % 256}"}},
                            o["metadata"]["namespace"], sub="status")
            except Exception:  # noqa: BLE001 - the watch resumes
                time.sleep(0.1)
    threading.Thread(target=runner, daemon=True).start()
    c.start_manager()
    mgr = c.procs["manager"].pid
    deadline = time.monotonic() + 300
    while time.monotonic() < deadline and "controllers running" not in c.log("manager"):
        time.sleep(0.2)  # every informer cache synced (the manager starts its workers then)
    time.sleep(2.0)
    s0 = _metrics(k.request("GET", "/metrics"))
    m0 = _metrics(c.manager_metrics())
    u0 = proc_usage(mgr)
    jobs = [f"gang-{i:03d}" for i in range(a.gangs)]
    t0 = time.perf_counter()
    for j in jobs:
        k.create(MI355XJOBS, {"apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xJob",
                              "metadata": {"name": j},
                              "spec": {"replicas": a.gang_size, "gpusPerReplica": 1,
                                       "template": {"spec": {"containers": [{
                                           "name": "m", "command": ["sleep", "1"]}]}}}}, "default")

    def scheduled(o):
        st = o.get("status") or {}
        c2 = {x["type"]: x for x in st.get("conditions", [])}
        return c2.get("Scheduled", {}).get("status") == "True" and \
            len(st.get("placement") or []) == a.gang_size

    def running(o):
        return ((o.get("status") or {}).get("phase")) == "Running"
    all_running = {}
    # followed through one watch (a LIST per poll would load the apiserver like the operator)
    got: dict[str, dict[str, float]] = {"placed": {}, "running": {}}

    def both(o):
        n = o["metadata"]["name"]
        now = time.perf_counter() - t0
        if scheduled(o):
            got["placed"].setdefault(n, now)
        if running(o):
            got["running"].setdefault(n, now)
        return n in got["running"]
    wait_all(k, jobs, both, t0, a.timeout, res=MI355XJOBS)
    done, all_running = got["placed"], got["running"]
    placed_s = max(done.values()) if done else a.timeout
    u1 = proc_usage(mgr)
    s1 = _metrics(k.request("GET", "/metrics"))
    m1 = _metrics(c.manager_metrics())
    # steady state: a minute of heartbeats with the placed gangs (and any unplaced) in place
    time.sleep(a.steady_s)
    s2 = _metrics(k.request("GET", "/metrics"))
    m2 = _metrics(c.manager_metrics())
    u2 = proc_usage(mgr)
    stop.set()
    lists = lambda s: {k2.split('"')[1]: int(v) for k2, v in s.items()  # noqa: E731
                       if k2.startswith("apiserver_list_total")}
    l0, l1, l2 = lists(s0), lists(s1), lists(s2)
    diff = lambda x, y: {r: y.get(r, 0) - x.get(r, 0) for r in sorted(set(x) | set(y))  # noqa: E731
                         if y.get(r, 0) - x.get(r, 0)}
    out = {"mode": "jobs", "nodes": a.nodes, "filler_pods": a.filler_pods, "gangs": a.gangs,
           "gang_size": a.gang_size, "manager_bin": a.manager_bin or "build/native/gpupool-manager",
           "setup_s": round(setup_s, 1),
           "placement": {**pstats(list(done.values())), "all_placed": len(done) == len(jobs),
                         "placed": len(done), "wall_s": round(placed_s, 3)},
           "running": {**pstats(list(all_running.values())),
                       "all_running": len(all_running) == len(jobs)},
           "apiserver_lists": {"at_manager_sync": l0, "during_placement": diff(l0, l1),
                               "steady_per_min": {r: round(v * 60.0 / a.steady_s, 1)
                                                  for r, v in diff(l1, l2).items()}},
           "node_events": {"relevant": _sum(m2, 'gpupool_node_events_total{relevant="true"'),
                           "ignored": _sum(m2, 'gpupool_node_events_total{relevant="false"')},
           "scheduler_reads": {k2.split("{", 1)[1].rstrip("}"): int(v) for k2, v in m2.items()
                               if k2.startswith("gpupool_job_scheduler_reads_total")},
           "reconciles": {"during_placement": int(_sum(m1, "gpupool_reconcile_total") -
                                                  _sum(m0, "gpupool_reconcile_total")),
                          "steady_per_min": round((_sum(m2, "gpupool_reconcile_total") -
                                                   _sum(m1, "gpupool_reconcile_total")) * 60.0 /
                                                  a.steady_s, 1),
                          "steady_per_min_by_label": {
                              k2.split("{", 1)[1].rstrip("}"): round((v - m1.get(k2, 0)) * 60.0 /
                                                                     a.steady_s, 1)
                              for k2, v in m2.items() if k2.startswith("gpupool_reconcile_total{")
                              and v - m1.get(k2, 0) > 0}},
           "manager": {"cpu_s_placement": round(u1["cpu_s"] - u0["cpu_s"], 3),
                       "cpu_s_steady_per_min": round((u2["cpu_s"] - u1["cpu_s"]) * 60.0 /
                                                     a.steady_s, 3),
                       "rss_mib_after_sync": u0["rss_mib"], "rss_mib_end": u2["rss_mib"]},
           "host_cpus": os.cpu_count()}
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    c.stop()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["pools", "jobs"], default="pools")
    ap.add_argument("--filler-pods", type=int, default=5000, help="jobs mode")
    ap.add_argument("--gangs", type=int, default=200, help="jobs mode")
    ap.add_argument("--gang-size", type=int, default=2, help="jobs mode: workers x 1 GPU")
    ap.add_argument("--steady-s", type=float, default=60.0, help="jobs mode: steady-state window")
    ap.add_argument("--manager-bin", default=None, help="jobs mode: another gpupool-manager build")
    ap.add_argument("--nodes", type=int, default=16)
    ap.add_argument("--pools", type=int, default=48)
    ap.add_argument("--replicas", type=int, default=2)
    ap.add_argument("--workers", type=int, default=8, help="manager reconcile workers")
    ap.add_argument("--timeout", type=float, default=180.0)
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.mode == "jobs":
        return jobs_mode(a)
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

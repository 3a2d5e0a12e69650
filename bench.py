#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): p50 reconcile-to-Ready latency + readyReplicas accuracy.

One *step* = one full declarative scale cycle of a ``Mi355xPool`` on one node:
  replicas 0 -> N   (timed: PATCH accepted by the apiserver -> watch sees status.readyReplicas == N,
                     Ready=True at the new observedGeneration; on the way the manager claims N GPUs
                     via the node agent, the agent probes every GPU with the gfx950 HIP kernels
                     (1 GiB HBM pattern test + bf16 MFMA GEMM, the CRD default) and advertises them
                     through the ROCm device plugin to the kubelet)
  accuracy check    (readyReplicas vs an independent ground truth: amd-smi CLI + ledger files +
                     kubelet allocatable; see gpupool/bench/ground_truth.py)
  replicas N -> 0   (drain + finalizer-free release, waited for; part of ms_per_step)

``value`` is the p50 over the K timed steps of the 0->N reconcile-to-Ready latency in seconds
(lower is better). With N GPUs visible (real MI355X) the agent uses the amdsmi backend and the
in-process HIP probe; without GPUs it falls back to the 8-GPU fake fixture with a simulated probe,
and says so in ``data``.

Launch contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 under
``torch.distributed.run`` every rank joins a gloo process group for the barriers and rank 0
drives the control plane, which manages all N GPUs of the node.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TARGET_S = 30.0  # p50 reconcile-to-Ready < 30 s (no published number)
METRIC = "p50 reconcile-to-Ready latency (s) + readyReplicas accuracy at replicas=1/2/4/8"


def _dist_init():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return rank, world


def _barrier(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def _sync_gpu(enabled: bool) -> None:
    if enabled:
        import torch
        torch.cuda.synchronize()


def _visible_gpus() -> int:
    # device_count() does not initialise HIP on this image (safe before spawning children)
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


def _gather_max(world: int, x: float) -> float:
    if world <= 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--backend", default="auto", choices=["auto", "real", "fake"])
    ap.add_argument("--hbm-bytes", type=int, default=1 << 30,
                    help="probe HBM bytes per GPU (CRD default 1 GiB)")
    ap.add_argument("--workdir", default="")
    ap.add_argument("--keep", action="store_true", help="keep the workdir (logs)")
    ap.add_argument("--timeout", type=float, default=120.0, help="per-transition timeout (s)")
    ap.add_argument("--health-steps", type=int, default=5,
                    help="fault->condition measurements after the timed steps (0 = skip)")
    args = ap.parse_args()

    rank, world = _dist_init()
    n = args.gpus
    visible = _visible_gpus()
    from gpupool.ops import native_dir
    have_probe = os.path.exists(os.path.join(native_dir(), "libmi355x_probe.so"))
    real = args.backend == "real" or (args.backend == "auto" and visible >= n and have_probe)

    cluster = None
    step_ms, lat, acc_ok, details = [], [], 0, []
    if rank == 0:
        from gpupool.kube import MI355XPOOLS
        from gpupool.testing.cluster import FIXTURE, Cluster, NodeSpec
        from gpupool.bench import ground_truth as gt
        workdir = args.workdir or tempfile.mkdtemp(prefix="gpupool-bench-")
        # fake mode: simulated probe latency calibrated to the measured real 1 GiB probe (2.6 ms,
        # profiles/r1_probe_ctypes_real.txt)
        node = NodeSpec("mi355x-node-0", backend="amdsmi" if real else "fake",
                        probe="inproc" if real else "simulated",
                        count=-1 if real else max(8, n),
                        extra_args=[] if real else ["--probe-sim-ms", "2.6"])
        cluster = Cluster(workdir, nodes=[node], sample_interval=1.0)
        cluster.start()  # all child processes exist before this process touches the GPU
        c = cluster.client
        ns, name = "default", "bench-pool"
        pool = c.create(MI355XPOOLS, {
            "apiVersion": "compute.my.domain/v1alpha1", "kind": "Mi355xPool",
            "metadata": {"name": name},
            "spec": {"replicas": 0, "nodeName": node.name,
                     "probe": {"enabled": True, "hbmBytes": args.hbm_bytes, "mfma": True}}}, ns)
        uid = pool["metadata"]["uid"]
        state_dir = os.path.join(workdir, f"state-{node.name}")

        def ready_at(r: int):
            def pred(o):
                if not o:
                    return False
                st = o.get("status") or {}
                conds = {x["type"]: x for x in st.get("conditions", [])}
                return st.get("observedGeneration") == o["metadata"]["generation"] and \
                    st.get("readyReplicas") == r and len(st.get("devices", [])) == r and \
                    conds.get("Ready", {}).get("status") == "True"
            return pred

        c.wait_for(MI355XPOOLS, name, ns, ready_at(0), timeout=args.timeout)

        def healthy_set() -> set[str]:
            if real:
                return gt.healthy_uuids_cli()
            return gt.healthy_uuids_fixture(node.fixture, cluster.faults_path(node.name), node.name)

        def cycle(timed: bool):
            t0 = time.perf_counter()
            c.patch(MI355XPOOLS, name, {"spec": {"replicas": n}}, ns)
            obj = c.wait_for(MI355XPOOLS, name, ns, ready_at(n), timeout=args.timeout)
            t_ready = time.perf_counter() - t0
            truth = gt.truth(c, node.name, uid, state_dir, "amd.com/gpu", healthy_set())
            ok = truth["ready"] == obj["status"]["readyReplicas"] == n
            c.patch(MI355XPOOLS, name, {"spec": {"replicas": 0}}, ns)
            c.wait_for(MI355XPOOLS, name, ns, ready_at(0), timeout=args.timeout)
            total = time.perf_counter() - t0
            probe_ms = [d.get("probe", {}).get("ms", 0.0) for d in obj["status"]["devices"]]
            return t_ready, total, ok, {"readySeconds": round(t_ready, 4), "truth": truth,
                                        "readyReplicas": obj["status"]["readyReplicas"],
                                        "probeMs": [round(x, 2) for x in probe_ms]}

        for _ in range(args.warmup):
            cycle(False)
    _barrier(world)
    _sync_gpu(real and rank == 0 and visible > 0)
    t_start = time.perf_counter()
    if rank == 0:
        for _ in range(args.steps):
            t_ready, total, ok, det = cycle(True)
            lat.append(t_ready)
            step_ms.append(total * 1e3)
            acc_ok += int(ok)
            details.append(det)
    _sync_gpu(real and rank == 0 and visible > 0)
    _barrier(world)
    elapsed = _gather_max(world, time.perf_counter() - t_start)

    health = {}
    if rank == 0 and args.health_steps > 0:
        # Secondary measurement, outside the timed region (BASELINE config 5): fault overlay on
        # one claimed GPU (uncorrectable ECC) -> HBMECCHealthy=False + Degraded=True on the pool,
        # and back after the fault clears. Event-driven: agent sample -> long-poll -> reconcile.
        c.patch(MI355XPOOLS, name, {"spec": {"replicas": 1, "replacePolicy": "Keep"}}, ns)
        obj = c.wait_for(MI355XPOOLS, name, ns, ready_at(1), timeout=args.timeout)
        victim = obj["status"]["devices"][0]["uuid"]

        def cond(o, t):
            return next((x for x in ((o or {}).get("status") or {}).get("conditions", [])
                         if x["type"] == t), {}).get("status")
        react, recover = [], []
        for _ in range(args.health_steps):
            t0 = time.perf_counter()
            cluster.set_faults(node.name, {"devices": {victim: {"ecc": {"uncorrectable": 1}}}})
            c.wait_for(MI355XPOOLS, name, ns, lambda o: cond(o, "HBMECCHealthy") == "False" and
                       cond(o, "Degraded") == "True", timeout=args.timeout)
            react.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            cluster.set_faults(node.name, {})
            c.wait_for(MI355XPOOLS, name, ns, lambda o: cond(o, "HBMECCHealthy") == "True" and
                       ready_at(1)(o), timeout=args.timeout)
            recover.append(time.perf_counter() - t0)
        health = {"fault_to_condition_p50_s": round(statistics.median(react), 4),
                  "fault_cleared_to_ready_p50_s": round(statistics.median(recover), 4),
                  "steps": args.health_steps}

    if rank == 0:
        try:
            metrics = cluster.manager_metrics()
        except Exception:
            metrics = ""
        try:
            traces = cluster.manager_traces(key=f"Mi355xPool/{ns}/{name}", n=256)
        except Exception:
            traces = []
        cluster.stop()
        # latency breakdown of the scale-up passes (the reconcile that claims): median per span
        claim_traces = [t for t in traces
                        if any(s["name"] == "agent:POST /v1/claims" for s in t["spans"])][:args.steps]
        span_ms: dict[str, list[float]] = {}
        for t in claim_traces:
            per: dict[str, float] = {}
            for s in t["spans"]:
                per[s["name"]] = per.get(s["name"], 0.0) + s["ms"]
            per["total"] = t["totalMs"]
            for k2, v in per.items():
                span_ms.setdefault(k2, []).append(v)
        span_p50 = {k2: round(statistics.median(v), 3) for k2, v in sorted(span_ms.items())}
        p50 = statistics.median(lat) if lat else float("nan")
        lat_sorted = sorted(lat)
        p90 = lat_sorted[min(len(lat_sorted) - 1, int(0.9 * len(lat_sorted)))] if lat else None
        accuracy = acc_ok / len(lat) if lat else None
        data = ("real MI355X: amdsmi discovery + gfx950 HIP probe (HBM %d MiB + bf16 MFMA) + "
                "device plugin -> fake kubelet" % (args.hbm_bytes >> 20)) if real else \
               ("synthetic: 8x MI355X fake fixture (no GPU visible), simulated probe, device "
                "plugin -> fake kubelet")
        out = {
            "metric": METRIC,
            "value": round(p50, 4),
            "unit": "s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / max(1, args.steps), 2),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": round(p50 / BASELINE_TARGET_S, 5),
            "dtype": "bf16",
            "data": data,
            "config": {
                "model": "Mi355xPool scale 0->N (BASELINE configs 2/3)",
                "global_batch": n,
                "seq_len": 0,
                "parallelism": f"replicas{n}",
                "backend": "amdsmi+hip" if real else "fake",
                "baseline_target_s": BASELINE_TARGET_S,
                "p90_s": round(p90, 4) if p90 is not None else None,
                "max_s": round(max(lat), 4) if lat else None,
                "readyReplicas_accuracy": accuracy,
                "world_size": world,
                "claim_pass_span_p50_ms": span_p50,
                "health_condition_latency": health,
                "steps_detail": details[:3],
            },
        }
        print(json.dumps(out), flush=True)
        if not args.keep and not args.workdir:
            shutil.rmtree(cluster.workdir, ignore_errors=True)
        else:
            print(f"# workdir kept: {cluster.workdir}", file=sys.stderr)
            with open(os.path.join(cluster.workdir, "manager_metrics.txt"), "w") as f:
                f.write(metrics)
            with open(os.path.join(cluster.workdir, "traces.json"), "w") as f:
                json.dump(traces, f, indent=1)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

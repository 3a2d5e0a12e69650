"""Collective check across the node's GPUs: ``python -m gpupool.parallel.rccl_check`` per rank.

The operator's promise to a multi-GPU pod is that its GPUs talk to each other: `torch.distributed`
over RCCL (backend "nccl" IS RCCL on ROCm) riding the xGMI mesh — the path DDP's gradient
all-reduce takes (gpupool/parallel/ddp.py). One process per GPU:

  * exactness: rank r contributes a buffer of r + 1 (fp32, exact to 2^24), so the sum must be
    world(world+1)/2 everywhere — a value only a real reduction over every rank's data produces.
    A rank that skipped the collective, or a local copy (world = 1 aside), keeps r + 1 and fails;
  * bandwidth: a bf16 buffer all-reduced ``--iters`` times, reported as algorithm and bus bandwidth
    (busbw = algbw * 2(n-1)/n, the ring all-reduce's per-link traffic — on an 8x MI355X node each
    of a GPU's 7 xGMI links carries one ring's share).

bench.py launches it once per rank after its timed region when N > 1 GPUs are real (each in its own
child process under a time limit, so a fabric problem cannot hang the bench) and reports it as
``config.rccl_allreduce``. ``--backend gloo --device cpu`` runs the same harness on CPU (tests).
"""
from __future__ import annotations

import argparse
import datetime as _dt
import json
import os
import time


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=int(os.environ.get("RANK", "0")))
    ap.add_argument("--world", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--local-rank", type=int, default=int(os.environ.get("LOCAL_RANK", "0")))
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, required=True)
    ap.add_argument("--bytes", type=int, default=256 << 20)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--inject", default="", choices=["", "skip-reduce"],
                    help="test hook: skip the exactness reduction on this rank")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    # its own rendezvous (a torchrun parent's agent store must not be reused)
    for k in [k for k in os.environ if k.startswith("TORCHELASTIC_")]:
        del os.environ[k]
    dev = torch.device(f"cuda:{a.local_rank}") if a.device == "cuda" else torch.device("cpu")
    if a.device == "cuda":
        torch.cuda.set_device(dev)
    dist.init_process_group(a.backend, init_method=f"tcp://{a.master_addr}:{a.master_port}",
                            rank=a.rank, world_size=a.world, timeout=_dt.timedelta(seconds=60))
    n = a.bytes // 2
    x = torch.ones(n, dtype=torch.bfloat16, device=dev)

    def sync():
        if a.device == "cuda":
            torch.cuda.synchronize(dev)
    chk = torch.full((1 << 16,), float(a.rank + 1), dtype=torch.float32, device=dev)
    if a.inject == "skip-reduce":
        dist.all_reduce(chk.clone())  # joins the collective (peers do not hang), drops the result
    else:
        dist.all_reduce(chk)
    want = a.world * (a.world + 1) // 2
    sync()
    got = chk.cpu()
    ok = bool((got == want).all().item())
    for _ in range(a.warmup):
        x.fill_(1)
        dist.all_reduce(x)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        dist.all_reduce(x)
    sync()
    dt = (time.perf_counter() - t0) / a.iters
    algbw = a.bytes / dt / 1e9
    out = {"rank": a.rank, "world": a.world, "backend": a.backend, "bytes": a.bytes,
           "iters": a.iters, "ms": round(dt * 1e3, 3), "algbw_GBps": round(algbw, 1),
           "busbw_GBps": round(algbw * 2 * (a.world - 1) / a.world, 1), "exact": ok,
           "expected": want, "got": [float(got.min()), float(got.max())]}
    if a.device == "cuda":
        out["device"] = torch.cuda.get_device_properties(dev).name
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    return 0 if ok else 2


if __name__ == "__main__":
    raise SystemExit(main())

"""Data-parallel helpers for pool workloads: one process per GPU, ``torch.distributed`` over RCCL.

The reference's ``train_distributed`` is a stub that calls ``train_single``
(GPU调度平台搭建.md:606-611). Here a pod that was allocated k GPUs by the device plugin
(``ROCR_VISIBLE_DEVICES`` = its GPUs) runs k ranks via ``torch.distributed.run``; each rank binds
``cuda:LOCAL_RANK`` and gradients are all-reduced by DDP over RCCL (backend "nccl" IS RCCL on
ROCm), which rides xGMI between MI355X peers. For the 225k-parameter FMNIST CNN the gradient
all-reduce is ~0.9 MB per step — latency-bound, so one bucket (``bucket_cap_mb=25``) is right.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_from_env(prefer_gpu: bool = True) -> DistEnv:
    """Initialise from torchrun / Kubeflow PyTorchJob env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*;
    PET_* variables set by the training operator, GPU调度平台搭建.md:623, are consumed by
    torch.distributed.run, which exports the variables read here)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    device = torch.device(f"cuda:{local}") if use_gpu else torch.device("cpu")
    backend = "nccl" if use_gpu else "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if use_gpu:
            torch.cuda.set_device(device)
        dist.init_process_group(backend, rank=rank, world_size=world)
    return DistEnv(rank, world, local, device, backend)


def wrap(model: torch.nn.Module, env: DistEnv) -> torch.nn.Module:
    model = model.to(env.device)
    if env.world > 1:
        kw = {"device_ids": [env.local_rank]} if env.device.type == "cuda" else {}
        model = torch.nn.parallel.DistributedDataParallel(model, bucket_cap_mb=25, **kw)
    return model


def sampler(dataset, env: DistEnv, shuffle: bool = True):
    """Epoch-seeded order on every rank (also for a single process): a job resumed mid-epoch can
    skip exactly the batches it already trained on."""
    return torch.utils.data.distributed.DistributedSampler(dataset, num_replicas=env.world,
                                                           rank=env.rank, shuffle=shuffle)


def broadcast_object(obj, env: DistEnv, src: int = 0):
    """Rank ``src``'s Python object on every rank (e.g. a checkpoint only rank 0 can read: ranks on
    other nodes have no shared volume, and a per-rank load would desynchronise the collectives)."""
    if env.world <= 1:
        return obj
    box = [obj if env.rank == src else None]
    dist.broadcast_object_list(box, src=src, device=env.device if env.backend == "nccl" else None)
    return box[0]


def all_reduce_mean(x: float, env: DistEnv) -> float:
    if env.world <= 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=env.device)
    dist.all_reduce(t)
    return float(t.item()) / env.world


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()

"""The reference's example workload model (GPU调度平台搭建.md:570-582, ``get_model``):
Conv(1->32,k3) -> ReLU -> MaxPool2 -> Conv(32->64,k3) -> ReLU -> MaxPool2 -> Flatten ->
Linear(1600->128) -> ReLU -> Linear(128->10); 225,034 parameters.

It is the "a pod actually got a working GPU" validation job of the platform, not a hot path
(SURVEY.md §2.4): stock PyTorch-ROCm ops (MIOpen / hipBLASLt) are the right tool here.
"""
from __future__ import annotations

import os
import struct

import torch
from torch import nn


def get_model() -> nn.Module:
    return nn.Sequential(
        nn.Conv2d(1, 32, kernel_size=3), nn.ReLU(), nn.MaxPool2d(2),
        nn.Conv2d(32, 64, kernel_size=3), nn.ReLU(), nn.MaxPool2d(2),
        nn.Flatten(),
        nn.Linear(64 * 5 * 5, 128), nn.ReLU(),
        nn.Linear(128, 10),
    )


def synthetic_fmnist(n: int, seed: int = 0) -> torch.utils.data.TensorDataset:
    """FashionMNIST-shaped data (no network): 10 class prototypes + noise, so the model can learn
    and the loss visibly drops (a real training signal, not random labels)."""
    g = torch.Generator().manual_seed(seed)
    protos = torch.rand(10, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (n,), generator=g)
    x = protos[y] + 0.35 * torch.randn(n, 1, 28, 28, generator=g)
    return torch.utils.data.TensorDataset(x.clamp_(0, 1), y)


def _read_idx(path: str) -> torch.Tensor:
    with open(path, "rb") as f:
        magic = struct.unpack(">I", f.read(4))[0]
        ndim = magic & 0xFF
        dims = struct.unpack(">" + "I" * ndim, f.read(4 * ndim))
        data = torch.frombuffer(bytearray(f.read()), dtype=torch.uint8)
    return data.reshape(dims)


def load_fmnist(data_dir: str, train: bool = True) -> torch.utils.data.TensorDataset | None:
    """Real FashionMNIST from raw idx files if they exist under ``data_dir`` (no download)."""
    prefix = "train" if train else "t10k"
    img = os.path.join(data_dir, f"{prefix}-images-idx3-ubyte")
    lab = os.path.join(data_dir, f"{prefix}-labels-idx1-ubyte")
    if not (os.path.exists(img) and os.path.exists(lab)):
        return None
    x = _read_idx(img).float().div_(255.0).unsqueeze(1)
    y = _read_idx(lab).long()
    return torch.utils.data.TensorDataset(x, y)

"""The validation workload (reference B20): model shape parity and a real 2-rank DDP run on CPU
(gloo), i.e. the distributed mode the reference left as a stub (GPU调度平台搭建.md:606-611)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import torch

from gpupool.models.fmnist import get_model, synthetic_fmnist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_model_matches_reference_architecture():
    m = get_model()
    assert sum(p.numel() for p in m.parameters()) == 225034
    x = torch.zeros(128, 1, 28, 28)
    assert m(x).shape == (128, 10)  # GPU调度平台搭建.md:570-582 shapes


def test_synthetic_data_is_learnable():
    ds = synthetic_fmnist(512)
    x, y = ds.tensors
    assert x.shape == (512, 1, 28, 28) and int(y.max()) <= 9


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_ddp_two_ranks_gloo(tmp_path):
    out = tmp_path / "out"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1",
                        f"--master-port={_free_port()}",
                        os.path.join(ROOT, "examples", "fmnist_train.py"), "--mode", "distributed",
                        "--cpu", "--synthetic", "--samples", "2048", "--steps", "24",
                        "--epochs", "5", "--output", str(out)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    done = [json.loads(x) for x in r.stdout.splitlines() if '"event": "done"' in x]
    assert done and done[0]["world"] == 2 and done[0]["steps"] == 24
    assert (out / "fashion_mnist_cnn.pth").exists()
    sd = torch.load(out / "fashion_mnist_cnn.pth", weights_only=True)
    assert "0.weight" in sd  # plain (unwrapped) state_dict, loadable by get_model()
    get_model().load_state_dict(sd)

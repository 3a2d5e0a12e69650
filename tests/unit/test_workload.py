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


def test_resume_on_two_ranks_without_a_shared_volume(tmp_path):
    """only rank 0's node holds the checkpoint (no shared volume). Attempt 1 fails at
    step 25 (checkpoint at step 20, batch 20 of epoch 0 with 2 ranks x 1024 samples / 32); on the
    restart rank 0 loads and broadcasts it, BOTH ranks resume at step 20 / batch 20 (rank 1 has
    an empty checkpoint dir), the collectives stay aligned and the job finishes at step 40."""
    port = _free_port()
    dirs = [tmp_path / "ckpt-rank0", tmp_path / "ckpt-rank1"]

    def launch(attempt: str):
        procs = []
        for rank in range(2):
            env = dict(os.environ, OMP_NUM_THREADS="2", RANK=str(rank), LOCAL_RANK="0",
                       WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       GPUPOOL_JOB_ATTEMPT=attempt)
            procs.append(subprocess.Popen(
                [sys.executable, os.path.join(ROOT, "examples", "fmnist_train.py"), "--mode",
                 "distributed", "--cpu", "--synthetic", "--samples", "2048", "--batch_size", "32",
                 "--steps", "40", "--epochs", "3", "--checkpoint_dir", str(dirs[rank]),
                 "--checkpoint_every", "10", "--fail_at_step", "25", "--output",
                 str(tmp_path / f"out{rank}")], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                stderr=subprocess.STDOUT, text=True))
        return [(p.communicate(timeout=300)[0], p.returncode) for p in procs]
    first = launch("1")
    assert all(rc == 3 for _, rc in first), first
    assert (dirs[0] / "fmnist_ckpt.pt").exists() and not (dirs[1] / "fmnist_ckpt.pt").exists()
    second = launch("2")
    assert all(rc == 0 for _, rc in second), [o[-2000:] for o, _ in second]
    out0 = [json.loads(x) for x in second[0][0].splitlines() if x.startswith("{")]
    resume = next(e for e in out0 if e["event"] == "resume")
    assert (resume["step"], resume["epoch"], resume["batch"]) == (20, 0, 20)
    done = next(e for e in out0 if e["event"] == "done")
    assert done["steps"] == 40 and done["world"] == 2

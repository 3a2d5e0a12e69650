#!/usr/bin/env python3
"""FashionMNIST CNN training job (ROCm version of the reference's train.py,
GPU调度平台搭建.md:557-636): same model, SGD lr 0.01, CrossEntropy, argparse flags
(--epochs --batch_size --lr --data_dir --mode), auto mode from PET_NNODES / WORLD_SIZE /
device count, checkpoint to --output.

Differences by design: the distributed mode is real DDP over RCCL (the reference's is a stub);
without FashionMNIST idx files (no network here) it trains on synthetic FMNIST-shaped data;
``--steps`` caps iterations for smoke runs. Run inside a pool pod: the device plugin sets
ROCR_VISIBLE_DEVICES so ``cuda:0`` is the allotted MI355X.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch import nn  # noqa: E402

from gpupool.models.fmnist import get_model, load_fmnist, synthetic_fmnist  # noqa: E402
from gpupool.parallel import ddp  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--data_dir", default="/dataset")
    ap.add_argument("--mode", default="auto", choices=["auto", "single", "distributed"])
    ap.add_argument("--output", default=os.environ.get("GPUPOOL_OUTPUT", "/tmp/fmnist_out"))
    ap.add_argument("--synthetic", action="store_true", help="force synthetic data")
    ap.add_argument("--samples", type=int, default=8192, help="synthetic dataset size")
    ap.add_argument("--steps", type=int, default=0, help="stop after N steps (0 = full epochs)")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--checkpoint_dir", default=os.environ.get("GPUPOOL_CHECKPOINT_DIR", ""),
                    help="save/resume {model, optimizer, step} here (Mi355xJob spec.checkpointDir)")
    ap.add_argument("--checkpoint_every", type=int, default=10, help="steps between checkpoints")
    ap.add_argument("--fail_at_step", type=int, default=0,
                    help="test hook: exit 3 at this step on job attempt --fail_on_attempt")
    ap.add_argument("--fail_on_attempt", default="1")
    a = ap.parse_args()

    mode = a.mode
    if mode == "auto":  # GPU调度平台搭建.md:623-630
        nnodes = int(os.environ.get("PET_NNODES", "1"))
        mode = "distributed" if nnodes > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1 else "single"
    env = ddp.init_from_env(prefer_gpu=not a.cpu) if mode == "distributed" else \
        ddp.DistEnv(0, 1, 0, torch.device("cuda:0" if torch.cuda.is_available() and not a.cpu
                                           else "cpu"), "none")
    ds = None if a.synthetic else load_fmnist(a.data_dir, train=True)
    data_kind = "fashion-mnist" if ds is not None else "synthetic"
    if ds is None:
        ds = synthetic_fmnist(a.samples)
    smp = ddp.sampler(ds, env)
    loader = torch.utils.data.DataLoader(ds, batch_size=a.batch_size, sampler=smp, drop_last=True)
    base = get_model().to(env.device)
    opt = torch.optim.SGD(base.parameters(), lr=a.lr)
    loss_fn = nn.CrossEntropyLoss()
    # Resume: rank 0 reads the checkpoint and broadcasts it, so every rank restarts at the same
    # step/epoch/batch even when only rank 0's node holds GPUPOOL_CHECKPOINT_DIR (no shared volume);
    # the weights are loaded BEFORE the DDP wrapper is built (DDP then starts from them).
    step, start_epoch, skip = 0, 0, 0
    ckpt = os.path.join(a.checkpoint_dir, "fmnist_ckpt.pt") if a.checkpoint_dir else ""
    st = None
    if ckpt and env.is_main and os.path.exists(ckpt):
        st = torch.load(ckpt, map_location="cpu", weights_only=True)
    if mode == "distributed":
        st = ddp.broadcast_object(st, env)
    if st is not None:
        base.load_state_dict(st["model"])
        opt.load_state_dict(st["opt"])
        step, start_epoch, skip = int(st["step"]), int(st["epoch"]), int(st.get("batch", 0))
        if env.is_main:
            print(json.dumps({"event": "resume", "step": step, "epoch": start_epoch,
                              "batch": skip}), flush=True)
    model = ddp.wrap(base, env)
    info = {"rank": env.rank, "world": env.world, "device": str(env.device), "mode": mode,
            "data": data_kind, "rocr_visible": os.environ.get("ROCR_VISIBLE_DEVICES", "")}
    if env.device.type == "cuda":
        p = torch.cuda.get_device_properties(env.device)
        info.update({"gpu": p.name, "arch": getattr(p, "gcnArchName", "")})
    print(json.dumps({"event": "start", **info}), flush=True)
    t0, first_loss, loss_v = time.time(), None, float("nan")

    def save_checkpoint(epoch: int, batch: int) -> None:
        if not ckpt or not env.is_main:
            return
        os.makedirs(a.checkpoint_dir, exist_ok=True)
        tmp = ckpt + ".tmp"
        torch.save({"model": base.state_dict(), "opt": opt.state_dict(), "step": step,
                    "epoch": epoch, "batch": batch}, tmp)
        os.replace(tmp, ckpt)  # atomic: a crash never leaves a torn checkpoint
    for epoch in range(start_epoch, a.epochs):
        smp.set_epoch(epoch)  # same order as before the restart: the skipped batches are exact
        model.train()
        for bi, (x, y) in enumerate(loader):
            if epoch == start_epoch and bi < skip:
                continue  # already trained on before the checkpoint (no replay)
            x, y = x.to(env.device, non_blocking=True), y.to(env.device, non_blocking=True)
            opt.zero_grad(set_to_none=True)
            loss = loss_fn(model(x), y)
            loss.backward()
            opt.step()
            step += 1
            if ckpt and step % a.checkpoint_every == 0:
                save_checkpoint(epoch, bi + 1)
            if a.fail_at_step and step == a.fail_at_step and \
                    os.environ.get("GPUPOOL_JOB_ATTEMPT", "1") == a.fail_on_attempt:
                print(json.dumps({"event": "injected_failure", "step": step}), flush=True)
                sys.exit(3)
            if step % 20 == 0 or step == 1:
                loss_v = ddp.all_reduce_mean(float(loss.item()), env)
                first_loss = loss_v if first_loss is None else first_loss
                if env.is_main:
                    print(json.dumps({"event": "step", "epoch": epoch, "step": step,
                                      "loss": round(loss_v, 4)}), flush=True)
            if a.steps and step >= a.steps:
                break
        if a.steps and step >= a.steps:
            break
    loss_v = ddp.all_reduce_mean(float(loss.item()), env)
    if env.device.type == "cuda":
        torch.cuda.synchronize()
    if env.is_main:
        os.makedirs(a.output, exist_ok=True)
        torch.save(base.state_dict(), os.path.join(a.output, "fashion_mnist_cnn.pth"))  # GPU调度平台搭建.md:603
        print(json.dumps({"event": "done", "steps": step, "first_loss": first_loss,
                          "final_loss": round(loss_v, 4), "seconds": round(time.time() - t0, 3),
                          **info}), flush=True)
    ddp.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""MNIST LeNet: single process, torch DDP, or scaletorch_amd's arena DataParallel.

Reference: examples/torch_examples/mnist/{basic_mnist,multigpu_mnist,torchrun_mnist,
fsdp_mnist}.py (torchvision MNIST download).  There is no network here, so the
data is a synthetic MNIST-shaped set (28x28 digits drawn as class-dependent
stroke patterns + noise) that a LeNet learns in a few hundred steps; point
``--data`` at a local ``.npz`` with ``x`` [N,28,28] uint8 / ``y`` [N] to use real
MNIST.  Launch modes:

  python examples/mnist/mnist_ddp.py --mode single
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/mnist/mnist_ddp.py --mode ddp
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/mnist/mnist_ddp.py --mode arena
  python examples/mnist/mnist_ddp.py --mode spawn --nproc 2 --cpu   # mp.spawn launcher
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/mnist/mnist_ddp.py --mode fsdp  # FSDP1

Reference file -> mode: basic_mnist.py -> single, multigpu_mnist.py -> spawn,
torchrun_mnist.py -> ddp, fsdp_mnist.py -> fsdp (FullyShardedDataParallel with a
size-based auto-wrap policy and a full-state-dict checkpoint of the sharded model).
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def synthetic_mnist(n: int, seed: int = 0):
    """Class c = a fixed random 28x28 stroke template (per class) + noise + random shift."""
    rng = np.random.default_rng(seed)
    templates = (rng.random((10, 28, 28)) > 0.82).astype(np.float32)
    y = rng.integers(0, 10, n)
    x = templates[y] + 0.35 * rng.standard_normal((n, 28, 28)).astype(np.float32)
    shift = rng.integers(-2, 3, (n, 2))
    for i in range(n):
        x[i] = np.roll(x[i], tuple(shift[i]), axis=(0, 1))
    return torch.from_numpy(x).unsqueeze(1), torch.from_numpy(y).long()


def load_data(path: str | None, n: int):
    if path:
        d = np.load(path, allow_pickle=False)
        x = torch.from_numpy(d["x"]).float().div(255.0).unsqueeze(1)
        return (x - 0.1307) / 0.3081, torch.from_numpy(d["y"]).long()
    return synthetic_mnist(n)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="ddp", choices=["single", "ddp", "arena", "spawn", "fsdp"])
    ap.add_argument("--save-model", default="", help="fsdp: write the full (gathered) state dict here")
    ap.add_argument("--nproc", type=int, default=2)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1.0)
    ap.add_argument("--gamma", type=float, default=0.7)
    ap.add_argument("--samples", type=int, default=4096)
    ap.add_argument("--data", default=None)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--max-steps", type=int, default=0)
    return ap.parse_args(argv)


def train(args) -> dict:
    from scaletorch_amd.dist.launch import init_dist
    from scaletorch_amd.models.attention_variants import LeNet
    from scaletorch_amd.parallel.data_parallel import DataParallel

    distributed = args.mode in ("ddp", "arena", "fsdp")
    if distributed:
        rank, local_rank, world = init_dist(backend="gloo" if args.cpu else None, use_cpu=args.cpu)
    else:
        rank, local_rank, world = 0, 0, 1
    dev = torch.device("cpu") if (args.cpu or not torch.cuda.is_available()) else torch.device("cuda", local_rank)
    torch.manual_seed(1)
    model = LeNet().to(dev)
    if args.mode == "ddp" and world > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local_rank] if dev.type == "cuda" else None)
    elif args.mode == "arena":
        model = DataParallel(model, bucket_size=1 << 20, expose_grads=True)  # flat fp32 grad arena + RCCL buckets
    elif args.mode == "fsdp":
        import functools

        from torch.distributed.fsdp import FullyShardedDataParallel as FSDP
        from torch.distributed.fsdp.wrap import size_based_auto_wrap_policy

        policy = functools.partial(size_based_auto_wrap_policy, min_num_params=20000)  # fc1 gets its own unit
        model = FSDP(model, auto_wrap_policy=policy, device_id=dev, use_orig_params=True)
    opt = torch.optim.Adadelta(model.parameters(), lr=args.lr)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=args.gamma)
    x, y = load_data(args.data, args.samples)
    n_test = len(x) // 8
    xt, yt, xtr, ytr = x[:n_test], y[:n_test], x[n_test:], y[n_test:]
    shard = torch.arange(rank, len(xtr), world)  # DistributedSampler equivalent
    steps = 0
    for epoch in range(args.epochs):
        model.train()
        perm = shard[torch.randperm(len(shard), generator=torch.Generator().manual_seed(epoch))]
        for i in range(0, len(perm) - args.batch_size + 1, args.batch_size):
            idx = perm[i: i + args.batch_size]
            xb, yb = xtr[idx].to(dev), ytr[idx].to(dev)
            opt.zero_grad()
            if args.mode == "arena":
                model.zero_grad()
            loss = F.nll_loss(model(xb), yb)
            loss.backward()
            opt.step()
            steps += 1
            if args.max_steps and steps >= args.max_steps:
                break
        sched.step()
    model.eval()
    with torch.no_grad():
        pred = model(xt.to(dev)).argmax(1).cpu()
    acc = (pred == yt).float().mean().item()
    if args.mode == "fsdp" and args.save_model:
        from torch.distributed.checkpoint.state_dict import StateDictOptions, get_model_state_dict

        sd = get_model_state_dict(model, options=StateDictOptions(full_state_dict=True, cpu_offload=dev.type == "cuda"))
        if rank == 0:
            torch.save(sd, args.save_model)
    if rank == 0:
        print(f"mnist[{args.mode}] world {world}: test accuracy {acc:.3f} after {steps} steps", flush=True)
    return {"acc": acc, "steps": steps, "world": world}


def _spawn_entry(rank, args, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(args.nproc), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    args.mode = "ddp"
    train(args)
    dist.destroy_process_group()


def main(argv=None):
    args = parse(argv)
    if args.mode == "spawn":
        import socket

        import torch.multiprocessing as mp

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        mp.spawn(_spawn_entry, args=(args, port), nprocs=args.nproc)
        return None
    return train(args)


if __name__ == "__main__":
    main()
    if dist.is_initialized():
        dist.destroy_process_group()

#!/usr/bin/env python3
"""DeviceMesh / DTensor demos (reference: examples/device_mesh/*.py:
device_mesh_api, dtensor_demo, manual_process_group, tensor_parallel_demo,
sequence_parallel_demo, fsdp_dp_demo, fsdp_tp_demo) as one script with
sub-commands; every demo asserts its own result so it doubles as a test.

  torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/device_mesh/demos.py all
  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/device_mesh/demos.py all --cpu

On MI355X one rank per GPU, RCCL over xGMI; on CPU gloo.  The 2-D meshes put
TP on the fastest-varying dimension so a TP group is a set of xGMI peers.
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402


def _mesh_2d(dev: str, world: int):
    from torch.distributed.device_mesh import init_device_mesh

    tp = 2 if world % 2 == 0 and world > 1 else 1
    return init_device_mesh(dev, (world // tp, tp), mesh_dim_names=("dp", "tp"))


def demo_mesh(dev: str) -> None:
    """init_device_mesh, named sub-meshes, their process groups and coordinates."""
    world, rank = dist.get_world_size(), dist.get_rank()
    mesh = _mesh_2d(dev, world)
    dp, tp = mesh["dp"], mesh["tp"]
    assert dp.size() * tp.size() == world
    coord = mesh.get_coordinate()
    assert coord == [rank // tp.size(), rank % tp.size()]
    t = torch.ones(1, device=dev) * rank
    dist.all_reduce(t, group=tp.get_group())
    tp_ranks = [coord[0] * tp.size() + i for i in range(tp.size())]
    assert t.item() == sum(tp_ranks)


def demo_dtensor(dev: str) -> None:
    """distribute_tensor with Shard / Replicate placements and redistribute."""
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Replicate, Shard, distribute_tensor

    world = dist.get_world_size()
    mesh = init_device_mesh(dev, (world,))
    torch.manual_seed(0)
    full = torch.randn(4 * world, 8, device=dev)
    dt = distribute_tensor(full, mesh, [Shard(0)])
    assert dt.to_local().shape == (4, 8)
    rep = dt.redistribute(mesh, [Replicate()])
    assert torch.allclose(rep.to_local(), full)
    col = dt.redistribute(mesh, [Shard(1)]) if 8 % world == 0 else dt
    assert torch.allclose(col.full_tensor(), full)


def demo_manual(dev: str) -> None:
    """The same 2-D layout built by hand with new_group (what init_device_mesh does)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    tp = 2 if world % 2 == 0 and world > 1 else 1
    my_tp = my_dp = None
    for d in range(world // tp):  # every rank must create every group, in the same order
        g = dist.new_group(list(range(d * tp, (d + 1) * tp)))
        if rank // tp == d:
            my_tp = g
    for t in range(tp):
        g = dist.new_group(list(range(t, world, tp)))
        if rank % tp == t:
            my_dp = g
    x = torch.ones(1, device=dev)
    dist.all_reduce(x, group=my_dp)
    assert x.item() == world // tp
    dist.all_reduce(x, group=my_tp)
    assert x.item() == (world // tp) * tp


class _MLP(nn.Module):
    def __init__(self, h=64, i=128):
        super().__init__()
        self.w1, self.w2 = nn.Linear(h, i, bias=False), nn.Linear(i, h, bias=False)

    def forward(self, x):
        return self.w2(torch.relu(self.w1(x)))


def demo_tp(dev: str) -> None:
    """Megatron column -> row MLP with parallelize_module, equal to the dense module."""
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor.parallel import ColwiseParallel, RowwiseParallel, parallelize_module

    world = dist.get_world_size()
    torch.manual_seed(0)
    ref = _MLP().to(dev)
    mlp = _MLP().to(dev)
    mlp.load_state_dict(ref.state_dict())
    mesh = init_device_mesh(dev, (world,))
    parallelize_module(mlp, mesh, {"w1": ColwiseParallel(), "w2": RowwiseParallel()})
    x = torch.randn(5, 64, device=dev)
    assert torch.allclose(mlp(x), ref(x), atol=1e-5)


def demo_sp(dev: str) -> None:
    """Sequence parallel: activations sharded on the sequence dim between the TP regions."""
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Shard
    from torch.distributed.tensor.parallel import ColwiseParallel, RowwiseParallel, parallelize_module

    world = dist.get_world_size()
    torch.manual_seed(0)
    ref = _MLP().to(dev)
    mlp = _MLP().to(dev)
    mlp.load_state_dict(ref.state_dict())
    mesh = init_device_mesh(dev, (world,))
    parallelize_module(mlp, mesh, {"w1": ColwiseParallel(input_layouts=Shard(1)),
                                   "w2": RowwiseParallel(output_layouts=Shard(1))})
    x = torch.randn(2, 4 * world, 64, device=dev)
    r = dist.get_rank()
    local = x[:, 4 * r: 4 * (r + 1)]
    out = mlp(local)
    assert torch.allclose(out, ref(x)[:, 4 * r: 4 * (r + 1)], atol=1e-5)


def demo_fsdp_tp(dev: str) -> None:
    """2-D: TP inside each dp group (xGMI peers), FSDP2 sharding across dp groups; trains 3 steps."""
    from torch.distributed.fsdp import fully_shard
    from torch.distributed.tensor.parallel import ColwiseParallel, RowwiseParallel, parallelize_module

    world = dist.get_world_size()
    mesh = _mesh_2d(dev, world)
    torch.manual_seed(0)
    model = nn.Sequential(_MLP(), _MLP()).to(dev)
    if mesh["tp"].size() > 1:
        for blk in model:
            parallelize_module(blk, mesh["tp"], {"w1": ColwiseParallel(), "w2": RowwiseParallel()})
    for blk in model:
        fully_shard(blk, mesh=mesh["dp"])
    fully_shard(model, mesh=mesh["dp"])
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    g = torch.Generator().manual_seed(7 + mesh.get_coordinate()[0])  # same data inside a tp group
    first = last = None
    x = torch.randn(8, 64, generator=g).to(dev)  # fixed batch: the loss must go down
    for _ in range(5):
        loss = (model(x) - x).pow(2).mean()
        loss.backward()
        opt.step()
        opt.zero_grad()
        first = loss.item() if first is None else first
        last = loss.item()
    assert last < first


DEMOS = {"mesh": demo_mesh, "dtensor": demo_dtensor, "manual": demo_manual, "tp": demo_tp, "sp": demo_sp,
         "fsdp_tp": demo_fsdp_tp}


def main(argv=None) -> list[str]:
    ap = argparse.ArgumentParser()
    ap.add_argument("demo", nargs="?", default="all", choices=["all", *DEMOS])
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args(argv)
    from scaletorch_amd.dist.launch import init_dist

    _, local_rank, _ = init_dist(backend="gloo" if args.cpu else None, use_cpu=args.cpu)
    dev = "cpu" if (args.cpu or not torch.cuda.is_available()) else "cuda"
    ran = []
    for name, fn in DEMOS.items():
        if args.demo in ("all", name):
            fn(dev)
            ran.append(name)
            if dist.get_rank() == 0:
                print(f"[device_mesh] {name}: ok", flush=True)
    return ran


if __name__ == "__main__":
    main()
    if dist.is_initialized():
        dist.destroy_process_group()

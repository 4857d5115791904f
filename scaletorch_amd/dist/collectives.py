"""Collective-communication facade over ``torch.distributed`` (RCCL on ROCm, gloo on CPU).

Covers the reference's ``scaletorch.dist`` surface (scaletorch/dist/collective_ops.py,
p2p_ops.py, object_ops.py, gather_utils.py): string reduce ops, no-ops at world
size 1, async handles.  Differences by design:

* no host<->device "comm device" round trips on the hot path: RCCL tensors stay
  on the GPU; only gloo moves CPU tensors (reference cast_data_device,
  scaletorch/dist/utils.py:544-620, copied every tensor);
* ``mean`` is a SUM followed by an in-place scale (RCCL has AVG but gloo does not);
* ``all_gather`` returns one concatenated tensor by default (one collective,
  one output buffer) and a list when ``as_list=True``;
* ``reduce_scatter`` / ``all_gather_into_tensor`` use the flat-tensor
  collectives, which RCCL implements without the per-rank list copies.
"""
from __future__ import annotations

import os
import pickle
import tempfile
from typing import Any

import torch
import torch.distributed as dist

_OPS = {
    "sum": dist.ReduceOp.SUM,
    "mean": dist.ReduceOp.SUM,
    "avg": dist.ReduceOp.SUM,
    "product": dist.ReduceOp.PRODUCT,
    "prod": dist.ReduceOp.PRODUCT,
    "min": dist.ReduceOp.MIN,
    "max": dist.ReduceOp.MAX,
    "band": dist.ReduceOp.BAND,
    "bor": dist.ReduceOp.BOR,
    "bxor": dist.ReduceOp.BXOR,
}


def reduce_op(op: str | dist.ReduceOp) -> dist.ReduceOp:
    """Map a string reduce op to ``torch.distributed.ReduceOp`` (reference: scaletorch/dist/_reduce_op.py)."""
    if isinstance(op, dist.ReduceOp) or not isinstance(op, str):
        return op
    try:
        return _OPS[op.lower()]
    except KeyError:
        raise ValueError(f"unsupported reduce op {op!r}; expected one of {sorted(_OPS)}") from None


class _Single:
    """Sentinel for a size-1 process-group family (no communicator is created)."""

    def __repr__(self) -> str:
        return "SINGLE"


SINGLE = _Single()


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_rank(group=None) -> int:
    if group is SINGLE:
        return 0
    return dist.get_rank(group) if is_distributed() else 0


def get_world_size(group=None) -> int:
    if group is SINGLE:
        return 1
    return dist.get_world_size(group) if is_distributed() else 1


def global_rank_of(group, group_rank: int) -> int:
    """Translate a rank inside ``group`` to a global rank."""
    if group is SINGLE or group is None or not is_distributed():
        return get_rank() if group is SINGLE else group_rank
    return dist.get_global_rank(group, group_rank)


def get_local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def get_local_world_size() -> int:
    return int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))


def is_main_process(group=None) -> bool:
    return get_rank(group) == 0


def barrier(group=None) -> None:
    if group is SINGLE:
        return
    if is_distributed():
        if dist.get_backend(group) == "nccl" and torch.cuda.is_available():
            dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=group)


def new_group(ranks=None, backend=None, **kw):
    if not is_distributed():
        return None
    return dist.new_group(ranks=ranks, backend=backend, **kw)


def destroy_group(group) -> None:
    if group is not None and group is not SINGLE and is_distributed():
        dist.destroy_process_group(group)


def _finish_mean(t: torch.Tensor, op: str | Any, group) -> None:
    if isinstance(op, str) and op.lower() in ("mean", "avg"):
        t.div_(get_world_size(group))


def all_reduce(tensor: torch.Tensor, op: str = "sum", group=None, async_op: bool = False):
    """In-place all-reduce; returns the work handle when ``async_op``."""
    if get_world_size(group) == 1:
        return None
    work = dist.all_reduce(tensor, op=reduce_op(op), group=group, async_op=async_op)
    if async_op:
        if isinstance(op, str) and op.lower() in ("mean", "avg"):
            raise ValueError("async mean all_reduce: pre-divide and use op='sum'")
        return work
    _finish_mean(tensor, op, group)
    return None


def all_gather(tensor: torch.Tensor, group=None, dim: int = 0, as_list: bool = False,
               async_op: bool = False):
    """Gather ``tensor`` from every rank, concatenated along ``dim`` (or a list)."""
    ws = get_world_size(group)
    if ws == 1:
        return [tensor] if as_list else tensor
    t = tensor.contiguous()
    out = torch.empty((ws * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    work = dist.all_gather_into_tensor(out, t, group=group, async_op=async_op)
    if async_op:
        return out, work
    parts = list(out.chunk(ws, dim=0))
    if as_list:
        return parts
    return out if dim == 0 else torch.cat(parts, dim=dim)


def reduce_scatter(tensor: torch.Tensor, op: str = "sum", group=None, dim: int = 0,
                   async_op: bool = False):
    """Reduce across ranks and keep this rank's 1/ws slice along ``dim``."""
    ws = get_world_size(group)
    if ws == 1:
        return tensor
    t = tensor if dim == 0 else tensor.transpose(0, dim)
    t = t.contiguous()
    if t.shape[0] % ws:
        raise ValueError(f"reduce_scatter: dim {dim} size {t.shape[0]} not divisible by world {ws}")
    out = torch.empty((t.shape[0] // ws,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    work = dist.reduce_scatter_tensor(out, t, op=reduce_op(op), group=group, async_op=async_op)
    if async_op:
        return out, work
    _finish_mean(out, op, group)
    return out if dim == 0 else out.transpose(0, dim).contiguous()


def broadcast(tensor: torch.Tensor, src: int = 0, group=None, async_op: bool = False):
    if get_world_size(group) == 1:
        return tensor
    work = dist.broadcast(tensor, src=src, group=group, async_op=async_op)
    return work if async_op else tensor


def reduce(tensor: torch.Tensor, dst: int = 0, op: str = "sum", group=None):
    if get_world_size(group) == 1:
        return tensor
    dist.reduce(tensor, dst=dst, op=reduce_op(op), group=group)
    if get_rank() == dst:
        _finish_mean(tensor, op, group)
    return tensor


def scatter(data: list[torch.Tensor] | None, out: torch.Tensor, src: int = 0, group=None):
    if get_world_size(group) == 1:
        if data:
            out.copy_(data[0])
        return out
    dist.scatter(out, scatter_list=data if get_rank() == src else None, src=src, group=group)
    return out


def gather(tensor: torch.Tensor, dst: int = 0, group=None) -> list[torch.Tensor] | None:
    ws = get_world_size(group)
    if ws == 1:
        return [tensor]
    out = [torch.empty_like(tensor) for _ in range(ws)] if get_rank() == dst else None
    dist.gather(tensor, gather_list=out, dst=dst, group=group)
    return out


def all_to_all(tensor: torch.Tensor, group=None, output_split_sizes=None, input_split_sizes=None,
               async_op: bool = False):
    """Variable-split all-to-all of dim 0 (RCCL all_to_all_single)."""
    if get_world_size(group) == 1:
        return (tensor, None) if async_op else tensor
    if output_split_sizes is None:
        out = torch.empty_like(tensor)
    else:
        out = tensor.new_empty((sum(output_split_sizes),) + tuple(tensor.shape[1:]))
    work = dist.all_to_all_single(out, tensor.contiguous(), output_split_sizes=output_split_sizes,
                                  input_split_sizes=input_split_sizes, group=group, async_op=async_op)
    return (out, work) if async_op else out


# ------------------------------------------------------------------ p2p
def isend(tensor: torch.Tensor, dst: int, group=None, tag: int = 0):
    return dist.isend(tensor, dst=dst, group=group, tag=tag)


def irecv(tensor: torch.Tensor, src: int, group=None, tag: int = 0):
    return dist.irecv(tensor, src=src, group=group, tag=tag)


P2POp = dist.P2POp


def batch_isend_irecv(ops: list) -> list:
    if not ops:
        return []
    return dist.batch_isend_irecv(ops)


# ------------------------------------------------------------------ objects
def broadcast_object_list(objs: list, src: int = 0, group=None) -> list:
    if get_world_size(group) > 1:
        dist.broadcast_object_list(objs, src=src, group=group)
    return objs


def all_gather_object(obj: Any, group=None) -> list:
    ws = get_world_size(group)
    if ws == 1:
        return [obj]
    out: list = [None] * ws
    dist.all_gather_object(out, obj, group=group)
    return out


def gather_object(obj: Any, dst: int = 0, group=None) -> list | None:
    ws = get_world_size(group)
    if ws == 1:
        return [obj]
    out = [None] * ws if get_rank() == dst else None
    dist.gather_object(obj, out, dst=dst, group=group)
    return out


def collect_results(part: list, size: int, mode: str = "device", tmpdir: str | None = None) -> list | None:
    """Gather per-rank result lists on rank 0, interleaved like a DistributedSampler
    split and truncated to ``size`` (reference: scaletorch/dist/gather_utils.py:24-211).
    ``mode='cpu'`` goes through a shared temp dir instead of the communicator."""
    ws, rank = get_world_size(), get_rank()
    if ws == 1:
        return part[:size]
    if mode == "cpu":
        d = [tmpdir or (tempfile.mkdtemp() if rank == 0 else None)]
        broadcast_object_list(d, 0)
        path = os.path.join(d[0], f"part_{rank}.pkl")
        with open(path, "wb") as f:
            pickle.dump(part, f)
        barrier()
        if rank != 0:
            return None
        parts = []
        for r in range(ws):
            with open(os.path.join(d[0], f"part_{r}.pkl"), "rb") as f:  # our own files
                parts.append(pickle.load(f))
    else:
        parts = all_gather_object(part)
        if rank != 0:
            return None
    out = []
    for items in zip(*parts):
        out.extend(items)
    longest = max(len(p) for p in parts)
    for p in parts:
        if len(p) == longest and len(p) > len(parts[-1]):
            out.append(p[-1])
    return out[:size]


def collect_results_cpu(result_part: list, size: int, tmpdir: str | None = None) -> list | None:
    """Reference name (scaletorch/dist/gather_utils.py:74): collection through a shared directory."""
    return collect_results(result_part, size, mode="cpu", tmpdir=tmpdir)


def collect_results_gpu(result_part: list, size: int) -> list | None:
    """Reference name (scaletorch/dist/gather_utils.py:181): collection over the communicator."""
    return collect_results(result_part, size, mode="device")


def _coalesced_buckets(tensors: list[torch.Tensor], bucket_size_mb: int) -> list[list[torch.Tensor]]:
    """Group by (dtype, device) -- a flat buffer has one of each -- then cut each group
    into buckets of at most ``bucket_size_mb`` (<= 0: one bucket per group).  A tensor
    larger than the limit gets a bucket of its own."""
    groups: dict = {}
    for t in tensors:
        groups.setdefault((t.dtype, t.device), []).append(t)
    limit = bucket_size_mb * 1024 * 1024 if bucket_size_mb > 0 else None
    out = []
    for group in groups.values():
        cur, cur_bytes = [], 0
        for t in group:
            nb = t.numel() * t.element_size()
            if limit is not None and cur and cur_bytes + nb > limit:
                out.append(cur)
                cur, cur_bytes = [], 0
            cur.append(t)
            cur_bytes += nb
        if cur:
            out.append(cur)
    return out


def _all_reduce_coalesced(tensors: list[torch.Tensor], bucket_size_mb: int = -1, op: str = "sum",
                          group=None) -> None:
    """All-reduce a list of tensors in place with one collective per flat bucket
    (reference: scaletorch/dist/collective_ops.py:868-907).  Each bucket is packed into
    one contiguous buffer, so RCCL sees a few large messages instead of many small
    ones -- on xGMI the per-call latency, not the bytes, dominates small tensors."""
    if not isinstance(tensors, list):
        raise TypeError(f"tensors must be a list, got {type(tensors)}")
    for i, t in enumerate(tensors):
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"item {i} is not a tensor: {type(t)}")
    if get_world_size(group) == 1:
        return
    for bucket in _coalesced_buckets(tensors, bucket_size_mb):
        flat = torch.cat([t.reshape(-1) for t in bucket])
        all_reduce(flat, op=op, group=group)
        off = 0
        for t in bucket:
            n = t.numel()
            t.copy_(flat[off: off + n].view_as(t))
            off += n


def all_reduce_params(params, coalesce: bool = True, bucket_size_mb: int = -1, op: str = "sum",
                      group=None) -> None:
    """All-reduce parameters or buffers in place (reference: collective_ops.py:910-960),
    coalesced into flat buckets by default."""
    import types

    if not isinstance(params, (list, types.GeneratorType)):
        raise TypeError(f"params must be a list or generator, got {type(params)}")
    if get_world_size(group) == 1:
        return
    data = [p.data if isinstance(p, torch.nn.Parameter) else p for p in params]
    if coalesce:
        _all_reduce_coalesced(data, bucket_size_mb, op=op, group=group)
    else:
        for t in data:
            all_reduce(t, op=op, group=group)


def all_reduce_dict(data: dict[str, torch.Tensor], op: str = "sum", group=None) -> dict[str, torch.Tensor]:
    """All-reduce a dict of tensors with ONE flat collective (reference: collective_ops.py:800-865)."""
    if get_world_size(group) == 1 or not data:
        return data
    keys = sorted(data)
    flat = torch.cat([data[k].reshape(-1).float() for k in keys])
    all_reduce(flat, op=op, group=group)
    out, off = {}, 0
    for k in keys:
        n = data[k].numel()
        out[k] = flat[off: off + n].view_as(data[k]).to(data[k].dtype)
        off += n
    return out


def sync_random_seed(seed: int | None = None, device: str | torch.device = "cpu", group=None) -> int:
    """Rank 0 picks a seed, every rank returns the same value."""
    import numpy as np

    if seed is None:
        seed = int(np.random.randint(2**31))
    if get_world_size(group) == 1:
        return seed
    t = torch.tensor([seed], dtype=torch.int64, device=device)
    broadcast(t, src=0, group=group)
    return int(t.item())

"""MFU, parameter counts, seeding, readable numbers, rank-serialised printing.

Reference: scaletorch/utils/misc.py:51-249.
"""
from __future__ import annotations

import fcntl
import os
import random

import numpy as np
import torch

from ..dist import collectives as C
from .device import get_theoretical_flops


def set_all_seed(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def to_readable_format(num: float, precision: int = 2) -> str:
    num = float(num)
    for unit, div in (("T", 1e12), ("B", 1e9), ("M", 1e6), ("K", 1e3)):
        if abs(num) >= div:
            return f"{num / div:.{precision}f}{unit}"
    return f"{num:.{precision}f}"


def flops_per_token(num_params: int, num_layers: int, num_heads: int, head_dim: int, seq_len: int,
                    causal: bool = False) -> float:
    """Training FLOPs/token = 6N + 12 L H d S (reference misc.py:136-174).

    ``causal=True`` halves the attention term (the work a causal kernel does);
    the default matches the reference's MFU definition for comparability.
    """
    attn = 12 * num_layers * num_heads * head_dim * seq_len
    return 6 * num_params + (attn / 2 if causal else attn)


def get_mfu(tokens_per_second_per_gpu: float, num_params: int, model_config, seq_len: int | None = None,
            theoretical_flops: float | None = None) -> float:
    if tokens_per_second_per_gpu <= 0 or num_params <= 0:
        return 0.0
    peak = theoretical_flops or get_theoretical_flops()
    L = getattr(model_config, "num_hidden_layers", 1)
    H = getattr(model_config, "num_attention_heads", 1)
    d = getattr(model_config, "head_dim", None) or getattr(model_config, "hidden_size", 1) // H
    S = seq_len or getattr(model_config, "max_position_embeddings", 2048)
    return tokens_per_second_per_gpu * flops_per_token(num_params, L, H, d, S) / peak * 100


def get_num_params(model: torch.nn.Module, pp_group=None, tp_size: int = 1) -> int:
    """Full-model parameter count from a TP/PP shard (TP-sharded params x tp, summed over PP)."""
    seen, local = set(), 0
    for p in model.parameters():
        if id(p) in seen:
            continue
        seen.add(id(p))
        n = p.numel()
        if getattr(p, "_st_tp_sharded", False) or getattr(p, "_st_expert", False):
            n *= tp_size
        local += n
    if pp_group is not None and C.get_world_size(pp_group) > 1:
        t = torch.tensor([local], dtype=torch.float64,
                         device="cuda" if torch.cuda.is_available() and C.is_distributed()
                         and torch.distributed.get_backend(pp_group) == "nccl" else "cpu")
        C.all_reduce(t, group=pp_group)
        local = int(t.item())
    return local


def assert_no_meta_tensors(model: torch.nn.Module) -> None:
    bad = [n for n, p in list(model.named_parameters()) + list(model.named_buffers()) if p.is_meta]
    if bad:
        raise RuntimeError(f"meta tensors left after materialisation: {bad[:5]}")


def rank_print(*args, is_print_rank: bool = True, **kw) -> None:
    """Print serialised across local processes with a file lock (reference misc.py:51-85)."""
    if not is_print_rank:
        return
    path = os.environ.get("SCALETORCH_PRINT_LOCK", "/tmp/scaletorch_print.lock")
    try:
        with open(path, "a") as fh:
            fcntl.flock(fh, fcntl.LOCK_EX)
            try:
                print(*args, flush=True, **kw)
            finally:
                fcntl.flock(fh, fcntl.LOCK_UN)
    except OSError:
        print(*args, flush=True, **kw)


def average_loss_across_dp_cp_ranks(loss: torch.Tensor, group) -> torch.Tensor:
    if C.get_world_size(group) > 1:
        C.all_reduce(loss, op="mean", group=group)
    return loss


def pipeline_bubble_fraction(pp: int, micro_batches: int, virtual_stages: int = 1) -> float:
    """Idle share of a 1F1B / AFAB pipeline step, (P-1) / (V*M + P-1) (interleaved 1F1B
    with V model chunks per rank shrinks it V-fold); 0 without pipeline parallelism."""
    if pp <= 1:
        return 0.0
    return (pp - 1) / (virtual_stages * micro_batches + pp - 1)


def comm_per_step(before: dict, after: dict, steps: int) -> dict:
    """Per-step calls / bytes of every communication op between two
    ``scaletorch_amd.dist.trace.stats()`` snapshots."""
    out = {}
    for op, v in after.items():
        b = before.get(op, {"calls": 0, "bytes": 0})
        calls, nbytes = v["calls"] - b["calls"], v["bytes"] - b["bytes"]
        if calls:
            out[op] = {"calls": calls / max(1, steps), "bytes": nbytes / max(1, steps)}
    return out

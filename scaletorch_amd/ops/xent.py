"""(Vocab-parallel) softmax cross-entropy (csrc/xent.hip).

Reference: ``F.cross_entropy(logits.view(-1, V), targets)`` after gathering the
full vocabulary across TP ranks (scaletorch/trainer/train_step.py:89-103,
scaletorch/parallel/tensor_parallel/tensor_parallel.py:247-248: a [b, S, V]
all-gather, 500 MiB per step for Llama-3).  Here each TP rank keeps its
[N, V/tp] logit shard; only two length-N fp32 vectors cross the TP group
(the per-rank log-sum-exp, all-gathered, and the target logit, all-reduced).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import _lib


def _combine(lse_local: torch.Tensor, tlogit: torch.Tensor, group):
    if group is None or dist.get_world_size(group) == 1:
        return lse_local, tlogit
    ws = dist.get_world_size(group)
    parts = [torch.empty_like(lse_local) for _ in range(ws)]
    dist.all_gather(parts, lse_local.contiguous(), group=group)
    lse = torch.logsumexp(torch.stack(parts, 0), dim=0)
    dist.all_reduce(tlogit, group=group)
    return lse, tlogit


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, vocab_start, group, ignore_index):
        valid = target != ignore_index
        tgt = torch.where(valid, target, torch.zeros_like(target)).contiguous()
        if _lib.use_native(logits) and logits.dtype == torch.bfloat16 and logits.shape[-1] % 8 == 0:
            lse_l, tl = _lib.ops().xent_fwd(logits, tgt, vocab_start)
            native = True
        else:
            lf = logits.float()
            lse_l = torch.logsumexp(lf, dim=-1)
            loc = tgt - vocab_start
            inr = (loc >= 0) & (loc < logits.shape[-1])
            tl = torch.where(inr, lf.gather(1, loc.clamp(0, logits.shape[-1] - 1)[:, None])[:, 0],
                             torch.zeros_like(lse_l))
            native = False
        lse, tl = _combine(lse_l, tl, group)
        n_valid = valid.sum().clamp(min=1)
        loss_rows = torch.where(valid, lse - tl, torch.zeros_like(lse))
        ctx.save_for_backward(logits, tgt, lse, valid, n_valid)
        ctx.vocab_start, ctx.native = vocab_start, native
        return loss_rows.sum() / n_valid

    @staticmethod
    def backward(ctx, g):
        logits, tgt, lse, valid, n_valid = ctx.saved_tensors
        dloss = torch.where(valid, (g / n_valid).expand_as(lse), torch.zeros_like(lse)).float().contiguous()
        if ctx.native:
            dlogits = torch.empty_like(logits)
            _lib.ops().xent_bwd_(logits, tgt, ctx.vocab_start, lse, dloss, dlogits)
        else:
            p = torch.exp(logits.float() - lse[:, None])
            loc = tgt - ctx.vocab_start
            inr = (loc >= 0) & (loc < logits.shape[-1])
            onehot = torch.zeros_like(p)
            rows = torch.nonzero(inr)[:, 0]
            onehot[rows, loc[rows]] = 1.0
            dlogits = ((p - onehot) * dloss[:, None]).to(logits.dtype)
        return dlogits, None, None, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, vocab_start: int = 0, group=None,
                  ignore_index: int = -100) -> torch.Tensor:
    """Mean CE over non-ignored rows.  ``logits`` [..., V_local], ``target`` [...] (global ids)."""
    l2 = logits.reshape(-1, logits.shape[-1])
    t = target.reshape(-1)
    if group is None and not _lib.use_native(l2):
        return F.cross_entropy(l2.float(), t, ignore_index=ignore_index)
    return _XentFn.apply(l2, t, vocab_start, group, ignore_index)

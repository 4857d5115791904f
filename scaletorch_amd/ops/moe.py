"""MoE routing ops: fused softmax/top-k router, stable expert permutation,
row gather and weighted combine (csrc/moe.hip), each with a PyTorch reference
path used on CPU and by the numerics tests.

Reference: scaletorch/models/model_qwen3_moe.py:30-171 (softmax + topk +
renorm, then per-expert ``nonzero`` gathers and an ``index_add`` combine).
Entries are (token, slot) pairs i = t*k + s; the permutation sorts them by
expert, ties in entry order, so the native and reference paths agree exactly.
"""
from __future__ import annotations

from typing import NamedTuple

import torch

from . import _lib


class Permutation(NamedTuple):
    pos: torch.Tensor           # [T*k] row of entry i in the sorted buffer
    sorted_entry: torch.Tensor  # [T*k] entry at sorted row p
    counts: torch.Tensor        # [E] rows per expert
    k: int


# ---------------------------------------------------------------- router
def _router_ref(logits: torch.Tensor, k: int, renorm: bool):
    probs = torch.softmax(logits, dim=-1)
    topw, topi = torch.topk(probs, k, dim=-1)
    if renorm:
        topw = topw / topw.sum(-1, keepdim=True)
    return probs, topw, topi.to(torch.int32)


class _RouterFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, k, renorm):
        probs, topw, topi = _lib.ops().moe_topk_softmax(logits.contiguous(), k, renorm)
        ctx.save_for_backward(probs, topw, topi)
        ctx.renorm = renorm
        ctx.mark_non_differentiable(topi)
        return probs, topw, topi

    @staticmethod
    def backward(ctx, dprobs, dtopw, _dtopi):
        probs, topw, topi = ctx.saved_tensors
        ti = topi.long()
        g = dprobs.clone() if dprobs is not None else torch.zeros_like(probs)
        if dtopw is not None:
            if ctx.renorm:  # topw = p_sel / S
                S = probs.gather(1, ti).sum(-1, keepdim=True)
                dsel = (dtopw - (dtopw * topw).sum(-1, keepdim=True)) / S
            else:
                dsel = dtopw
            g.scatter_add_(1, ti, dsel)
        dlogits = probs * (g - (g * probs).sum(-1, keepdim=True))
        return dlogits, None, None


def router_topk(logits: torch.Tensor, k: int, renorm: bool):
    """fp32 logits [T, E] -> (probs [T, E], topw [T, k] fp32, topi [T, k] int32)."""
    logits = logits.float()
    if _lib.use_native(logits) and logits.shape[1] <= 512 and k <= 8:
        return _RouterFn.apply(logits, k, renorm)
    return _router_ref(logits, k, renorm)


# ---------------------------------------------------------------- permutation
def permutation(topi: torch.Tensor, num_experts: int) -> Permutation:
    """Stable sort of the T*k (token, slot) entries by expert."""
    k = topi.shape[-1]
    ids = topi.reshape(-1)
    if _lib.use_native(ids):
        pos, sorted_entry, counts, _ = _lib.ops().moe_permute(ids.to(torch.int32).contiguous(), num_experts)
        return Permutation(pos, sorted_entry, counts, k)
    order = torch.argsort(ids.long(), stable=True)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(order.numel(), device=order.device)
    counts = torch.bincount(ids.long(), minlength=num_experts)
    return Permutation(pos.to(torch.int32), order.to(torch.int32), counts.to(torch.int32), k)


class _GatherFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, perm_pos, perm_sorted, k):
        ctx.save_for_backward(perm_pos)
        ctx.k = k
        return _lib.ops().moe_gather_rows(x.contiguous(), perm_sorted, k)

    @staticmethod
    def backward(ctx, dxs):
        (pos,) = ctx.saved_tensors
        return _lib.ops().moe_combine(dxs.contiguous(), None, pos, ctx.k), None, None, None


def gather_rows(x2d: torch.Tensor, perm: Permutation) -> torch.Tensor:
    """Token rows [T, h] -> expert-sorted rows [T*k, h]."""
    if _lib.use_native(x2d) and x2d.dtype == torch.bfloat16 and x2d.shape[1] % 8 == 0:
        return _GatherFn.apply(x2d, perm.pos, perm.sorted_entry, perm.k)
    return x2d.index_select(0, (perm.sorted_entry.long() // perm.k))


class _CombineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, w, pos, sorted_entry, k):
        ctx.save_for_backward(y, w, pos, sorted_entry)
        ctx.k = k
        return _lib.ops().moe_combine(y.contiguous(), w.contiguous(), pos, k)

    @staticmethod
    def backward(ctx, dout):
        y, w, pos, sorted_entry = ctx.saved_tensors
        dy, dw = _lib.ops().moe_combine_bwd(dout.contiguous(), y, w, pos, sorted_entry, ctx.k,
                                            ctx.needs_input_grad[1])
        return dy, (dw if ctx.needs_input_grad[1] else None), None, None, None


def combine(y: torch.Tensor, topw: torch.Tensor, perm: Permutation) -> torch.Tensor:
    """Expert-sorted outputs [T*k, h] -> tokens [T, h]: out[t] = sum_s w[t, s] y[pos[t, s]]."""
    k = perm.k
    if _lib.use_native(y) and y.dtype == torch.bfloat16 and y.shape[1] % 8 == 0:
        return _CombineFn.apply(y, topw.float(), perm.pos, perm.sorted_entry, k)
    T = y.shape[0] // k
    yg = y.index_select(0, perm.pos.long()).view(T, k, -1)
    return (yg.float() * topw.float().unsqueeze(-1)).sum(1).to(y.dtype)

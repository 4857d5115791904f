"""Embedding lookup whose weight gradient is scattered straight into the fp32
``main_grad`` arena (one index_add over the N looked-up rows) instead of
materialising a dense [V, h] bf16 gradient (reference: F.embedding in
scaletorch/models/llama.py:382-420 / tensor_parallel.py:479-507)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops.grad import _grad_ready, take_fresh


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight):
        ctx.save_for_backward(ids)
        ctx.weight = weight
        return F.embedding(ids, weight)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        w = ctx.weight
        mg = w.main_grad
        if take_fresh(w):
            mg.zero_()
        mg.index_add_(0, ids.reshape(-1), dy.reshape(-1, dy.shape[-1]).to(mg.dtype))
        _grad_ready(w)
        return None, None


def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    if getattr(weight, "main_grad", None) is not None and torch.is_grad_enabled():
        return _EmbeddingFn.apply(ids, weight)
    return F.embedding(ids, weight)

"""Embedding lookup whose weight gradient is scattered straight into the fp32
``main_grad`` arena instead of materialising a dense [V, h] bf16 gradient
(reference: F.embedding in scaletorch/models/llama.py:382-420 /
tensor_parallel.py:479-507, whose backward sums with atomics).

On GPU the scatter is deterministic (csrc/embedding.hip): token ids are sorted
stably on device and one workgroup per distinct id sums its rows in token order,
so the step is bitwise reproducible run to run; runs longer than 64 tokens (pad/EOS
ids) are split over several workgroups and their pieces reduced in a fixed order.
``grad_ids`` (optional) are the ids the backward scatters to: -1 marks a token
whose row gets no gradient (TP: an id owned by another vocab shard), so the
masked tokens never form one giant run of a placeholder id.
CPU: ``index_add_`` (sequential)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops.grad import _grad_ready, take_fresh


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, grad_ids):
        ctx.save_for_backward(ids if grad_ids is None else grad_ids)
        ctx.weight = weight
        return F.embedding(ids, weight)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        w = ctx.weight
        mg = w.main_grad
        if take_fresh(w):
            mg.zero_()
        flat = ids.reshape(-1)
        rows = dy.reshape(-1, dy.shape[-1])
        from ..ops import _lib

        if (_lib.use_native(rows) and rows.dtype == torch.bfloat16 and mg.dtype == torch.float32
                and rows.shape[-1] % 4 == 0):
            sorted_ids, order = torch.sort(flat.to(torch.int64), stable=True)
            _lib.ops().embedding_bwd_(mg.view(mg.shape[0], -1), rows.contiguous(), sorted_ids.contiguous(),
                                      order.contiguous())
        else:
            keep = flat >= 0
            mg.index_add_(0, flat[keep], rows[keep].to(mg.dtype))
        _grad_ready(w)
        return None, None, None


def embedding(ids: torch.Tensor, weight: torch.Tensor, grad_ids: torch.Tensor | None = None) -> torch.Tensor:
    if getattr(weight, "main_grad", None) is not None and torch.is_grad_enabled():
        return _EmbeddingFn.apply(ids, weight, grad_ids)
    return F.embedding(ids, weight)

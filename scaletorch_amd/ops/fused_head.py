"""Fused, chunked LM head + (vocab-parallel) cross-entropy.

Reference: scaletorch/trainer/train_step.py:89-103 computes ``logits = model(x)``
([b, S, V] after the TP all-gather of scaletorch/parallel/tensor_parallel/
tensor_parallel.py:247-248) and then ``F.cross_entropy`` on it.  Here the
[N, V/tp] logits never outlive one chunk of tokens, and the whole backward of
the head is produced in the forward pass while each chunk is resident:

    for each chunk c of C tokens:
        Z     = X_c W^T                     hipBLASLt, bf16
        lse,t = xent_fwd(Z)                 csrc/xent.hip; TP: lse all-gathered, t all-reduced
        Z    <- (softmax(Z) - onehot) / n   xent_bwd, IN PLACE (Z becomes dZ)
        dX_c  = dZ W                        TN GEMM on the side-stream W^T copy (ops/grad.py)
        G    += dZ^T X_c                    fp32 (csrc/wgrad_gemm.hip or hipBLASLt)
    backward(g):  dX *= g;  main_grad(W) += g * G

What stays alive from the forward to the backward is dX [N, h] bf16 and G
[V/tp, h] fp32 instead of the logits and their gradient (2 x N x V/tp bf16): for
Llama-3-8B at micro-batch 4 x 4096 that is 2.2 GB instead of 8.4 GB, and the
chunk itself is C x V/tp bf16 (1 GB at the default C = 4096).  The gradient is
exact for any upstream scale ``g`` (G is scaled in the backward, not guessed in
the forward).  Tensor parallelism: the caller hands in X already replicated
(``CopyToTensorParallelRegion``: dX all-reduced in backward) or gathered along
the sequence (``AllGatherFromSequenceParallelRegion``: dX reduce-scattered).
"""
from __future__ import annotations

import os

import torch

from . import _lib
from .grad import _grad_ready, dgrad, prepare_dgrad_weight, take_fresh, wgrad_into
from .xent import _combine


def default_chunk() -> int:
    return int(os.environ.get("ST_LM_HEAD_CHUNK", "4096"))


def _chunk_stats(z: torch.Tensor, tgt: torch.Tensor, vocab_start: int, native: bool):
    """Per-row (local log-sum-exp, target logit or 0 when the target is not in this shard)."""
    if native:
        return _lib.ops().xent_fwd(z, tgt, vocab_start)
    zf = z.float()
    lse = torch.logsumexp(zf, dim=-1)
    loc = tgt - vocab_start
    inr = (loc >= 0) & (loc < z.shape[-1])
    tl = torch.where(inr, zf.gather(1, loc.clamp(0, z.shape[-1] - 1)[:, None])[:, 0], torch.zeros_like(lse))
    return lse, tl


def _chunk_grad_(z: torch.Tensor, tgt: torch.Tensor, vocab_start: int, lse: torch.Tensor, dloss: torch.Tensor,
                 native: bool) -> torch.Tensor:
    """z <- (softmax(z) - onehot(target)) * dloss, in place (row-wise global lse)."""
    if native:
        _lib.ops().xent_bwd_(z, tgt, vocab_start, lse, dloss, z)
        return z
    p = torch.exp(z.float() - lse[:, None])
    loc = tgt - vocab_start
    rows = torch.nonzero((loc >= 0) & (loc < z.shape[-1]))[:, 0]
    p[rows, loc[rows]] -= 1.0
    z.copy_(p * dloss[:, None])
    return z


def _is_native(x: torch.Tensor, weight: torch.Tensor) -> bool:
    return _lib.use_native(x) and x.dtype == torch.bfloat16 and weight.shape[0] % 8 == 0


def _loss_only(x, weight, tgt, valid, vocab_start, group, chunk) -> torch.Tensor:
    native = _is_native(x, weight)
    total = torch.zeros((), dtype=torch.float32, device=x.device)
    for s in range(0, x.shape[0], chunk):
        e = min(x.shape[0], s + chunk)
        z = torch.nn.functional.linear(x[s:e], weight)
        lse_l, tl = _chunk_stats(z, tgt[s:e], vocab_start, native)
        lse, tl = _combine(lse_l, tl, group)
        total += torch.where(valid[s:e], lse - tl, torch.zeros_like(lse)).sum()
    return total / valid.sum().clamp(min=1)


# Set on device when a direct-accumulation head (``grad_scale``) received an upstream
# gradient other than the promised one; Trainer.health_check raises on it.
_SCALE_MISMATCH: dict = {}


def check_grad_scale() -> None:
    """Raise if any direct-accumulation fused head saw an unexpected upstream gradient
    (one host sync; call at logging steps)."""
    for flag in _SCALE_MISMATCH.values():
        if bool(flag.item()):
            raise RuntimeError("fused LM head: the upstream gradient differed from its grad_scale, so the "
                               "weight gradient written during the forward is wrong; drop grad_scale")


class _FusedHeadCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, tgt, valid, vocab_start, group, chunk, grad_scale):
        N = x.shape[0]
        native = _is_native(x, weight)
        n_valid = valid.sum().clamp(min=1)
        inv = 1.0 / n_valid.float()
        prepare_dgrad_weight(weight)  # W^T for the TN data-gradient GEMM (no-op off-arena)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        mg = getattr(weight, "main_grad", None)
        # direct mode: the caller promises the upstream gradient (e.g. 1 / grad-accumulation
        # steps), so dW goes straight into the fp32 main_grad arena chunk by chunk -- no
        # [V/tp, h] fp32 buffer and no scaling pass in the backward
        direct = grad_scale is not None and mg is not None and ctx.needs_input_grad[1] and mg.dtype == torch.float32
        if direct:
            inv = inv * float(grad_scale)
            G = mg.view(weight.shape[0], -1)
            first_beta = 0 if take_fresh(weight) else 1
        else:
            G = (torch.empty(weight.shape, dtype=torch.float32, device=x.device)
                 if ctx.needs_input_grad[1] else None)
            first_beta = 0
        total = torch.zeros((), dtype=torch.float32, device=x.device)
        for i, s in enumerate(range(0, N, chunk)):
            e = min(N, s + chunk)
            xc, tc, vc = x[s:e], tgt[s:e], valid[s:e]
            z = torch.nn.functional.linear(xc, weight)
            lse_l, tl = _chunk_stats(z, tc, vocab_start, native)
            lse, tl = _combine(lse_l, tl, group)
            total += torch.where(vc, lse - tl, torch.zeros_like(lse)).sum()
            dloss = torch.where(vc, inv, torch.zeros_like(inv)).float().contiguous()
            dz = _chunk_grad_(z, tc, vocab_start, lse, dloss, native)
            if dx is not None:
                dx[s:e] = dgrad(dz, weight)
            if G is not None:
                wgrad_into(G, dz, xc, first_beta if i == 0 else 1)
            del z, dz
        ctx.save_for_backward(dx, None if direct else G)
        ctx.weight, ctx.direct, ctx.grad_scale = weight, direct, grad_scale
        return total / n_valid

    @staticmethod
    def backward(ctx, g):
        dx, G = ctx.saved_tensors
        weight = ctx.weight
        if ctx.direct:
            # dX was produced pre-scaled; a different upstream gradient still rescales it
            # exactly, but the weight gradient is already in main_grad: flag the mismatch
            ratio = g.float() / ctx.grad_scale
            gx = dx * ratio if ctx.needs_input_grad[0] else None
            flag = _SCALE_MISMATCH.get(g.device)
            if flag is None:
                flag = _SCALE_MISMATCH[g.device] = torch.zeros((), dtype=torch.bool, device=g.device)
            flag.logical_or_((ratio - 1.0).abs() > 1e-6)
            _grad_ready(weight)
            return gx, None, None, None, None, None, None, None
        gx = dx * g if ctx.needs_input_grad[0] else None  # bf16 storage, fp32 math
        gw = None
        if G is not None:
            mg = getattr(weight, "main_grad", None)
            if mg is None:
                gw = (G * g).to(weight.dtype)
            else:
                m2 = mg.view(G.shape)
                if take_fresh(weight):
                    torch.mul(G, g, out=m2)
                else:
                    m2.addcmul_(G, g)
                _grad_ready(weight)
        return gx, gw, None, None, None, None, None, None


def fused_linear_cross_entropy(x: torch.Tensor, weight: torch.Tensor, target: torch.Tensor, vocab_start: int = 0,
                               group=None, ignore_index: int = -100, chunk: int | None = None,
                               grad_scale: float | None = None) -> torch.Tensor:
    """Mean CE of ``x @ weight^T`` against global token ids ``target`` (rows with
    ``ignore_index`` excluded), without materialising the logits.

    ``x`` [N, h] (replicated over the TP ``group``), ``weight`` [V/tp, h] this
    rank's vocab shard starting at ``vocab_start``, ``target`` [N].  ``grad_scale``:
    the upstream gradient the caller will back-propagate into the returned loss
    (the trainer's 1 / grad-accumulation steps); with a ``main_grad`` arena the weight
    gradient is then written during the forward (``check_grad_scale`` verifies it)."""
    x = x.reshape(-1, x.shape[-1])
    t = target.reshape(-1).to(x.device)
    if t.shape[0] != x.shape[0]:
        raise ValueError(f"fused LM head: {x.shape[0]} rows vs {t.shape[0]} targets")
    valid = t != ignore_index
    tgt = torch.where(valid, t, torch.zeros_like(t)).contiguous()
    chunk = max(1, int(chunk or default_chunk()))
    if not torch.is_grad_enabled() or not (x.requires_grad or weight.requires_grad):
        return _loss_only(x, weight, tgt, valid, vocab_start, group, chunk)
    return _FusedHeadCEFn.apply(x.contiguous(), weight, tgt, valid, vocab_start, group, chunk, grad_scale)

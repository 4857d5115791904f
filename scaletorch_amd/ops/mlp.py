"""SwiGLU activation and the main_grad-aware linear layer.

* ``swiglu(gate_up)`` -- csrc/swiglu.hip on the output of ONE fused gate|up GEMM
  (reference: ``down(silu(gate(x)) * up(x))``, scaletorch/models/llama.py:236-249).
* ``linear(x, w)`` -- hipBLASLt GEMM forward; backward computes dX with one GEMM
  and accumulates dW directly into ``w.main_grad`` (fp32) inside a second GEMM's
  epilogue (see ops/grad.py), which is what lets the DP bucket all-reduce start
  the moment a weight's gradient is final.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from .grad import accumulate_grad, accumulate_linear_wgrad, dgrad, prefetch_wgrad, prepare_dgrad_weight


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return _lib.ops().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dout):
        (gu,) = ctx.saved_tensors
        return _lib.ops().swiglu_bwd(dout.contiguous(), gu)


def swiglu_ref(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.chunk(2, dim=-1)
    return F.silu(g) * u


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    if _lib.use_native(gu) and gu.dtype == torch.bfloat16 and gu.shape[-1] % 16 == 0:
        return _SwiGLUFn.apply(gu)
    return swiglu_ref(gu)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.bias = bias
        if x.requires_grad:
            prepare_dgrad_weight(weight)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        pre = prefetch_wgrad(weight, dy2, x2) if ctx.needs_input_grad[1] else None  # overlaps the dgrad GEMM
        dx = dgrad(dy, weight) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            dw = accumulate_linear_wgrad(weight, dy2, x2, pre)
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = accumulate_grad(ctx.bias, dy2.float().sum(0))
        return dx, dw, db


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """F.linear whose weight gradient goes to ``weight.main_grad`` when it exists."""
    if getattr(weight, "main_grad", None) is not None and torch.is_grad_enabled():
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class _SwiGLULinearFn(torch.autograd.Function):
    """y = swiglu(gu) W^T without keeping swiglu(gu): the activation is recomputed in
    backward (one elementwise pass over gu) for the weight gradient, so a layer keeps
    gu [T, 2I] but not a [T, I] -- 1/3 of the MLP's saved activations (112 MiB per
    Llama-3-8B layer and 4096-token sample), which is what lets the 1-GPU step hold a
    larger micro-batch in 288 GB.  Reference: down(silu(gate(x)) * up(x)),
    scaletorch/models/llama.py:236-249 (autograd keeps every intermediate)."""

    @staticmethod
    def forward(ctx, gu, weight):
        gu = gu.contiguous()
        ctx.save_for_backward(gu, weight)
        if gu.requires_grad:
            prepare_dgrad_weight(weight)
        return F.linear(_lib.ops().swiglu_fwd(gu), weight)

    @staticmethod
    def backward(ctx, dy):
        gu, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        da = dgrad(dy, weight)
        if ctx.needs_input_grad[1]:
            a = _lib.ops().swiglu_fwd(gu)  # recomputed
            accumulate_linear_wgrad(weight, dy2, a.reshape(-1, a.shape[-1]))
            del a
        return _lib.ops().swiglu_bwd(da.contiguous(), gu), None


def swiglu_linear(gu: torch.Tensor, weight: torch.Tensor) -> torch.Tensor | None:
    """Fused SwiGLU + down projection that recomputes the activation in backward
    (``ST_MLP_RECOMPUTE_ACT=1``), or None (the default, and on CPU / without main_grad /
    shapes the kernels skip).  Off by default: on one MI355X at Llama-3-8B micro-batch 6
    it saves 22 GB but costs 14.5 ms/step (1026.8 vs 1012.3 ms), and the micro-batch 7 / 8
    it makes room for run at the same tokens/s (23.86k / 24.23k vs 24.28k,
    profiles/r03/swiglu_recompute_mbs.log) -- a memory lever for longer sequences."""
    import os

    if (os.environ.get("ST_MLP_RECOMPUTE_ACT", "0") == "1" and torch.is_grad_enabled()
            and getattr(weight, "main_grad", None) is not None and _lib.use_native(gu)
            and gu.dtype == torch.bfloat16 and gu.shape[-1] % 16 == 0):
        return _SwiGLULinearFn.apply(gu, weight)
    return None


class _GateUpSwiGLUFn(torch.autograd.Function):
    """h = silu(x W_gate^T) * (x W_up^T) as ONE kernel: the gate|up GEMM with the SwiGLU in its
    epilogue (csrc/gemm4w.hip ``st_gemm4w_swiglu``), which also stores gu = x [W_gate; W_up]^T
    for the backward -- the separate SwiGLU pass (read gu, write h) is gone.  Backward is the
    unfused path's: dgu = SwiGLU'(dh, gu), then the gate|up linear's dgrad / fp32 wgrad into
    ``main_grad``.  Reference: down(silu(gate(x)) * up(x)), scaletorch/models/llama.py:236-249."""

    @staticmethod
    def forward(ctx, x, weight):
        if x.requires_grad:
            prepare_dgrad_weight(weight)
        gu, h = _lib.ops().gemm_swiglu(x.reshape(-1, x.shape[-1]), weight)
        ctx.save_for_backward(x, weight, gu)
        return h.view(*x.shape[:-1], h.shape[-1])

    @staticmethod
    def backward(ctx, dh):
        x, weight, gu = ctx.saved_tensors
        dgu = _lib.ops().swiglu_bwd(dh.reshape(-1, dh.shape[-1]).contiguous(), gu)
        x2 = x.reshape(-1, x.shape[-1])
        pre = prefetch_wgrad(weight, dgu, x2) if ctx.needs_input_grad[1] else None  # overlaps the dgrad GEMM
        dx = dgrad(dgu.view(*x.shape[:-1], dgu.shape[-1]), weight) if ctx.needs_input_grad[0] else None
        dw = accumulate_linear_wgrad(weight, dgu, x2, pre) if ctx.needs_input_grad[1] else None
        return dx, dw


def _gemm_swiglu_tiles(x2: torch.Tensor, weight: torch.Tensor) -> bool:
    """The shapes / layouts csrc/gemm4w.hip ``st_gemm4w_swiglu`` takes (it returns -2 otherwise)."""
    K, I2 = x2.shape[1], weight.shape[0]
    ldx, ldw = x2.stride(0), weight.stride(0)
    return (K % 64 == 0 and I2 % 256 == 0 and x2.stride(1) == 1 and weight.stride(1) == 1 and ldx % 8 == 0
            and ldw % 8 == 0 and ldx >= K and ldw >= K and x2.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0
            and (256 + 32) * ldx * 2 < 2 ** 32 and I2 * ldw * 2 < 2 ** 32 and 0 < x2.shape[0] < 2 ** 31)


def gate_up_swiglu_ok(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """Whether ``gate_up_swiglu`` runs the fused kernel for these operands: opt-in
    ``ST_MLP_FUSED_SWIGLU=1`` (off by default), GPU bf16, shapes the kernel tiles, not the
    activation-recompute mode.  Measured (docs/PERF.md round 5, profiles/r05/gemm4w/): the
    kernel runs the gate|up GEMM at hipBLASLt's rate (4.19 vs 4.18 ms with the SwiGLU pass)
    but the headline step is 8-10 ms slower with it -- the side-stream AdamW overlaps it worse."""
    import os

    if (os.environ.get("ST_MLP_FUSED_SWIGLU", "0") != "1" or os.environ.get("ST_MLP_RECOMPUTE_ACT", "0") == "1"
            or not x.is_cuda or not _lib.use_native(x) or x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16
            or weight.dim() != 2 or x.numel() == 0):
        return False
    return _gemm_swiglu_tiles(x.reshape(-1, x.shape[-1]), weight)


def gate_up_swiglu(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """``swiglu(x @ weight^T)`` for a fused [gate; up] weight in ONE kernel (the caller checked
    ``gate_up_swiglu_ok``); the weight gradient goes to ``weight.main_grad`` when present."""
    if torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad):
        return _GateUpSwiGLUFn.apply(x, weight)
    gu, h = _lib.ops().gemm_swiglu(x.reshape(-1, x.shape[-1]), weight)
    return h.view(*x.shape[:-1], h.shape[-1])

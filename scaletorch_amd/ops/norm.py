"""RMSNorm and fused residual-add + RMSNorm (HIP kernels: csrc/rmsnorm.hip).

Reference: ``RMSNorm`` in scaletorch/models/attention_utils.py:247-271.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from .grad import accumulate_grad


def rms_norm_ref(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * weight.float()).to(x.dtype)


class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, eps):
        x = x.contiguous()
        y, rstd, _ = _lib.ops().rmsnorm_fwd(x, None, weight, eps)
        ctx.save_for_backward(x, weight, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, rstd = ctx.saved_tensors
        dw = torch.zeros(weight.numel(), dtype=torch.float32, device=x.device)
        dx = _lib.ops().rmsnorm_bwd(dy.contiguous(), x, weight, rstd, None, dw)
        return dx, accumulate_grad(weight, dw), None


class _AddRMSNormFn(torch.autograd.Function):
    """(x, residual) -> (rmsnorm(x + residual) * w, x + residual)."""

    @staticmethod
    def forward(ctx, x, residual, weight, eps):
        x = x.contiguous()
        residual = residual.contiguous()
        y, rstd, s = _lib.ops().rmsnorm_fwd(x, residual, weight, eps)
        ctx.save_for_backward(s, weight, rstd)
        return y, s

    @staticmethod
    def backward(ctx, dy, ds_extra):
        s, weight, rstd = ctx.saved_tensors
        dw = torch.zeros(weight.numel(), dtype=torch.float32, device=s.device)
        dres = ds_extra.contiguous() if ds_extra is not None else None
        ds = _lib.ops().rmsnorm_bwd(dy.contiguous(), s, weight, rstd, dres, dw)
        return ds, ds, accumulate_grad(weight, dw), None


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    if _lib.use_native(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192:
        return _RMSNormFn.apply(x, weight, eps)
    return rms_norm_ref(x, weight, eps)


def add_rms_norm(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor, eps: float):
    """Returns ``(rms_norm(x + residual), x + residual)`` with the add fused into the norm."""
    if _lib.use_native(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192:
        return _AddRMSNormFn.apply(x, residual, weight, eps)
    s = x + residual
    return rms_norm_ref(s, weight, eps), s


class RMSNorm(nn.Module):
    """Drop-in RMSNorm (``weight`` param name matches the reference checkpoint keys)."""

    def __init__(self, hidden_size: int, eps: float = 1e-6):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden_size))

    def reset_parameters(self) -> None:
        nn.init.ones_(self.weight)

    def forward(self, x: torch.Tensor, residual: torch.Tensor | None = None):
        if residual is None:
            return rms_norm(x, self.weight, self.eps)
        return add_rms_norm(x, residual, self.weight, self.eps)

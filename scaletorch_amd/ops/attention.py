"""Rotary embedding tables and fused RoPE + flash attention.

HIP kernels: csrc/rope.hip, csrc/flash_attn.hip.  Reference behaviour:
``apply_rotary_pos_emb`` / ``get_cos_sin`` (scaletorch/models/attention_utils.py:170-239)
and ``flash_attention`` (same file :130-152), which expands K/V to all query
heads and calls SDPA.  Here:

* ``rope_attention(qkv, ...)`` consumes the output of ONE fused QKV GEMM
  ``[B, S, (H + 2 Hkv) * D]``: RoPE is applied in place to the q and k sections
  (strided views, no copies), the flash kernel reads q/k/v straight out of that
  buffer with GQA-native indexing (K/V never expanded), and backward writes
  dQ/dK/dV straight into the slices of one ``dQKV`` buffer, then un-rotates
  dQ/dK in place.  The QKV GEMM output is not saved by the GEMM's own autograd
  node, so rotating it in place is safe.
* ``flash_attn(q, k, v, ...)`` exposes the raw kernels (with lse and global
  position offsets) for ring attention and the attention-variant modules.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _lib
from .grad import accumulate_grad


# ---------------------------------------------------------------- RoPE tables
def rope_tables(
    max_pos: int,
    head_dim: int,
    theta: float = 500000.0,
    scaling: dict | None = None,
    device: torch.device | str = "cpu",
):
    """fp32 cos/sin tables of shape [max_pos, head_dim/2] (rotate-half convention).

    Supports Llama-3.1 style ``rope_scaling={"rope_type": "llama3", ...}``.
    """
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and (scaling.get("rope_type") or scaling.get("type")) == "llama3":
        factor = scaling.get("factor", 8.0)
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        wavelen = 2 * math.pi / inv_freq
        lo_w, hi_w = old / lo, old / hi
        smooth = (old / wavelen - lo) / (hi - lo)
        scaled = torch.where(wavelen > lo_w, inv_freq / factor, inv_freq)
        mid = (wavelen <= lo_w) & (wavelen >= hi_w)
        inv_freq = torch.where(mid, (1 - smooth) * inv_freq / factor + smooth * inv_freq, scaled)
    elif scaling and (scaling.get("rope_type") or scaling.get("type")) == "linear":
        inv_freq = inv_freq / scaling.get("factor", 1.0)
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv_freq)
    return freqs.cos().float().to(device), freqs.sin().float().to(device)


def apply_rope_ref(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor | None,
                   inverse: bool = False) -> torch.Tensor:
    """x [B, S, NH, D]; cos/sin [max_pos, D/2]; pos [B, S] or None (= arange)."""
    B, S = x.shape[0], x.shape[1]
    if pos is None:
        c, s = cos[:S][None, :, None, :], sin[:S][None, :, None, :]
    else:
        c, s = cos[pos][:, :, None, :], sin[pos][:, :, None, :]
    if inverse:
        s = -s
    half = x.shape[-1] // 2
    xf = x.float()
    x1, x2 = xf[..., :half], xf[..., half:]
    out = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
    return out.to(x.dtype)


class _RopeFn(torch.autograd.Function):
    """Out-of-place RoPE on [B, S, NH, D] (copy + in-place HIP kernel); backward = inverse rotation."""

    @staticmethod
    def forward(ctx, x, cos, sin, pos):
        y = x.contiguous().clone()
        _lib.ops().rope_(y, cos, sin, pos, 0, False)
        ctx.save_for_backward(cos, sin, pos if pos is not None else torch.empty(0))
        ctx.has_pos = pos is not None
        return y

    @staticmethod
    def backward(ctx, g):
        cos, sin, pos = ctx.saved_tensors
        dx = g.contiguous().clone()
        _lib.ops().rope_(dx, cos, sin, pos if ctx.has_pos else None, 0, True)
        return dx, None, None, None


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor | None) -> torch.Tensor:
    """Rotate [B, S, NH, D] by global positions ``pos`` ([B, S]) or arange(S)."""
    if _lib.use_native(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 16 == 0:
        return _RopeFn.apply(x, cos, sin, pos.contiguous() if pos is not None else None)
    return apply_rope_ref(x, cos, sin, pos)


# ---------------------------------------------------------------- reference attention
def sdpa_ref(q, k, v, causal: bool, scale: float, q_offset: int = 0, k_offset: int = 0):
    """q [B,Sq,H,D], k/v [B,Sk,Hkv,D] -> (out [B,Sq,H,D], lse [B,H,Sq]) in fp32 math."""
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    g = H // Hkv
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3).repeat_interleave(g, dim=1)
    vf = v.float().permute(0, 2, 1, 3).repeat_interleave(g, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        qi = torch.arange(Sq, device=q.device)[:, None] + q_offset
        ki = torch.arange(Sk, device=q.device)[None, :] + k_offset
        s = s.masked_fill(ki > qi, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse[..., None])
    p = torch.nan_to_num(p, nan=0.0)
    out = torch.matmul(p, vf).permute(0, 2, 1, 3)
    return out.to(q.dtype), lse


# ---------------------------------------------------------------- raw flash kernels
def flash_attn_fwd(q, k, v, scale: float, causal: bool, q_offset: int = 0, k_offset: int = 0):
    """(out [B,Sq,H,D] bf16, lse [B,H,Sq] fp32)."""
    if _lib.use_native(q):
        out, lse = _lib.ops().flash_fwd(q, k, v, scale, causal, q_offset, k_offset)
        return out, lse
    return sdpa_ref(q, k, v, causal, scale, q_offset, k_offset)


def flash_attn_bwd(dout, q, k, v, out, lse, scale: float, causal: bool, q_offset: int = 0,
                   k_offset: int = 0, dq=None, dk=None, dv=None, one_shot: bool = False):
    """(dq, dk, dv) for one attention block (writes into dq/dk/dv when given).
    ``one_shot``: the recompute-dQ backward even where the dS-materialising one applies."""
    if _lib.use_native(q):
        return _lib.ops().flash_bwd(dout.contiguous(), q, k, v, out, lse, scale, causal, q_offset,
                                    k_offset, dq, dk, dv, 0 if one_shot else -1)
    gq, gk, gv = flash_bwd_ref(dout, q, k, v, out, lse, scale, causal, q_offset, k_offset)
    res = []
    for g, dst, ref in ((gq, dq, q), (gk, dk, k), (gv, dv, v)):
        if dst is not None:
            dst.copy_(g)
            res.append(dst)
        else:
            res.append(g.to(ref.dtype))
    return tuple(res)


def flash_bwd_ref(dout, q, k, v, out, lse, scale, causal, q_offset=0, k_offset=0):
    """fp32 reference of the flash backward for one K/V block, using the GIVEN
    (possibly global, ring-merged) ``out`` and ``lse`` -- exactly what the HIP kernel computes."""
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    g = H // Hkv
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3).repeat_interleave(g, dim=1)
    vf = v.float().permute(0, 2, 1, 3).repeat_interleave(g, dim=1)
    do = dout.float().permute(0, 2, 1, 3)
    o = out.float().permute(0, 2, 1, 3)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        qi = torch.arange(Sq, device=q.device)[:, None] + q_offset
        ki = torch.arange(Sk, device=q.device)[None, :] + k_offset
        s = s.masked_fill(ki > qi, float("-inf"))
    p = torch.exp(s - lse.float()[..., None]).nan_to_num(0.0)
    dv = torch.matmul(p.transpose(-1, -2), do)
    dp = torch.matmul(do, vf.transpose(-1, -2))
    delta = (do * o).sum(-1, keepdim=True)
    ds = p * (dp - delta)
    dq = torch.matmul(ds, kf) * scale
    dk = torch.matmul(ds.transpose(-1, -2), qf) * scale
    dk = dk.view(B, Hkv, g, Sk, D).sum(2)
    dv = dv.view(B, Hkv, g, Sk, D).sum(2)
    return dq.permute(0, 2, 1, 3), dk.permute(0, 2, 1, 3), dv.permute(0, 2, 1, 3)


def _sdpa_fp32(q, k, v, causal, scale, q_offset, k_offset):
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    g = H // Hkv
    qf = q.permute(0, 2, 1, 3)
    kf = k.permute(0, 2, 1, 3).repeat_interleave(g, dim=1)
    vf = v.permute(0, 2, 1, 3).repeat_interleave(g, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        qi = torch.arange(Sq, device=q.device)[:, None] + q_offset
        ki = torch.arange(Sk, device=q.device)[None, :] + k_offset
        s = s.masked_fill(ki > qi, float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    return torch.matmul(p, vf).permute(0, 2, 1, 3), None


class _FlashFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal):
        out, lse = _lib.ops().flash_fwd(q, k, v, scale, causal, 0, 0)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.scale, ctx.causal = scale, causal
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dq, dk, dv = _lib.ops().flash_bwd(dout.contiguous(), q, k, v, out, lse, ctx.scale, ctx.causal, 0, 0,
                                          None, None, None)
        return dq, dk, dv, None, None


def flash_attn(q, k, v, causal: bool = True, scale: float | None = None):
    """Autograd flash attention on [B, S, H, D] tensors (GQA when k/v have fewer heads)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if _lib.use_native(q) and q.dtype == torch.bfloat16 and q.shape[-1] in (64, 128):
        return _FlashFn.apply(q, k, v, scale, causal)
    g = q.shape[2] // k.shape[2]
    qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    if g > 1:
        kt = kt.repeat_interleave(g, dim=1)
        vt = vt.repeat_interleave(g, dim=1)
    o = F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal, scale=scale)
    return o.transpose(1, 2)


# ---------------------------------------------------------------- fused rope + attention
class DQLink:
    """Hand-off between an attention backward and the QKV projection's backward.

    With the dS-materialising flash backward, dQ = dS K is a separate HBM-bound pass
    (~0.7 ms per Llama-3-8B layer at micro-batch 6).  When the attention is given a link,
    its backward runs that pass (and dQ's inverse RoPE) on a side stream and returns at
    once; the QKV projection's backward -- the next node, holding the same link -- computes
    the k/v columns' data and weight gradients (compute-bound GEMMs) first, then waits on
    ``event`` and adds the q columns.  ``keep`` pins what the side stream still reads.
    Opt-in (``ST_FLASH_DQ_OVERLAP=1``): at Llama-3-8B micro-batch 6 it measured 3.7 ms per
    step slower than the inline pass (profiles/r03/dq_overlap_ab.log)."""

    __slots__ = ("event", "split", "keep")

    def __init__(self, split: int):
        self.event, self.split, self.keep = None, split, None

    def wait(self) -> None:
        if self.event is not None:
            torch.cuda.current_stream().wait_event(self.event)
        self.event, self.keep = None, None


_DQ_STREAMS: dict = {}


def _dq_stream(device: torch.device):
    st = _DQ_STREAMS.get(device.index)
    if st is None:
        st = _DQ_STREAMS[device.index] = torch.cuda.Stream(device=device)
    return st


class _RopeAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, pos, H, Hkv, D, causal, scale, link=None):
        B, S = qkv.shape[0], qkv.shape[1]
        qkv4 = qkv.view(B, S, H + 2 * Hkv, D)
        ops = _lib.ops()
        ops.rope_(qkv4[:, :, : H + Hkv], cos, sin, pos, 0, False)  # in place: q and k
        q, k, v = qkv4[:, :, :H], qkv4[:, :, H: H + Hkv], qkv4[:, :, H + Hkv:]
        out, lse = ops.flash_fwd(q, k, v, scale, causal, 0, 0)
        ctx.save_for_backward(qkv4, out, lse, cos, sin, pos if pos is not None else torch.empty(0))
        ctx.meta = (H, Hkv, D, causal, scale, pos is not None)
        ctx.link = link
        return out.view(B, S, H * D)

    @staticmethod
    def backward(ctx, dout):
        qkv4, out, lse, cos, sin, pos = ctx.saved_tensors
        H, Hkv, D, causal, scale, has_pos = ctx.meta
        B, S = qkv4.shape[0], qkv4.shape[1]
        ops = _lib.ops()
        dqkv = torch.empty_like(qkv4)
        q, k, v = qkv4[:, :, :H], qkv4[:, :, H: H + Hkv], qkv4[:, :, H + Hkv:]
        dout4 = dout.view(B, S, H, D).contiguous()
        pos_t = pos if has_pos else None
        link = ctx.link
        if link is not None:
            _, _, ws = ops.flash_bwd_kv(dout4, q, k, v, out, lse, scale, causal, 0, 0,
                                        dqkv[:, :, H: H + Hkv], dqkv[:, :, H + Hkv:])
            if ws.numel():
                ops.rope_(dqkv[:, :, H: H + Hkv], cos, sin, pos_t, 0, True)  # dK now; dQ on the side
                main = torch.cuda.current_stream()
                side = _dq_stream(qkv4.device)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    ops.flash_bwd_q_ds(q, k, ws, scale, causal, 0, 0, dqkv[:, :, :H])
                    ops.rope_(dqkv[:, :, :H], cos, sin, pos_t, 0, True)
                    ev = torch.cuda.Event()
                    ev.record(side)
                link.event, link.keep = ev, (ws, qkv4, cos, sin, pos_t, dqkv)
                return dqkv.view(B, S, -1), None, None, None, None, None, None, None, None, None
            # no dS workspace for this problem: the one-call backward (dK / dV are rewritten)
        ops.flash_bwd(dout4, q, k, v, out, lse, scale, causal, 0, 0,
                      dqkv[:, :, :H], dqkv[:, :, H: H + Hkv], dqkv[:, :, H + Hkv:])
        ops.rope_(dqkv[:, :, : H + Hkv], cos, sin, pos_t, 0, True)
        return dqkv.view(B, S, -1), None, None, None, None, None, None, None, None, None


class _QKNormRopeAttnFn(torch.autograd.Function):
    """Qwen3 attention core: per-head q/k RMSNorm + RoPE fused in place on the QKV
    buffer (csrc/qknorm_rope.hip), then flash attention; backward: flash backward,
    then the fused inverse-RoPE + RMSNorm backward on dQ / dK with the two weight
    gradients reduced on device."""

    @staticmethod
    def forward(ctx, qkv, wq, wk, cos, sin, pos, H, Hkv, D, causal, scale, eps):
        B, S = qkv.shape[0], qkv.shape[1]
        qkv4 = qkv.view(B, S, H + 2 * Hkv, D)
        ops = _lib.ops()
        xsave, rstd = ops.qknorm_rope_fwd_(qkv4, wq, wk, cos, sin, pos, H, Hkv, eps)
        q, k, v = qkv4[:, :, :H], qkv4[:, :, H: H + Hkv], qkv4[:, :, H + Hkv:]
        out, lse = ops.flash_fwd(q, k, v, scale, causal, 0, 0)
        ctx.save_for_backward(qkv4, out, lse, xsave, rstd, cos, sin, pos if pos is not None else torch.empty(0))
        ctx.wq, ctx.wk = wq, wk
        ctx.meta = (H, Hkv, D, causal, scale, pos is not None)
        return out.view(B, S, H * D)

    @staticmethod
    def backward(ctx, dout):
        qkv4, out, lse, xsave, rstd, cos, sin, pos = ctx.saved_tensors
        H, Hkv, D, causal, scale, has_pos = ctx.meta
        B, S = qkv4.shape[0], qkv4.shape[1]
        ops = _lib.ops()
        dqkv = torch.empty_like(qkv4)
        q, k, v = qkv4[:, :, :H], qkv4[:, :, H: H + Hkv], qkv4[:, :, H + Hkv:]
        ops.flash_bwd(dout.view(B, S, H, D).contiguous(), q, k, v, out, lse, scale, causal, 0, 0,
                      dqkv[:, :, :H], dqkv[:, :, H: H + Hkv], dqkv[:, :, H + Hkv:])
        dw = ops.qknorm_rope_bwd_(dqkv, xsave, rstd, ctx.wq, ctx.wk, cos, sin, pos if has_pos else None, H, Hkv)
        gq = accumulate_grad(ctx.wq, dw[0]) if ctx.needs_input_grad[1] else None
        gk = accumulate_grad(ctx.wk, dw[1]) if ctx.needs_input_grad[2] else None
        return dqkv.view(B, S, -1), gq, gk, None, None, None, None, None, None, None, None, None


def qknorm_rope_attention(qkv: torch.Tensor, q_weight: torch.Tensor, k_weight: torch.Tensor, eps: float,
                          cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor | None, n_heads: int,
                          n_kv_heads: int, head_dim: int, causal: bool = True,
                          scale: float | None = None) -> torch.Tensor | None:
    """Fused Qwen3 QK-norm + RoPE + attention on qkv [B, S, (H + 2 Hkv) D]; None when
    the HIP path does not apply (caller runs the unfused modules)."""
    if not (_lib.use_native(qkv) and qkv.dtype == torch.bfloat16 and head_dim in (64, 128)
            and q_weight.dtype == torch.bfloat16 and k_weight.dtype == torch.bfloat16):
        return None
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    if pos is not None:
        pos = pos.contiguous()
    return _QKNormRopeAttnFn.apply(qkv.contiguous(), q_weight, k_weight, cos, sin, pos, n_heads, n_kv_heads,
                                   head_dim, causal, scale, eps)


def rope_attention(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor | None,
                   n_heads: int, n_kv_heads: int, head_dim: int, causal: bool = True,
                   scale: float | None = None, link: DQLink | None = None) -> torch.Tensor:
    """qkv [B, S, (H + 2 Hkv) * D] -> attention output [B, S, H * D].  ``link``: the
    QKV projection's backward finishes dQ (see DQLink); only for a qkv that IS that
    projection's output."""
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    B, S = qkv.shape[0], qkv.shape[1]
    if (_lib.use_native(qkv) and qkv.dtype == torch.bfloat16 and head_dim in (64, 128)):
        if pos is not None:
            pos = pos.contiguous()
        return _RopeAttnFn.apply(qkv.contiguous(), cos, sin, pos, n_heads, n_kv_heads, head_dim, causal, scale,
                                 link)
    qkv4 = qkv.view(B, S, n_heads + 2 * n_kv_heads, head_dim)
    q = apply_rope_ref(qkv4[:, :, :n_heads], cos, sin, pos)
    k = apply_rope_ref(qkv4[:, :, n_heads: n_heads + n_kv_heads], cos, sin, pos)
    v = qkv4[:, :, n_heads + n_kv_heads:]
    return flash_attn(q, k, v, causal=causal, scale=scale).reshape(B, S, n_heads * head_dim)

"""Attention backend registry (reference: scaletorch/models/attention_utils.py:33-64,
backends registered in scaletorch/models/llama.py:38-57).

A backend maps the fused QKV projection output ``qkv [B, S, (H + 2 Hkv) * D]``
(RoPE not yet applied) to the attention output ``[B, S, H * D]``; the decoder's
attention module picks one by name.  Registered here:

* ``flash`` -- the gfx950 HIP path: RoPE in place on the QKV buffer + flash
  forward/backward kernels reading GQA K/V without expansion (ops/attention.py);
  on CPU the same math in fp32 PyTorch.
* ``sdpa`` -- RoPE + ``torch.nn.functional.scaled_dot_product_attention`` on K/V
  expanded to every query head (the reference's non-flash path); used when
  ``--use_flash_attention False``.
* ``ring`` / ``context_parallel`` -- context-parallel attention over the CP group
  (parallel/context_parallel.py: overlapped K/V all-gather, ring or Ulysses).

Selection (``resolve_attention_backend_name``) follows the reference: context
parallel first, then flash vs sdpa from the flag -- but it is read from the
trainer's config once, not from env vars at module construction (the reference's
CONTEXT_PARALLEL env var was set after the model was built).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import ops

_ATTENTION_REGISTRY: dict = {}
_DEFAULT = {"use_flash": True}


def register_attention_backend(name: str):
    """Decorator: register ``fn(qkv, cos, sin, position_ids, H, Hkv, D, scale)``."""

    def deco(fn):
        _ATTENTION_REGISTRY[name] = fn
        return fn

    return deco


def get_attention_backend(name: str):
    if name not in _ATTENTION_REGISTRY:
        raise KeyError(f"Unknown attention backend {name!r}. Registered: {sorted(_ATTENTION_REGISTRY)}")
    return _ATTENTION_REGISTRY[name]


def registered_attention_backends() -> list[str]:
    return sorted(_ATTENTION_REGISTRY)


def set_use_flash_attention(flag: bool) -> None:
    """Trainer hook for ``--use_flash_attention``."""
    _DEFAULT["use_flash"] = bool(flag)


def resolve_attention_backend_name(use_context_parallel: bool, use_flash_attn: bool | None = None) -> str:
    if use_context_parallel:
        return "ring"
    if use_flash_attn is None:
        use_flash_attn = _DEFAULT["use_flash"]
    return "flash" if use_flash_attn else "sdpa"


@register_attention_backend("flash")
def _flash_backend(qkv, cos, sin, position_ids, H, Hkv, D, scale):
    return ops.rope_attention(qkv, cos, sin, position_ids, H, Hkv, D, causal=True, scale=scale)


@register_attention_backend("sdpa")
def _sdpa_backend(qkv, cos, sin, position_ids, H, Hkv, D, scale):
    B, S = qkv.shape[0], qkv.shape[1]
    qkv4 = qkv.view(B, S, H + 2 * Hkv, D)
    q = ops.apply_rope(qkv4[:, :, :H], cos, sin, position_ids).transpose(1, 2)
    k = ops.apply_rope(qkv4[:, :, H: H + Hkv], cos, sin, position_ids).transpose(1, 2)
    v = qkv4[:, :, H + Hkv:].transpose(1, 2)
    if H != Hkv:  # the reference expands K/V to every query head (llama.py:175-191)
        k = k.repeat_interleave(H // Hkv, dim=1)
        v = v.repeat_interleave(H // Hkv, dim=1)
    o = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=scale)
    return o.transpose(1, 2).reshape(B, S, H * D)


@register_attention_backend("ring")
def _cp_backend(qkv, cos, sin, position_ids, H, Hkv, D, scale):
    from ..parallel.context_parallel import context_parallel_attention

    return context_parallel_attention(qkv, cos, sin, position_ids, H, Hkv, D, scale)


_ATTENTION_REGISTRY["context_parallel"] = _cp_backend


def attention(qkv: torch.Tensor, cos, sin, position_ids, H: int, Hkv: int, D: int, scale: float,
              backend: str | None = None) -> torch.Tensor:
    """Dispatch to ``backend`` (default: resolved from the mesh and the flash flag)."""
    if backend is None:
        from ..parallel import mesh

        backend = resolve_attention_backend_name(mesh.cp_size() > 1)
    return get_attention_backend(backend)(qkv, cos, sin, position_ids, H, Hkv, D, scale)

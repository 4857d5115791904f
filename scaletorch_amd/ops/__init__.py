"""Fused operators: hand-written gfx950 HIP kernels + PyTorch reference paths.

Every op dispatches on the tensor's device: GPU tensors go to the HIP kernels in
``csrc/`` (and raise if the library is missing), CPU tensors to the reference
implementation of the same op, which is also what the numerics tests compare
the kernels against.
"""
from . import _lib, moe
from .attention import (apply_rope, apply_rope_ref, flash_attn, flash_attn_bwd, flash_attn_fwd,
                        qknorm_rope_attention, rope_attention, rope_tables, sdpa_ref)
from .mlp import linear, swiglu, swiglu_ref
from .norm import RMSNorm, add_rms_norm, rms_norm, rms_norm_ref
from .xent import cross_entropy

__all__ = [
    "_lib", "moe", "apply_rope", "apply_rope_ref", "flash_attn", "flash_attn_fwd", "flash_attn_bwd", "rope_attention",
    "qknorm_rope_attention",
    "rope_tables", "sdpa_ref", "linear", "swiglu", "swiglu_ref", "RMSNorm", "add_rms_norm", "rms_norm",
    "rms_norm_ref", "cross_entropy",
]

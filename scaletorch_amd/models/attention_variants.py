"""Stand-alone attention variants: MHA, MQA, GQA, MLA.

Reference: scaletorch/models/attention/{base,mha,mqa,gqa,mla}.py -- educational
modules that materialise the S x S score matrix.  Here every variant shares
one core: projections -> (optional RoPE) -> the HIP flash kernel, which is
GQA-native, so MQA (1 KV head) and GQA (G KV heads) never expand K/V.  MLA
(DeepSeek-style latent attention) compresses K/V through a low-rank latent
(``kv_lora_rank``) and optionally Q through ``q_lora_rank``; its up-projections
produce per-head K/V that go through the same kernel.
Inputs/outputs are [batch, seq, hidden]; an optional boolean ``attention_mask``
([B, S] padding mask) falls back to masked SDPA.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


class BaseAttention(nn.Module):
    def __init__(self, hidden_size: int, num_heads: int, num_kv_heads: int, head_dim: int | None = None,
                 dropout: float = 0.0, bias: bool = False, causal: bool = True, rope_theta: float | None = None,
                 max_position: int = 4096):
        super().__init__()
        if num_heads % num_kv_heads:
            raise ValueError(f"num_heads {num_heads} must be a multiple of num_kv_heads {num_kv_heads}")
        self.hidden_size, self.num_heads, self.num_kv_heads = hidden_size, num_heads, num_kv_heads
        self.head_dim = head_dim or hidden_size // num_heads
        self.dropout, self.causal = dropout, causal
        self.scale = 1.0 / math.sqrt(self.head_dim)
        self.q_proj = nn.Linear(hidden_size, num_heads * self.head_dim, bias=bias)
        self.k_proj = nn.Linear(hidden_size, num_kv_heads * self.head_dim, bias=bias)
        self.v_proj = nn.Linear(hidden_size, num_kv_heads * self.head_dim, bias=bias)
        self.out_proj = nn.Linear(num_heads * self.head_dim, hidden_size, bias=bias)
        self.rope = rope_theta is not None
        if self.rope:
            cos, sin = ops.rope_tables(max_position, self.head_dim, rope_theta)
            self.register_buffer("cos", cos, persistent=False)
            self.register_buffer("sin", sin, persistent=False)

    def _attend(self, q, k, v, attention_mask=None):
        """q [B,S,H,D], k/v [B,S,Hkv,D] -> [B,S,H*D]."""
        B, S = q.shape[0], q.shape[1]
        if self.rope:
            q = ops.apply_rope(q, self.cos, self.sin, None)
            k = ops.apply_rope(k, self.cos, self.sin, None)
        if attention_mask is None and not (self.dropout and self.training):
            o = ops.flash_attn(q, k, v, causal=self.causal, scale=self.scale)
        else:
            g = self.num_heads // k.shape[2]
            qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
            if g > 1:
                kt, vt = kt.repeat_interleave(g, 1), vt.repeat_interleave(g, 1)
            mask = None
            if attention_mask is not None:
                mask = attention_mask[:, None, None, :].bool()
                if self.causal:
                    mask = mask & torch.ones(S, S, dtype=torch.bool, device=q.device).tril()
            o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=mask,
                                               dropout_p=self.dropout if self.training else 0.0,
                                               is_causal=self.causal and mask is None, scale=self.scale)
            o = o.transpose(1, 2)
        return o.reshape(B, S, -1)

    def forward(self, x: torch.Tensor, attention_mask: torch.Tensor | None = None) -> torch.Tensor:
        B, S, _ = x.shape
        q = self.q_proj(x).view(B, S, self.num_heads, self.head_dim)
        k = self.k_proj(x).view(B, S, self.num_kv_heads, self.head_dim)
        v = self.v_proj(x).view(B, S, self.num_kv_heads, self.head_dim)
        return self.out_proj(self._attend(q, k, v, attention_mask))


class MultiHeadAttention(BaseAttention):
    def __init__(self, hidden_size: int, num_heads: int, **kw):
        super().__init__(hidden_size, num_heads, num_heads, **kw)


class MultiQueryAttention(BaseAttention):
    def __init__(self, hidden_size: int, num_heads: int, **kw):
        super().__init__(hidden_size, num_heads, 1, **kw)


class GroupQueryAttention(BaseAttention):
    def __init__(self, hidden_size: int, num_heads: int, num_kv_groups: int, **kw):
        super().__init__(hidden_size, num_heads, num_kv_groups, **kw)
        self.num_kv_groups = num_kv_groups


class MultiHeadLatentAttention(nn.Module):
    """Latent (low-rank) K/V compression; KV cache would hold only the latent."""

    def __init__(self, hidden_size: int, num_heads: int, kv_lora_rank: int, q_lora_rank: int | None = None,
                 head_dim: int | None = None, causal: bool = True, bias: bool = False):
        super().__init__()
        self.num_heads, self.head_dim = num_heads, head_dim or hidden_size // num_heads
        self.causal, self.scale = causal, 1.0 / math.sqrt(self.head_dim)
        hd = num_heads * self.head_dim
        if q_lora_rank:
            self.q_down = nn.Linear(hidden_size, q_lora_rank, bias=bias)
            self.q_norm = ops.RMSNorm(q_lora_rank)
            self.q_up = nn.Linear(q_lora_rank, hd, bias=bias)
        else:
            self.q_proj = nn.Linear(hidden_size, hd, bias=bias)
        self.kv_down = nn.Linear(hidden_size, kv_lora_rank, bias=bias)
        self.kv_norm = ops.RMSNorm(kv_lora_rank)
        self.k_up = nn.Linear(kv_lora_rank, hd, bias=bias)
        self.v_up = nn.Linear(kv_lora_rank, hd, bias=bias)
        self.out_proj = nn.Linear(hd, hidden_size, bias=bias)

    def forward(self, x: torch.Tensor, attention_mask: torch.Tensor | None = None) -> torch.Tensor:
        B, S, _ = x.shape
        q = self.q_up(self.q_norm(self.q_down(x))) if hasattr(self, "q_down") else self.q_proj(x)
        latent = self.kv_norm(self.kv_down(x))
        k, v = self.k_up(latent), self.v_up(latent)
        H, D = self.num_heads, self.head_dim
        q, k, v = (t.view(B, S, H, D) for t in (q, k, v))
        o = ops.flash_attn(q, k, v, causal=self.causal, scale=self.scale)
        return self.out_proj(o.reshape(B, S, H * D))


class LeNet(nn.Module):
    """MNIST LeNet used by the examples (reference scaletorch/models/lenet.py)."""

    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.dropout1, self.dropout2 = nn.Dropout(0.25), nn.Dropout(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, num_classes)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = torch.flatten(self.dropout1(x), 1)
        x = self.dropout2(F.relu(self.fc1(x)))
        return F.log_softmax(self.fc2(x), dim=1)

"""nanoGPT-style GPT with optional Mixture-of-Experts blocks (+ minGPT sizes).

Reference: scaletorch/models/moe.py (GPTConfig, CausalSelfAttention, MLPExperts,
Router with noisy top-k / capacity / aux + router-z losses, MOELayer, GPT with
weight tying, generate, estimate_mfu, analyze_moe_usage).

MI355X-specific choices: attention runs through the HIP flash kernel
(head_dim 64/128) instead of a masked S^2 matmul; expert dispatch sorts the
(token, expert) assignments once and scatters them into a capacity-padded
[E, C, d] buffer so ALL experts run as one batched GEMM (``torch.bmm`` ->
hipBLASLt batched), instead of building a dense [T, E, C] dispatch tensor and
two einsums.
"""
from __future__ import annotations

import inspect
import math
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..utils.device import get_theoretical_flops


@dataclass
class GPTConfig:
    block_size: int = 1024
    vocab_size: int = 50304
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    dropout: float = 0.0
    bias: bool = True
    use_moe: bool = False
    moe_layers: list[int] | None = None
    n_experts: int = 8
    top_k: int = 2
    capacity_factor: float = 1.25
    use_aux_loss: bool = False
    use_router_z_loss: bool = False
    use_noisy_top_k: bool = True
    aux_loss_weight: float = 0.01
    router_z_loss_weight: float = 0.01
    train_capacity: float = 1.25
    eval_capacity: float = 2.0
    min_capacity: float = 0.0
    use_switch_tfm_init: bool = False
    switch_tfm_init_scale: float = 1.0
    use_optimized_routing: bool = True
    use_einsum_aggregation: bool = True
    expert_capacity_roundup: bool = True

    def __post_init__(self) -> None:
        for n in ("block_size", "vocab_size", "n_layer", "n_head", "n_embd"):
            if getattr(self, n) <= 0:
                raise ValueError(f"{n} must be positive, got {getattr(self, n)}")
        if self.n_embd % self.n_head:
            raise ValueError(f"n_embd ({self.n_embd}) must be divisible by n_head ({self.n_head})")
        if not 0.0 <= self.dropout <= 1.0:
            raise ValueError(f"dropout must be in [0, 1], got {self.dropout}")
        if self.use_moe:
            if self.n_experts <= 0:
                raise ValueError(f"n_experts must be positive, got {self.n_experts}")
            if not 1 <= self.top_k <= self.n_experts:
                raise ValueError(f"top_k ({self.top_k}) must be between 1 and n_experts ({self.n_experts})")
            if self.capacity_factor <= 0:
                raise ValueError(f"capacity_factor must be positive, got {self.capacity_factor}")
        if self.switch_tfm_init_scale <= 0:
            raise ValueError(f"switch_tfm_init_scale must be positive, got {self.switch_tfm_init_scale}")


# minGPT presets (examples/torch_examples/minigpt: gpt-mini = 6L/6H/192)
GPT_PRESETS = {
    "openai-gpt": dict(n_layer=12, n_head=12, n_embd=768),
    "gpt2": dict(n_layer=12, n_head=12, n_embd=768),
    "gpt2-medium": dict(n_layer=24, n_head=16, n_embd=1024),
    "gpt-mini": dict(n_layer=6, n_head=6, n_embd=192),
    "gpt-micro": dict(n_layer=4, n_head=4, n_embd=128),
    "gpt-nano": dict(n_layer=3, n_head=3, n_embd=48),
}


class LayerNorm(nn.Module):
    def __init__(self, ndim: int, bias: bool):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(ndim))
        self.bias = nn.Parameter(torch.zeros(ndim)) if bias else None

    def forward(self, x):
        return F.layer_norm(x, self.weight.shape, self.weight, self.bias, 1e-5)


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.c_attn = nn.Linear(cfg.n_embd, 3 * cfg.n_embd, bias=cfg.bias)
        self.c_proj = nn.Linear(cfg.n_embd, cfg.n_embd, bias=cfg.bias)
        self.attn_dropout, self.resid_dropout = nn.Dropout(cfg.dropout), nn.Dropout(cfg.dropout)
        self.n_head, self.n_embd, self.dropout = cfg.n_head, cfg.n_embd, cfg.dropout

    def forward(self, x):
        B, T, C = x.shape
        q, k, v = self.c_attn(x).split(self.n_embd, dim=2)
        D = C // self.n_head
        q, k, v = (t.view(B, T, self.n_head, D) for t in (q, k, v))
        if self.dropout > 0 and self.training:
            y = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                               dropout_p=self.dropout, is_causal=True).transpose(1, 2)
        else:
            y = ops.flash_attn(q, k, v, causal=True)
        return self.resid_dropout(self.c_proj(y.reshape(B, T, C)))


class GELUMLP(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.c_fc = nn.Linear(cfg.n_embd, 4 * cfg.n_embd, bias=cfg.bias)
        self.c_proj = nn.Linear(4 * cfg.n_embd, cfg.n_embd, bias=cfg.bias)
        self.dropout = nn.Dropout(cfg.dropout)

    def forward(self, x):
        return self.dropout(self.c_proj(F.gelu(self.c_fc(x))))


class Block(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.ln_1, self.attn = LayerNorm(cfg.n_embd, cfg.bias), CausalSelfAttention(cfg)
        self.ln_2, self.mlp = LayerNorm(cfg.n_embd, cfg.bias), GELUMLP(cfg)

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class MLPExperts(nn.Module):
    """All experts' weights stacked: c_fc [E, d, 4d], c_proj [E, 4d, d] (batched GEMMs)."""

    def __init__(self, cfg: GPTConfig):
        super().__init__()
        d, E = cfg.n_embd, cfg.n_experts
        self.bias = cfg.bias
        self.c_fc = nn.Parameter(torch.empty(E, d, 4 * d))
        self.c_proj = nn.Parameter(torch.empty(E, 4 * d, d))
        self.fc_bias = nn.Parameter(torch.zeros(E, 1, 4 * d)) if cfg.bias else None
        self.proj_bias = nn.Parameter(torch.zeros(E, 1, d)) if cfg.bias else None
        self.dropout = nn.Dropout(cfg.dropout)
        self.cfg = cfg
        self._init_weights()

    def _init_weights(self) -> None:
        if self.cfg.use_switch_tfm_init:
            s = self.cfg.switch_tfm_init_scale
            for w in (self.c_fc, self.c_proj):
                fan_in = w.shape[1]
                std = math.sqrt(s / fan_in)
                nn.init.trunc_normal_(w, mean=0.0, std=std, a=-2 * std, b=2 * std)
        else:
            nn.init.normal_(self.c_fc, 0.0, 0.02)
            nn.init.normal_(self.c_proj, 0.0, 0.02 / math.sqrt(2 * self.cfg.n_layer))

    def forward(self, x):  # x [E, C, d]
        h = torch.bmm(x, self.c_fc)
        if self.fc_bias is not None:
            h = h + self.fc_bias
        h = torch.bmm(F.gelu(h), self.c_proj)
        if self.proj_bias is not None:
            h = h + self.proj_bias
        return self.dropout(h)


class Router(nn.Module):
    """Noisy top-k router with expert capacity, Switch aux loss and router z-loss."""

    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.cfg = cfg
        self.top_k, self.n_exp = cfg.top_k, cfg.n_experts
        self.w_g = nn.Linear(cfg.n_embd, cfg.n_experts, bias=False)
        self.w_noise = nn.Linear(cfg.n_embd, cfg.n_experts, bias=False) if cfg.use_noisy_top_k else None

    def _compute_expert_capacity(self, tokens: int) -> int:
        cf = self.cfg.train_capacity if self.training else self.cfg.eval_capacity
        cap = math.floor(self.top_k * cf * tokens / self.n_exp)
        if self.cfg.expert_capacity_roundup:
            cap += cap % 2
        return max(int(cap), int(self.cfg.min_capacity), 1)

    def compute_router_z_loss(self, logits):
        return torch.logsumexp(logits.float(), dim=-1).pow(2).mean()

    def compute_aux_loss(self, probs, indices):
        T = probs.shape[0]
        one_hot = torch.zeros(T, self.n_exp, device=probs.device).scatter_(1, indices, 1.0)
        f = one_hot.mean(0) / self.top_k
        P = probs.mean(0)
        return self.n_exp * (f * P).sum()

    def forward(self, x2d):
        logits = self.w_g(x2d).float()
        if self.w_noise is not None and self.training:
            noise = F.softplus(self.w_noise(x2d).float()) * torch.randn_like(logits)
            logits = logits + noise
        topv, topi = logits.topk(self.top_k, dim=-1)
        w = torch.softmax(topv, dim=-1)  # softmax over the selected experts
        aux = z = None
        if self.training and self.cfg.use_aux_loss:
            aux = self.compute_aux_loss(torch.softmax(logits, -1), topi)
        if self.training and self.cfg.use_router_z_loss:
            z = self.compute_router_z_loss(logits)
        return w, topi, self._compute_expert_capacity(x2d.shape[0]), aux, z


class MOELayer(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.router = Router(cfg)
        self.experts = MLPExperts(cfg)
        self.cfg = cfg
        self.last_usage = None

    def forward(self, x):
        B, T, d = x.shape
        x2 = x.reshape(-1, d)
        w, idx, cap, aux, z = self.router(x2)
        N, k, E = x2.shape[0], self.cfg.top_k, self.cfg.n_experts
        flat_e = idx.reshape(-1)
        order = torch.argsort(flat_e, stable=True)  # token-major priority within each expert
        se = flat_e[order]
        counts = torch.bincount(flat_e, minlength=E)
        starts = torch.cumsum(counts, 0) - counts
        slot = torch.arange(N * k, device=x.device) - starts[se]
        keep = slot < cap  # capacity: overflow assignments are dropped
        tok = order // k
        buf = x2.new_zeros(E, cap, d)
        buf[se[keep], slot[keep]] = x2[tok[keep]]
        out_e = self.experts(buf)
        y = out_e[se[keep], slot[keep]] * w.reshape(-1)[order][keep].to(x.dtype)[:, None]
        out = torch.zeros_like(x2).index_add(0, tok[keep], y)
        self.last_usage = counts.detach()
        loss = None
        if aux is not None:
            loss = self.cfg.aux_loss_weight * aux
        if z is not None:
            loss = (loss or 0) + self.cfg.router_z_loss_weight * z
        return out.view(B, T, d), loss


class MoEBlock(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.ln_1, self.attn = LayerNorm(cfg.n_embd, cfg.bias), CausalSelfAttention(cfg)
        self.ln_2, self.mlp = LayerNorm(cfg.n_embd, cfg.bias), MOELayer(cfg)

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        m, loss = self.mlp(self.ln_2(x))
        return x + m, loss


class GPT(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.config = cfg
        moe_layers = (list(range(cfg.n_layer // 2, cfg.n_layer)) if cfg.use_moe and cfg.moe_layers is None
                      else (cfg.moe_layers or []))
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(cfg.vocab_size, cfg.n_embd),
            wpe=nn.Embedding(cfg.block_size, cfg.n_embd),
            drop=nn.Dropout(cfg.dropout),
            blocks=nn.ModuleList([MoEBlock(cfg) if i in moe_layers else Block(cfg) for i in range(cfg.n_layer)]),
            ln_f=LayerNorm(cfg.n_embd, cfg.bias),
        ))
        self.lm_head = nn.Linear(cfg.n_embd, cfg.vocab_size, bias=False)
        self.transformer.wte.weight = self.lm_head.weight
        self.apply(self._init_weights)
        for pn, p in self.named_parameters():
            if pn.endswith("c_proj.weight"):
                nn.init.normal_(p, 0.0, 0.02 / math.sqrt(2 * cfg.n_layer))

    @staticmethod
    def _init_weights(m):
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, 0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, 0.02)

    def get_num_params(self, non_embedding: bool = True) -> int:
        n = sum(p.numel() for p in self.parameters())
        if non_embedding:
            n -= self.transformer.wpe.weight.numel()
        return n

    def forward(self, idx, targets=None):
        B, T = idx.shape
        if T > self.config.block_size:
            raise ValueError(f"Sequence length {T} exceeds block size {self.config.block_size}")
        pos = torch.arange(T, device=idx.device)
        x = self.transformer.drop(self.transformer.wte(idx) + self.transformer.wpe(pos))
        aux, n_aux = 0.0, 0
        for blk in self.transformer.blocks:
            if isinstance(blk, MoEBlock):
                x, l = blk(x)
                if l is not None:
                    aux, n_aux = aux + l, n_aux + 1
            else:
                x = blk(x)
        x = self.transformer.ln_f(x)
        if targets is not None:
            logits = self.lm_head(x)
            loss = F.cross_entropy(logits.reshape(-1, logits.size(-1)).float(), targets.reshape(-1), ignore_index=-1)
            if n_aux:
                loss = loss + aux / n_aux
        else:
            logits, loss = self.lm_head(x[:, [-1], :]), None
        return logits, loss

    def crop_block_size(self, block_size: int) -> None:
        assert block_size <= self.config.block_size
        self.config.block_size = block_size
        self.transformer.wpe.weight = nn.Parameter(self.transformer.wpe.weight[:block_size])

    def configure_optimizers(self, weight_decay, learning_rate, betas, device_type="cuda"):
        params = [p for p in self.parameters() if p.requires_grad]
        decay = [p for p in params if p.dim() >= 2]
        nodecay = [p for p in params if p.dim() < 2]
        groups = [{"params": decay, "weight_decay": weight_decay}, {"params": nodecay, "weight_decay": 0.0}]
        fused = "fused" in inspect.signature(torch.optim.AdamW).parameters and device_type == "cuda"
        return torch.optim.AdamW(groups, lr=learning_rate, betas=betas, fused=fused)

    @torch.no_grad()
    def generate(self, idx, max_new_tokens: int, temperature: float = 1.0, top_k: int | None = None,
                 do_sample: bool = True):
        for _ in range(max_new_tokens):
            ctx = idx if idx.size(1) <= self.config.block_size else idx[:, -self.config.block_size:]
            logits, _ = self(ctx)
            logits = logits[:, -1, :].float() / temperature
            if top_k is not None:
                v, _ = torch.topk(logits, min(top_k, logits.size(-1)))
                logits[logits < v[:, [-1]]] = -float("inf")
            probs = F.softmax(logits, dim=-1)
            nxt = torch.multinomial(probs, 1) if do_sample else probs.argmax(-1, keepdim=True)
            idx = torch.cat((idx, nxt), dim=1)
        return idx

    def estimate_mfu(self, fwdbwd_per_iter: int, dt: float) -> float:
        """MFU against the MI355X dense bf16 peak (the reference used A100 312 TF)."""
        N = self.get_num_params()
        c = self.config
        L, H, Q, T = c.n_layer, c.n_head, c.n_embd // c.n_head, c.block_size
        flops = (6 * N + 12 * L * H * Q * T) * T * fwdbwd_per_iter
        return flops / dt / get_theoretical_flops()


def analyze_moe_usage(model: GPT) -> dict:
    out = {}
    for i, blk in enumerate(model.transformer.blocks):
        if isinstance(blk, MoEBlock) and blk.mlp.last_usage is not None:
            u = blk.mlp.last_usage.float()
            out[f"layer_{i}"] = {"usage": u.tolist(), "balance_cv": (u.std() / u.mean().clamp(min=1e-9)).item()}
    return out


def get_moe_layer_info(model: GPT, layer_idx: int) -> dict | None:
    blk = model.transformer.blocks[layer_idx]
    if not isinstance(blk, MoEBlock):
        return None
    return {"n_experts": model.config.n_experts, "top_k": model.config.top_k,
            "expert_params": sum(p.numel() for p in blk.mlp.experts.parameters())}

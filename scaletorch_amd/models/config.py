"""Model configuration + built-in registry (no network needed for synthetic runs).

The reference builds every model from ``AutoConfig.from_pretrained``
(scaletorch/trainer/model_builder.py:61-74); with no hub access here, the
common architectures are registered by name (values from their public HF
configs) and a local HF directory (config.json) still works.
"""
from __future__ import annotations

import copy
import json
import os
from dataclasses import asdict, dataclass, field, fields


@dataclass
class ModelConfig:
    model_type: str = "llama"  # llama | qwen3 | qwen3_moe | mixtral
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int | None = None
    head_dim: int | None = None
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: dict | None = None
    tie_word_embeddings: bool = False
    qk_norm: bool = False
    attention_bias: bool = False
    initializer_range: float = 0.02
    init: str = "uniform"  # reference llama: uniform(+-1/sqrt(fan_in)); qwen3: normal(0.02)
    # MoE
    num_experts: int = 0
    num_experts_per_tok: int = 2
    moe_intermediate_size: int | None = None
    norm_topk_prob: bool = True
    router_aux_loss_coef: float = 0.001
    decoder_sparse_step: int = 1
    mlp_only_layers: list = field(default_factory=list)
    name: str = "custom"

    def __post_init__(self):
        if self.num_key_value_heads is None:
            self.num_key_value_heads = self.num_attention_heads
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_attention_heads
        if self.num_experts and self.moe_intermediate_size is None:
            self.moe_intermediate_size = self.intermediate_size

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    def layer_is_moe(self, i: int) -> bool:
        return (self.is_moe and i not in self.mlp_only_layers
                and (i + 1) % max(1, self.decoder_sparse_step) == 0)

    def to_dict(self) -> dict:
        return asdict(self)

    def num_params(self) -> int:
        """Analytic parameter count (full model, unsharded)."""
        h, d = self.hidden_size, self.head_dim
        attn = h * d * (self.num_attention_heads + 2 * self.num_key_value_heads) + self.num_attention_heads * d * h
        if self.qk_norm:
            attn += 2 * d
        dense_mlp = 3 * h * self.intermediate_size
        total = 0
        for i in range(self.num_hidden_layers):
            total += attn + 2 * h
            if self.layer_is_moe(i):
                total += self.num_experts * 3 * h * self.moe_intermediate_size + h * self.num_experts
            else:
                total += dense_mlp
        total += self.vocab_size * h + h
        if not self.tie_word_embeddings:
            total += self.vocab_size * h
        return total

    def matmul_params(self, active: bool = True) -> int:
        """Parameters that take part in a GEMM per token: ``active_params`` minus the input
        embedding table, a gather (kept when tied: the same matrix is the LM head GEMM).
        6x this (+ causal attention) is the strict model-FLOP count (bench ``mfu_pct_strict``)."""
        n = self.active_params() if active else self.num_params()
        return n if self.tie_word_embeddings else n - self.vocab_size * self.hidden_size

    def active_params(self) -> int:
        """Parameters touched per token (MoE: top-k experts only)."""
        if not self.is_moe:
            return self.num_params()
        c = copy.deepcopy(self)
        n_moe = sum(self.layer_is_moe(i) for i in range(self.num_hidden_layers))
        full = self.num_params()
        inactive = n_moe * (self.num_experts - self.num_experts_per_tok) * 3 * self.hidden_size * self.moe_intermediate_size
        del c
        return full - inactive


_REGISTRY: dict[str, dict] = {
    # Llama family (meta-llama/* config.json)
    "llama3-8b": dict(model_type="llama", vocab_size=128256, hidden_size=4096, intermediate_size=14336,
                      num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                      max_position_embeddings=8192, rms_norm_eps=1e-5, rope_theta=500000.0),
    "llama3.1-8b": dict(model_type="llama", vocab_size=128256, hidden_size=4096, intermediate_size=14336,
                        num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                        max_position_embeddings=131072, rms_norm_eps=1e-5, rope_theta=500000.0,
                        rope_scaling=dict(rope_type="llama3", factor=8.0, low_freq_factor=1.0,
                                          high_freq_factor=4.0, original_max_position_embeddings=8192)),
    "llama3-70b": dict(model_type="llama", vocab_size=128256, hidden_size=8192, intermediate_size=28672,
                       num_hidden_layers=80, num_attention_heads=64, num_key_value_heads=8,
                       max_position_embeddings=8192, rms_norm_eps=1e-5, rope_theta=500000.0),
    "llama3.2-1b": dict(model_type="llama", vocab_size=128256, hidden_size=2048, intermediate_size=8192,
                        num_hidden_layers=16, num_attention_heads=32, num_key_value_heads=8, head_dim=64,
                        max_position_embeddings=131072, rms_norm_eps=1e-5, rope_theta=500000.0,
                        tie_word_embeddings=True),
    "llama2-7b": dict(model_type="llama", vocab_size=32000, hidden_size=4096, intermediate_size=11008,
                      num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=32,
                      max_position_embeddings=4096, rms_norm_eps=1e-5, rope_theta=10000.0),
    # Qwen3 family (Qwen/Qwen3-* config.json)
    "qwen3-0.6b": dict(model_type="qwen3", vocab_size=151936, hidden_size=1024, intermediate_size=3072,
                       num_hidden_layers=28, num_attention_heads=16, num_key_value_heads=8, head_dim=128,
                       max_position_embeddings=40960, rms_norm_eps=1e-6, rope_theta=1000000.0,
                       tie_word_embeddings=True, qk_norm=True, init="normal"),
    "qwen3-1.7b": dict(model_type="qwen3", vocab_size=151936, hidden_size=2048, intermediate_size=6144,
                       num_hidden_layers=28, num_attention_heads=16, num_key_value_heads=8, head_dim=128,
                       max_position_embeddings=40960, rms_norm_eps=1e-6, rope_theta=1000000.0,
                       tie_word_embeddings=True, qk_norm=True, init="normal"),
    "qwen3-4b": dict(model_type="qwen3", vocab_size=151936, hidden_size=2560, intermediate_size=9728,
                     num_hidden_layers=36, num_attention_heads=32, num_key_value_heads=8, head_dim=128,
                     max_position_embeddings=40960, rms_norm_eps=1e-6, rope_theta=1000000.0,
                     tie_word_embeddings=True, qk_norm=True, init="normal"),
    "qwen3-8b": dict(model_type="qwen3", vocab_size=151936, hidden_size=4096, intermediate_size=12288,
                     num_hidden_layers=36, num_attention_heads=32, num_key_value_heads=8, head_dim=128,
                     max_position_embeddings=40960, rms_norm_eps=1e-6, rope_theta=1000000.0,
                     qk_norm=True, init="normal"),
    "qwen3-14b": dict(model_type="qwen3", vocab_size=151936, hidden_size=5120, intermediate_size=17408,
                      num_hidden_layers=40, num_attention_heads=40, num_key_value_heads=8, head_dim=128,
                      max_position_embeddings=40960, rms_norm_eps=1e-6, rope_theta=1000000.0,
                      qk_norm=True, init="normal"),
    "qwen3-32b": dict(model_type="qwen3", vocab_size=151936, hidden_size=5120, intermediate_size=25600,
                      num_hidden_layers=64, num_attention_heads=64, num_key_value_heads=8, head_dim=128,
                      max_position_embeddings=40960, rms_norm_eps=1e-6, rope_theta=1000000.0,
                      qk_norm=True, init="normal"),
    "qwen3-30b-a3b": dict(model_type="qwen3_moe", vocab_size=151936, hidden_size=2048, intermediate_size=6144,
                          moe_intermediate_size=768, num_hidden_layers=48, num_attention_heads=32,
                          num_key_value_heads=4, head_dim=128, max_position_embeddings=40960, rms_norm_eps=1e-6,
                          rope_theta=1000000.0, qk_norm=True, num_experts=128, num_experts_per_tok=8,
                          norm_topk_prob=True, init="normal"),
    # Mixtral (mistralai/Mixtral-8x7B-v0.1)
    "mixtral-8x7b": dict(model_type="mixtral", vocab_size=32000, hidden_size=4096, intermediate_size=14336,
                         num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                         max_position_embeddings=32768, rms_norm_eps=1e-5, rope_theta=1000000.0,
                         num_experts=8, num_experts_per_tok=2, norm_topk_prob=True, router_aux_loss_coef=0.02),
    # tiny test / smoke configs
    "tiny-llama": dict(model_type="llama", vocab_size=512, hidden_size=256, intermediate_size=512,
                       num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                       max_position_embeddings=1024, rms_norm_eps=1e-5, rope_theta=10000.0),
    "tiny-qwen3": dict(model_type="qwen3", vocab_size=512, hidden_size=256, intermediate_size=512,
                       num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, head_dim=64,
                       max_position_embeddings=1024, rms_norm_eps=1e-6, rope_theta=1000000.0,
                       tie_word_embeddings=True, qk_norm=True, init="normal"),
    "tiny-moe": dict(model_type="qwen3_moe", vocab_size=512, hidden_size=256, intermediate_size=512,
                     moe_intermediate_size=128, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                     head_dim=64, max_position_embeddings=1024, rms_norm_eps=1e-6, rope_theta=1000000.0,
                     qk_norm=True, num_experts=8, num_experts_per_tok=2, init="normal"),
    # 8 query / 8 KV heads: every TP size of the reference's 8-device table (scripts/bench_reference_rows_8gpu.py --smoke)
    "tiny-qwen3-8h": dict(model_type="qwen3", vocab_size=512, hidden_size=256, intermediate_size=512,
                          num_hidden_layers=2, num_attention_heads=8, num_key_value_heads=8, head_dim=32,
                          max_position_embeddings=1024, rms_norm_eps=1e-6, rope_theta=1000000.0,
                          tie_word_embeddings=True, qk_norm=True, init="normal"),
    "tiny-moe-8h": dict(model_type="qwen3_moe", vocab_size=512, hidden_size=256, intermediate_size=512,
                        moe_intermediate_size=128, num_hidden_layers=2, num_attention_heads=8, num_key_value_heads=8,
                        head_dim=32, max_position_embeddings=1024, rms_norm_eps=1e-6, rope_theta=1000000.0,
                        qk_norm=True, num_experts=8, num_experts_per_tok=2, init="normal"),
    "tiny-mixtral": dict(model_type="mixtral", vocab_size=512, hidden_size=256, intermediate_size=256,
                         num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                         max_position_embeddings=1024, rms_norm_eps=1e-5, rope_theta=1000000.0,
                         num_experts=8, num_experts_per_tok=2),
}

_ALIASES = {
    "meta-llama/meta-llama-3-8b": "llama3-8b", "meta-llama/llama-3-8b": "llama3-8b",
    "meta-llama/llama-3.1-8b": "llama3.1-8b", "meta-llama/meta-llama-3.1-8b": "llama3.1-8b",
    "meta-llama/llama-2-7b-hf": "llama2-7b", "qwen/qwen3-0.6b": "qwen3-0.6b", "qwen/qwen3-1.7b": "qwen3-1.7b",
    "qwen/qwen3-4b": "qwen3-4b", "qwen/qwen3-8b": "qwen3-8b", "qwen/qwen3-14b": "qwen3-14b",
    "qwen/qwen3-32b": "qwen3-32b", "qwen/qwen3-30b-a3b": "qwen3-30b-a3b",
    "mistralai/mixtral-8x7b-v0.1": "mixtral-8x7b",
}


def registered_models() -> list[str]:
    return sorted(_REGISTRY)


def _from_hf_dict(d: dict) -> ModelConfig:
    mt = d.get("model_type", "llama")
    kw = {}
    names = {f.name for f in fields(ModelConfig)}
    for k, v in d.items():
        if k in names:
            kw[k] = v
    if mt == "qwen3":
        kw.setdefault("qk_norm", True)
        kw.setdefault("init", "normal")
    elif mt == "qwen3_moe":
        kw.setdefault("qk_norm", True)
        kw.setdefault("init", "normal")
    elif mt == "mixtral":
        kw["num_experts"] = d.get("num_local_experts", 8)
    kw["model_type"] = mt if mt in ("llama", "qwen3", "qwen3_moe", "mixtral") else "llama"
    return ModelConfig(**kw)


def get_model_config(name_or_path: str, **overrides) -> ModelConfig:
    """Registry name, alias, local HF dir (config.json) or a JSON file."""
    key = name_or_path.lower()
    key = _ALIASES.get(key, key)
    if key in _REGISTRY:
        cfg = ModelConfig(name=key, **_REGISTRY[key])
    elif os.path.isdir(name_or_path) and os.path.exists(os.path.join(name_or_path, "config.json")):
        with open(os.path.join(name_or_path, "config.json")) as f:
            cfg = _from_hf_dict(json.load(f))
        cfg.name = name_or_path
    elif os.path.isfile(name_or_path) and name_or_path.endswith(".json"):
        with open(name_or_path) as f:
            cfg = _from_hf_dict(json.load(f))
        cfg.name = name_or_path
    else:
        raise ValueError(f"unknown model {name_or_path!r}; registered: {', '.join(registered_models())}")
    for k, v in overrides.items():
        if v is not None:
            setattr(cfg, k, v)
    if overrides.get("num_attention_heads") is not None and overrides.get("head_dim") is None:
        pass
    return cfg

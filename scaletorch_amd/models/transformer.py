"""Decoder-only transformer: Llama-2/3, Qwen3 (QK-norm, tied embeddings),
Qwen3-MoE and Mixtral (MoE MLP), built TP/SP/CP/PP/EP-aware from the mesh.

Reference: scaletorch/models/llama.py (Llama), model_qwen3.py (Qwen3),
model_qwen3_moe.py (Qwen3-MoE).  Module / parameter names follow the reference
contract (``embedding``, ``decoder_layers.{i}.{input_layernorm, attention,
post_attention_layernorm, mlp|moe}``, ``final_norm``, ``final_proj``) so
checkpoints map 1:1; the fused QKV / gate-up GEMMs are split back into
``q_proj/k_proj/v_proj`` and ``gate_proj/up_proj`` by
``reference_state_dict``.

Hot path per layer on MI355X (all bf16):
  add+RMSNorm (HIP)  -> QKV GEMM (hipBLASLt) -> RoPE in place + flash fwd (HIP)
  -> out_proj GEMM -> add+RMSNorm (HIP) -> gate|up GEMM -> SwiGLU (HIP) -> down GEMM
The residual add of every sub-block is fused into the next norm kernel: layers
pass ``(x, residual)`` pairs, so no standalone elementwise add kernel runs.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint as torch_checkpoint

from .. import ops
from ..parallel import mesh
from ..parallel.tensor_parallel import (ColumnParallelLinear, FusedColumnParallelLinear, RowParallelLinear,
                                        VocabParallelEmbedding)
from .config import ModelConfig


class Attention(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int, sequence_parallel: bool = False):
        super().__init__()
        tp = mesh.tp_size()
        H, Hkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        if H % tp or Hkv % tp:
            raise ValueError(f"heads ({H}, kv {Hkv}) must be divisible by tp={tp}")
        self.layer_idx = layer_idx
        self.H, self.Hkv, self.D = H // tp, Hkv // tp, D
        self.scale = 1.0 / math.sqrt(D)
        init = dict(init=cfg.init, init_std=cfg.initializer_range)
        self.qkv_proj = FusedColumnParallelLinear(cfg.hidden_size, [H * D, Hkv * D, Hkv * D],
                                                  ["q_proj", "k_proj", "v_proj"], bias=cfg.attention_bias,
                                                  sequence_parallel=sequence_parallel, **init)
        self.out_proj = RowParallelLinear(H * D, cfg.hidden_size, bias=False, sequence_parallel=sequence_parallel,
                                          **init)
        self.qk_norm = cfg.qk_norm
        if cfg.qk_norm:
            self.q_norm = ops.RMSNorm(D, eps=cfg.rms_norm_eps)
            self.k_norm = ops.RMSNorm(D, eps=cfg.rms_norm_eps)
            self.q_norm._per_head = self.k_norm._per_head = True  # grads summed over this rank's heads only
            # the fused QK-norm+RoPE kernel reads these weights without calling the modules:
            # DataParallel makes this module's forward wait for their optimizer buckets too
            self._st_reads = (self.q_norm, self.k_norm)

    def reset_parameters(self) -> None:
        self.qkv_proj.reset_parameters()
        self.out_proj.reset_parameters()
        if self.qk_norm:
            self.q_norm.reset_parameters()
            self.k_norm.reset_parameters()

    def forward(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                position_ids: torch.Tensor | None) -> torch.Tensor:
        from .attention_backends import attention, resolve_attention_backend_name

        H, Hkv, D = self.H, self.Hkv, self.D
        backend = resolve_attention_backend_name(mesh.cp_size() > 1)
        link = None
        if (backend == "flash" and not self.qk_norm and self.qkv_proj.tp == 1 and torch.is_grad_enabled()
                and x.is_cuda and getattr(self.qkv_proj.weight, "main_grad", None) is not None
                and os.environ.get("ST_FLASH_DQ_OVERLAP", "0") == "1"):
            # the QKV projection's backward finishes dQ beside its own k/v GEMMs (ops.attention.DQLink);
            # opt-in: measured 3.7 ms/step SLOWER at Llama-3-8B mbs 6 (profiles/r03/dq_overlap_ab.log)
            link = ops.attention.DQLink(H * D)
        self.qkv_proj._st_link = link
        try:
            qkv = self.qkv_proj(x)
        finally:
            self.qkv_proj._st_link = None
        B, S = qkv.shape[0], qkv.shape[1]
        if link is not None:
            out = ops.rope_attention(qkv, cos, sin, position_ids, H, Hkv, D, causal=True, scale=self.scale,
                                     link=link)
            return self.out_proj(out)
        if self.qk_norm and backend == "flash" and os.environ.get("ST_FUSED_QKNORM", "1") == "1":
            # Qwen3: per-head QK-norm + RoPE fused in place on the QKV buffer (csrc/qknorm_rope.hip)
            out = ops.qknorm_rope_attention(qkv, self.q_norm.weight, self.k_norm.weight, self.q_norm.eps, cos, sin,
                                            position_ids, H, Hkv, D, causal=True, scale=self.scale)
            if out is not None:
                return self.out_proj(out)
        if self.qk_norm:
            q, k, v = qkv.view(B, S, H + 2 * Hkv, D).split([H, Hkv, Hkv], dim=2)
            q = self.q_norm(q.contiguous())
            k = self.k_norm(k.contiguous())
            qkv = torch.cat([q, k, v], dim=2).view(B, S, -1)
        out = attention(qkv, cos, sin, position_ids, H, Hkv, D, self.scale, backend)  # registry dispatch
        return self.out_proj(out)


class MLP(nn.Module):
    """SwiGLU MLP with one fused gate|up GEMM (reference llama.py:207-249)."""

    def __init__(self, cfg: ModelConfig, intermediate_size: int | None = None, sequence_parallel: bool = False):
        super().__init__()
        I = intermediate_size or cfg.intermediate_size
        init = dict(init=cfg.init, init_std=cfg.initializer_range)
        self.gate_up_proj = FusedColumnParallelLinear(cfg.hidden_size, [I, I], ["gate_proj", "up_proj"],
                                                      sequence_parallel=sequence_parallel, **init)
        self.down_proj = RowParallelLinear(I, cfg.hidden_size, sequence_parallel=sequence_parallel, **init)
        # the fused SP MLP path reads both weights directly (DataParallel bucket waits); the
        # other paths call both projections as modules (ST_MLP_WAIT_BOTH=0: each waits for its
        # own bucket only -- A/B)
        import os

        if sequence_parallel or os.environ.get("ST_MLP_WAIT_BOTH", "1") == "1":
            self._st_reads = (self.gate_up_proj, self.down_proj)

    def reset_parameters(self) -> None:
        self.gate_up_proj.reset_parameters()
        self.down_proj.reset_parameters()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from ..parallel.tensor_parallel import sp_mlp_applies, sp_mlp

        if sp_mlp_applies(self, x):
            # the whole SP MLP in the gathered row layout (tensor_parallel._SPMLPFn)
            return sp_mlp(x, self.gate_up_proj.weight, self.down_proj.weight, self.gate_up_proj.group)
        gu_lin = self.gate_up_proj
        if gu_lin.tp == 1 and gu_lin.bias is None and not gu_lin.sequence_parallel:
            from ..ops.mlp import gate_up_swiglu_ok

            if gate_up_swiglu_ok(x, gu_lin.weight):  # one kernel: gate|up GEMM + SwiGLU epilogue
                return self.down_proj(gu_lin(x, act="swiglu"))
        return self.down_proj(gu_lin(x), act="swiglu")


class DecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int, sequence_parallel: bool = False):
        super().__init__()
        self.layer_idx = layer_idx
        self.input_layernorm = ops.RMSNorm(cfg.hidden_size, eps=cfg.rms_norm_eps)
        self.attention = Attention(cfg, layer_idx, sequence_parallel)
        self.post_attention_layernorm = ops.RMSNorm(cfg.hidden_size, eps=cfg.rms_norm_eps)
        self.is_moe = cfg.layer_is_moe(layer_idx)
        if self.is_moe:
            from .moe import MoELayer

            self.moe = MoELayer(cfg, sequence_parallel=sequence_parallel)
        else:
            self.mlp = MLP(cfg, sequence_parallel=sequence_parallel)

    def reset_parameters(self) -> None:
        for m in (self.input_layernorm, self.attention, self.post_attention_layernorm,
                  self.moe if self.is_moe else self.mlp):
            m.reset_parameters()

    def forward(self, x, residual, cos, sin, position_ids, selective_recompute: bool = False):
        """(x, residual) -> (block output, residual stream).  ``residual`` None = first layer.

        ``selective_recompute``: the attention sub-block keeps its activations (QKV,
        flash output + lse -- the expensive S^2 part is never recomputed) and only the
        norm + MLP sub-block is checkpointed: it holds most of a layer's activation
        bytes (gate|up output 2I, SwiGLU output I per token) and costs only GEMMs to
        recompute.  (Reference: full-layer torch.utils.checkpoint, llama.py:535-545.)"""
        if residual is None:
            h = self.input_layernorm(x)
            residual = x
        else:
            h, residual = self.input_layernorm(x, residual)
        a = self.attention(h, cos, sin, position_ids)
        if selective_recompute and self.training and torch.is_grad_enabled():
            return torch_checkpoint(self._mlp_block, a, residual, use_reentrant=False)
        return self._mlp_block(a, residual)

    def _mlp_block(self, a, residual):
        h, residual = self.post_attention_layernorm(a, residual)
        out = self.moe(h) if self.is_moe else self.mlp(h)
        return out, residual


def stage_layer_range(num_layers: int, pp_size: int, pp_rank: int,
                      distribution: list[int] | None = None) -> tuple[int, int]:
    """Contiguous layer range of a pipeline stage.

    Default split: even, first ``remainder`` stages get one extra layer
    (reference pipeline_parallel.py:83-133); ``distribution`` overrides it.
    """
    if distribution:
        if len(distribution) != pp_size or sum(distribution) != num_layers:
            raise ValueError(f"layer distribution {distribution} must have {pp_size} entries summing to {num_layers}")
        start = sum(distribution[:pp_rank])
        return start, start + distribution[pp_rank]
    base, rem = divmod(num_layers, pp_size)
    start = pp_rank * base + min(pp_rank, rem)
    return start, start + base + (1 if pp_rank < rem else 0)


class TransformerLM(nn.Module):
    """Causal LM.  ``forward`` returns this TP rank's vocab shard of the logits
    (last PP stage) or the hidden states to send to the next stage."""

    def __init__(self, cfg: ModelConfig, sequence_parallel: bool = False, layer_distribution: list[int] | None = None,
                 virtual_stages: int = 1):
        super().__init__()
        self.config = self.model_config = cfg
        self.sequence_parallel = sequence_parallel and mesh.tp_size() > 1
        pp, pr = mesh.pp_size(), (mesh.pgm.pp_rank if mesh.pgm else 0)
        self.first_stage, self.last_stage = pr == 0, pr == pp - 1
        # virtual pipeline stages (interleaved 1F1B, parallel/interleaved.py): the layers are split
        # evenly into pp*V chunks; this rank holds global chunks v*pp + pr, v = 0..V-1
        self.virtual_stages = max(1, int(virtual_stages))
        if self.virtual_stages > 1:
            nchunks = pp * self.virtual_stages
            if cfg.num_hidden_layers < nchunks:
                raise ValueError(f"{cfg.num_hidden_layers} layers cannot fill {pp} x {self.virtual_stages} chunks")
            # layer_distribution with virtual stages: one entry per GLOBAL chunk (chunk v * pp + stage,
            # in model order), e.g. "9,8,8,7" at pp 2 x V 2 gives stage 0 chunks 0 + 2 (17 layers) and
            # the last stage, which also runs the LM head and the loss, chunks 1 + 3 (15 layers)
            if layer_distribution and (len(layer_distribution) != nchunks or min(layer_distribution) < 1):
                raise ValueError(f"layer distribution {layer_distribution}: need {nchunks} entries (pp x virtual "
                                 f"stages, global chunk order), each >= 1")
            self.chunk_ranges = [stage_layer_range(cfg.num_hidden_layers, nchunks, v * pp + pr, layer_distribution)
                                 for v in range(self.virtual_stages)]
        else:
            self.chunk_ranges = [stage_layer_range(cfg.num_hidden_layers, pp, pr, layer_distribution)]
        self.layer_start, self.layer_end = self.chunk_ranges[0][0], self.chunk_ranges[-1][1]
        sp = self.sequence_parallel
        std = cfg.initializer_range if cfg.init == "normal" else None
        if self.first_stage or (cfg.tie_word_embeddings and self.last_stage):
            self.embedding = VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, sequence_parallel=sp, init_std=std)
        self.decoder_layers = nn.ModuleDict(
            {str(i): DecoderLayer(cfg, i, sp) for lo, hi in self.chunk_ranges for i in range(lo, hi)})
        if self.last_stage:
            self.final_norm = ops.RMSNorm(cfg.hidden_size, eps=cfg.rms_norm_eps)
            self.final_proj = ColumnParallelLinear(cfg.hidden_size, cfg.vocab_size, bias=False,
                                                   sequence_parallel=sp, init=cfg.init,
                                                   init_std=cfg.initializer_range)
            if cfg.tie_word_embeddings:
                self.final_proj.weight = self.embedding.weight
        # TP-replicated weights whose gradient each TP rank only sees part of
        if mesh.tp_size() > 1:
            from .moe import MoERouter

            for m in self.modules():
                partial = isinstance(m, ops.RMSNorm) and (self.sequence_parallel or getattr(m, "_per_head", False))
                partial = partial or (isinstance(m, MoERouter) and self.sequence_parallel)
                if partial:
                    for p in m.parameters():
                        p._st_tp_partial_grad = True
        # parallelism-invariant init: every weight generated in full from (seed, global name), then sharded
        from ..parallel.init import assign_init_keys

        assign_init_keys(self)
        self.reset_parameters()
        dev = next(self.parameters()).device  # tables live with the weights (kernels read them on device)
        cos, sin = ops.rope_tables(cfg.max_position_embeddings, cfg.head_dim, cfg.rope_theta, cfg.rope_scaling,
                                   device=dev)
        self.register_buffer("cos", cos, persistent=False)
        self.register_buffer("sin", sin, persistent=False)

    # ------------------------------------------------------------------ helpers
    @property
    def vocab_start(self) -> int:
        ref = self.final_proj if self.last_stage else None
        if ref is None:
            return 0
        return mesh.tp_rank() * ref.out_per_rank

    def reset_parameters(self) -> None:
        if hasattr(self, "embedding"):
            self.embedding.reset_parameters()
        for layer in self.decoder_layers.values():
            layer.reset_parameters()
        if self.last_stage:
            self.final_norm.reset_parameters()
            if not self.config.tie_word_embeddings:
                self.final_proj.reset_parameters()

    def aux_loss(self, chunk: int | None = None) -> torch.Tensor | None:
        """Sum of the MoE load-balancing losses of the last forward (of local chunk
        ``chunk`` only, with virtual pipeline stages)."""
        layers = self.decoder_layers.values() if chunk is None else \
            [self.decoder_layers[str(i)] for i in range(*self.chunk_ranges[chunk])]
        losses = [l.moe.last_aux_loss for l in layers if l.is_moe and l.moe.last_aux_loss is not None]
        if not losses:
            return None
        return torch.stack([x.float() for x in losses]).sum()

    # ------------------------------------------------------------------ forward
    def forward(self, input_ids: torch.Tensor | None = None, position_ids: torch.Tensor | None = None,
                hidden_states: torch.Tensor | None = None, gradient_checkpointing: bool = False,
                attention_mask: torch.Tensor | None = None, labels: torch.Tensor | None = None,
                lm_head_chunk: int | None = None, chunk: int | None = None,
                lm_head_grad_scale: float | None = None) -> torch.Tensor:
        """Logits shard (last stage), or -- with ``labels`` (global target ids) on
        the last stage -- the mean cross-entropy from the fused chunked LM head
        (ops/fused_head.py), which never materialises the logits.  ``chunk`` (virtual
        pipeline stages): run only local chunk v -- embedding on rank 0's chunk 0,
        final norm + head on the last rank's last chunk, hidden states otherwise."""
        V = self.virtual_stages
        if chunk is None and V > 1:
            raise ValueError("a model with virtual pipeline stages is run one chunk at a time")
        v = 0 if chunk is None else int(chunk)
        embeds = self.first_stage and v == 0
        heads = self.last_stage and v == V - 1
        lo, hi = self.chunk_ranges[v]
        if embeds:
            x = self.embedding(input_ids)
        else:
            if hidden_states is None:
                raise ValueError("hidden_states required on non-first pipeline stages")
            x = hidden_states
        residual = None
        full = gradient_checkpointing in (True, "full") and self.training
        selective = gradient_checkpointing == "selective"
        for i in range(lo, hi):
            layer = self.decoder_layers[str(i)]
            if full:
                x, residual = torch_checkpoint(layer, x, residual, self.cos, self.sin, position_ids,
                                               use_reentrant=False)
            else:
                x, residual = layer(x, residual, self.cos, self.sin, position_ids, selective_recompute=selective)
        if not heads:
            return x if residual is None else x + residual
        x = self.final_norm(x) if residual is None else self.final_norm(x, residual)[0]
        # a module call (SP: gather along seq inside the column-parallel fn), so the head's
        # forward pre-hook orders it after the weight's optimizer update / ZeRO-1 gather
        if labels is not None:
            return self.final_proj(x, labels=labels, chunk=lm_head_chunk, grad_scale=lm_head_grad_scale)
        return self.final_proj(x)

    # ------------------------------------------------------------------ checkpoints in reference layout
    def reference_state_dict(self) -> dict[str, torch.Tensor]:
        """State dict with the reference's key names (fused layers split back)."""
        out = {}
        fused = {n: m for n, m in self.named_modules() if isinstance(m, FusedColumnParallelLinear)}
        for k, v in self.state_dict().items():
            mod = k.rsplit(".", 1)[0]
            if mod in fused:
                m = fused[mod]
                parent = mod.rsplit(".", 1)[0] + "." if "." in mod else ""
                suffix = k.rsplit(".", 1)[1]
                for n, piece in zip(m.names, m.reference_pieces(v)):
                    out[f"{parent}{n}.{suffix}"] = piece
            else:
                out[k] = v
        from .moe import MoELayer

        for name, m in self.named_modules():
            if isinstance(m, MoELayer):
                out.pop(f"{name}.experts.w_gate_up", None)
                out.pop(f"{name}.experts.w_down", None)
                for k, v in m.reference_items().items():
                    out[f"{name}.{k}"] = v
        if self.config.tie_word_embeddings and "final_proj.weight" in out and "embedding.weight" in out:
            out.pop("final_proj.weight")
        return out

    def load_reference_state_dict(self, sd: dict[str, torch.Tensor], strict: bool = True):
        sd = dict(sd)
        fused = {n: m for n, m in self.named_modules() if isinstance(m, FusedColumnParallelLinear)}
        for mod, m in fused.items():
            parent = mod.rsplit(".", 1)[0] + "." if "." in mod else ""
            for suffix in ("weight", "bias"):
                keys = [f"{parent}{n}.{suffix}" for n in m.names]
                if all(k in sd for k in keys):
                    sd[f"{mod}.{suffix}"] = torch.cat([sd.pop(k) for k in keys], dim=0)
        from .moe import MoELayer

        for name, m in self.named_modules():
            if isinstance(m, MoELayer):
                gu, dn = [], []
                for e in range(m.num_local):
                    p = f"{name}.experts.experts.{e}."
                    if f"{p}gate_proj.weight" not in sd:
                        break
                    gu.append(torch.cat([sd.pop(f"{p}gate_proj.weight"), sd.pop(f"{p}up_proj.weight")], 0))
                    dn.append(sd.pop(f"{p}down_proj.weight"))
                if len(gu) == m.num_local:
                    sd[f"{name}.experts.w_gate_up"] = torch.stack(gu)
                    sd[f"{name}.experts.w_down"] = torch.stack(dn)
        if self.config.tie_word_embeddings and "final_proj.weight" not in sd and hasattr(self, "final_proj"):
            if "embedding.weight" in sd:
                sd["final_proj.weight"] = sd["embedding.weight"]
        return self.load_state_dict(sd, strict=strict)


def build_model(cfg: ModelConfig, sequence_parallel: bool = False, layer_distribution=None,
                virtual_stages: int = 1) -> TransformerLM:
    return TransformerLM(cfg, sequence_parallel=sequence_parallel, layer_distribution=layer_distribution,
                         virtual_stages=virtual_stages)

"""Per-rank HBM estimate for a (model, layout) pair, sized against 288 GB of HBM3E.

Used by ``bench.py --layout`` and ``tools/train.py`` to print what a rank will
hold before anything is allocated, so an 8-GPU layout that would not fit is
caught on the host.  The terms follow this framework's storage layout
(parallel/data_parallel.py, optim.py): bf16 parameters (+ their bf16 W^T copies), fp32 ``main_grad``
arena, fp32 master + Adam m/v (sharded over the reduction group under ZeRO-1),
and activations calibrated on one MI355X: Llama-3-8B at micro-batch 4 x 4096
peaked at 226.5 GB (profiles/micro_batch_sweep_1gpu.log), i.e. ~34 bytes per
hidden element per token per layer once the 144.5 GB of model state and the
bf16 logits (+ grad) are taken out.
"""
from __future__ import annotations

from dataclasses import dataclass

HBM_GB = 288.0
_ACT_ATTN = 14  # bytes per (token, layer, hidden element): norms, QKV, attention out, residual
_ACT_MLP = 20   # gate|up output, SwiGLU output, down input (dense MLP with I = 3.5 h)
# resident outside every term above: library GEMM workspaces, RoPE tables, the side streams'
# buffers -- measured between steps of the per-rank slices (bench.py --slice,
# profiles/r06/slices): +1.5 GB over the resident terms at DP 8, +2.0-2.5 GB at TP 2 x PP 2
_WORKSPACE_GB = 2.0
_TP_ACT_UPLIFT = 1.08
_ACT_SWIGLU = 7  # the SwiGLU output alone (I = 3.5 h bf16): not kept when it is recomputed
                 # in backward (ops/mlp.swiglu_linear: one rank, opt-in ST_MLP_RECOMPUTE_ACT=1)


@dataclass
class MemoryEstimate:
    params_gb: float
    grads_gb: float
    optimizer_gb: float
    activations_gb: float
    logits_gb: float
    comm_gb: float
    workspace_gb: float = 0.0

    @property
    def total_gb(self) -> float:
        return (self.params_gb + self.grads_gb + self.optimizer_gb + self.activations_gb + self.logits_gb
                + self.comm_gb + self.workspace_gb)

    def fits(self, capacity_gb: float = HBM_GB, headroom_gb: float | None = None) -> bool:
        import os

        if headroom_gb is None:  # allocator fragmentation + workspaces; ST_HBM_HEADROOM_GB overrides
            headroom_gb = float(os.environ.get("ST_HBM_HEADROOM_GB", "16"))
        return self.total_gb + headroom_gb <= capacity_gb

    def summary(self) -> str:
        return (f"{self.total_gb:.1f} GB/rank (params {self.params_gb:.1f}, grads {self.grads_gb:.1f}, "
                f"optimizer {self.optimizer_gb:.1f}, activations {self.activations_gb:.1f}, "
                f"logits {self.logits_gb:.1f}, comm buffers {self.comm_gb:.1f}, workspaces {self.workspace_gb:.1f}) "
                f"of {HBM_GB:.0f} GB")


def estimate_rank_memory(cfg, tp: int = 1, pp: int = 1, cp: int = 1, ep: int = 1, dp: int = 1,
                         micro_batch: int = 1, seq_len: int = 4096, grad_acc: int = 1, zero1: bool = False,
                         sequence_parallel: bool = False, gradient_checkpointing: bool = False,
                         pp_engine: str = "1f1b", grad_reduce_dtype: str = "bf16",
                         fused_head_chunk: int = 0, recompute_swiglu: bool | None = None,
                         moe_dropless: bool = False, optimizer_state_dtype: str = "fp32",
                         xgmi_ipc_bytes: float = 0.0, cp_ds_budget_bytes: float | None = None,
                         pp_rank: int = 0, virtual_pipeline: int = 1, moe_exact_rows: bool = False,
                         layer_distribution: list[int] | None = None) -> MemoryEstimate:
    """Per-rank estimate: weights of the largest stage, activations of pipeline stage
    ``pp_rank`` (default 0, the first stage: it holds the most micro-batches in flight, so
    the default is the worst rank).  In-flight work per stage: plain 1F1B holds
    min(pp - pp_rank, grad_acc) micro-batches of the whole stage; interleaved 1F1B
    (``virtual_pipeline`` V > 1) holds warm-up + 1 chunk-micro-batches of layers/V each
    (parallel/interleaved.num_warmup); AFAB holds all of them.  ``layer_distribution``: layers
    per pipeline chunk (``--layer_distribution``), this stage's sum replaces the even split.

    ``fused_head_chunk`` > 0: the fused chunked LM head (ops/fused_head.py) -- one
    chunk of logits and dX instead of the logits and their gradient.
    ``moe_dropless`` (EP > 1, models/moe.py dropless exchange): each MoE layer keeps its
    expert input and gate|up output at the host bound R_max = ep * T * min(k, E/ep) rows
    (the SwiGLU output is recomputed in backward), plus the sorted rows of the combine;
    ``moe_exact_rows`` (the RCCL transport, host counts): the buffers hold the rows the rank
    receives, T * k at uniform routing, and the SwiGLU output is kept."""
    h, d = cfg.hidden_size, cfg.head_dim
    H, Hkv = cfg.num_attention_heads, cfg.num_key_value_heads
    L = cfg.num_hidden_layers
    layers = -(-L // pp)
    if layer_distribution and pp > 1:
        # per-chunk layer counts (global chunk order v * pp + stage): this stage's chunks
        layers = sum(layer_distribution[v * pp + pp_rank] for v in range(len(layer_distribution) // pp))
    attn = (h * d * (H + 2 * Hkv) + H * d * h) / tp + 2 * h
    dense, expert = 0.0, 0.0
    for i in range(layers):
        dense += attn
        if cfg.layer_is_moe(i):
            expert += (cfg.num_experts // ep) * 3 * h * cfg.moe_intermediate_size / tp
            dense += h * cfg.num_experts
        else:
            dense += 3 * h * cfg.intermediate_size / tp
    emb = cfg.vocab_size * h / tp
    dense += emb * (1 if pp > 1 or cfg.tie_word_embeddings else 2)  # embedding (+ untied LM head)
    n = dense + expert
    dense_dp = dp * cp * ep
    expert_dp = dp * cp
    opt_bytes = 4 + (4 if optimizer_state_dtype == "bf16" else 8)  # fp32 master + m/v
    opt = opt_bytes * (dense / (dense_dp if zero1 else 1) + expert / (expert_dp if zero1 else 1))
    # activations of the micro-batches a rank holds at once
    tokens = micro_batch * seq_len / cp
    if pp > 1:
        if pp_engine == "afab":
            tokens *= grad_acc
        elif virtual_pipeline > 1:
            from ..parallel.interleaved import num_warmup

            tokens *= (num_warmup(pp, virtual_pipeline, grad_acc, pp_rank) + 1) / virtual_pipeline
        else:
            tokens *= min(pp - pp_rank, grad_acc)
    if cfg.is_moe:
        k_eff = cfg.num_experts_per_tok * cfg.moe_intermediate_size / max(1, cfg.intermediate_size)
    else:
        k_eff = 1.0
    if recompute_swiglu is None:
        import os

        recompute_swiglu = os.environ.get("ST_MLP_RECOMPUTE_ACT", "0") == "1"
    mlp_b = _ACT_MLP - (_ACT_SWIGLU if (recompute_swiglu and tp == 1 and not cfg.is_moe) else 0)
    per_layer = _ACT_ATTN * h + mlp_b * h * k_eff * cfg.intermediate_size / (3.5 * h)
    moe_extra = 0.0  # bytes per MoE layer outside the per-token model (dropless R_max buffers)
    if cfg.is_moe and ep > 1 and moe_dropless:
        k = cfg.num_experts_per_tok
        per_layer = _ACT_ATTN * h
        t_micro = micro_batch * seq_len / cp
        if moe_exact_rows:
            rows, per_row = t_micro * k, 2 * h + 6 * cfg.moe_intermediate_size / tp  # x, gu, a
        else:
            rows, per_row = ep * t_micro * min(k, cfg.num_experts // ep), 2 * h + 4 * cfg.moe_intermediate_size / tp
        moe_extra = (rows * per_row + t_micro * k * 4 * h) * (tokens / t_micro)
    if tp > 1:
        per_layer = per_layer / tp if sequence_parallel else 8 * h + (per_layer - 8 * h) / tp
        # measured: the tp 2 + SP pipeline stages hold 6-16 % more per (layer, micro-batch) than
        # the dense calibration divided by tp (bench.py --slice, profiles/r06/slices: 1.21-1.32
        # vs 1.14 GB) -- buffers that do not shard with the heads (full-sequence gathers in
        # flight, the fused head's chunk on the last stage)
        per_layer *= _TP_ACT_UPLIFT
    if gradient_checkpointing == "selective":  # attention activations kept, norm + MLP recomputed
        mlp = _ACT_MLP * h * k_eff * cfg.intermediate_size / (3.5 * h) / tp
        kept = max(per_layer - mlp, 2 * h)
        act = tokens * kept * layers + tokens * per_layer
    elif gradient_checkpointing:
        act = tokens * (2 * h * layers) + tokens * per_layer
    else:
        act = tokens * per_layer * layers
    act += moe_extra * sum(1 for i in range(layers) if cfg.layer_is_moe(i))
    head_tokens = micro_batch * seq_len / cp
    if fused_head_chunk:
        # one chunk of logits + dX (the head's dW goes straight into main_grad)
        logits = min(fused_head_chunk, head_tokens) * cfg.vocab_size / tp * 2 + head_tokens * h * 2
    else:
        logits = head_tokens * cfg.vocab_size / tp * 2 * 2  # bf16 logits + grad (last stage)
    comm = n * 2 if grad_reduce_dtype in ("bf16", "bfloat16") and dense_dp > 1 else 0.0
    comm += xgmi_ipc_bytes
    if cp > 1:
        # transient dS workspace of the CP backward: one layer at a time, causal lower triangle
        # of a zig-zag chunk pair (B * Hq * chunk * prefix, bf16) capped by the budget
        if cp_ds_budget_bytes is None:
            from ..parallel.context_parallel import _ds_budget_bytes

            cp_ds_budget_bytes = _ds_budget_bytes()
        s_loc = seq_len / cp
        widest = micro_batch * (H / tp) * (s_loc / 2) * seq_len * 2  # last zig-zag chunk x its full prefix
        from ..parallel.context_parallel import _CP_ONE_SHOT_REST

        # default (ST_CP_ONE_SHOT_REST=1): only the widest-prefix chunk keeps a dS workspace, the
        # others run the one-shot backward; all-dS mode: the budgeted workspaces + the widest
        act += widest if _CP_ONE_SHOT_REST[0] else min(cp_ds_budget_bytes, widest) + widest
    # bf16 W^T copies of the dense projection weights (TN data-gradient GEMMs, ops/grad.py)
    wt = 2 * (dense - 2 * h * layers - (h * cfg.num_experts if cfg.is_moe else 0) * layers)
    g = 1e9
    return MemoryEstimate(params_gb=(2 * n + wt) / g, grads_gb=4 * n / g, optimizer_gb=opt / g, activations_gb=act / g,
                          logits_gb=logits / g, comm_gb=comm / g, workspace_gb=_WORKSPACE_GB)

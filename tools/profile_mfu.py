#!/usr/bin/env python3
"""Analytic FLOP / byte breakdown of one training step, optionally joined with a
measured rocprofv3 kernel-stats CSV -> per-component achieved TF/s and the
step-time budget that the MFU number hides.

Reference: tools/profile_mfu.py:41-148 (analytic breakdown linear / attention /
embedding, x3 for training).  Here the breakdown is per GEMM family (QKV, O,
gate|up, down, LM head; forward / dgrad / wgrad), attention (causal, fwd + bwd
as the flash kernels execute it: 2 + 5 matmuls), the memory-bound ops (norms,
SwiGLU, RoPE, CE, AdamW bytes), and the MI355X peaks (2.5 PF dense bf16,
~6.3 TB/s measured HBM copy).

  python tools/profile_mfu.py --model llama3-8b --mbs 2 --seq 4096
  python tools/profile_mfu.py --model llama3-8b --mbs 2 --seq 4096 \\
      --stats profiles/llama3_8b_1gpu_kernel_stats.csv --steps 4 --step-ms 395
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_BF16 = 2.5e15
HBM_BW = 6.29e12  # measured float4 copy (MI355X_MICROARCH.md)


def breakdown(cfg, mbs: int, seq: int, tp: int = 1) -> dict:
    """FLOPs (and bytes for the memory-bound ops) of one optimizer step on one GPU."""
    T = mbs * seq
    h, d, L = cfg.hidden_size, cfg.head_dim, cfg.num_hidden_layers
    H, Hkv = cfg.num_attention_heads // tp, cfg.num_key_value_heads // max(1, min(tp, cfg.num_key_value_heads))
    I = (cfg.moe_intermediate_size * cfg.num_experts_per_tok if cfg.is_moe else cfg.intermediate_size) // tp
    V = cfg.vocab_size // tp
    gemms = {  # name: (M = tokens, N = out, K = in) per layer (x L) or once
        "qkv": (T, (H + 2 * Hkv) * d, h, L),
        "o_proj": (T, h, H * d, L),
        "gate_up": (T, 2 * I, h, L),
        "down": (T, h, I, L),
        "lm_head": (T, V, h, 1),
    }
    out = {}
    for name, (M, N, K, n) in gemms.items():
        f = 2.0 * M * N * K * n
        out[f"gemm_{name}_fwd"] = f
        out[f"gemm_{name}_dgrad"] = f
        out[f"gemm_{name}_wgrad"] = f
    # causal attention: QK^T and PV forward (2 matmuls), backward recomputes S and
    # does dV, dP, dQ, dK (5 matmuls); each matmul is 2*S*S*d/2 per head (causal half)
    att = 2.0 * mbs * H * seq * seq * d / 2 * L
    out["attn_fwd"] = 2 * att
    out["attn_bwd"] = 5 * att
    # memory-bound ops: bytes moved (bf16 activations, fp32 states)
    p = cfg.num_params() / tp
    byt = {
        "rmsnorm": (2 * L + 1) * T * h * 2 * (2 + 3),  # fwd r/w + bwd ~3 passes
        "swiglu": L * T * I * 2 * (3 + 5),
        "rope": L * T * (H + Hkv) * d * 2 * 2 * 2,
        "cross_entropy": T * V * 2 * 3,
        "adamw": p * 30.0,  # fp32 master/m/v/grad r+w + bf16 param write
        "grad_norm": p * 4.0,
    }
    return {"flops": out, "bytes": byt, "tokens": T}


# kernel-name -> component (rocprofv3 --stats names)
CLASSES = [
    ("attn_fwd", r"flash_fwd_kernel"),
    ("attn_bwd", r"flash_bwd_(dq|dkdv|pre)_kernel"),
    ("gemm_wgrad_hip", r"wgrad_gemm_kernel"),
    ("gemm_hipblaslt", r"^Cijk_|Custom_Cijk"),
    ("adamw", r"adamw_kernel"),
    ("grad_norm", r"sumsq_kernel|sum_partials_kernel"),
    ("rmsnorm", r"rmsnorm_(fwd|bwd)_kernel|colsum_kernel"),
    ("swiglu", r"swiglu_(fwd|bwd)_kernel"),
    ("rope", r"rope_kernel"),
    ("cross_entropy", r"xent_(fwd|bwd)_kernel"),
    ("comm", r"ncclDevKernel|rccl|xgmi|oneshot_kernel|twoshot_kernel"),
]


def measured(stats_csv: str, steps: int) -> dict:
    got = {}
    with open(stats_csv) as f:
        for row in csv.DictReader(f):
            name = row["Name"]
            cls = next((c for c, rx in CLASSES if re.search(rx, name)), "other")
            got[cls] = got.get(cls, 0.0) + float(row["TotalDurationNs"]) / 1e6 / steps
    return got


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--stats", default=None, help="rocprofv3 --stats kernel_stats.csv")
    ap.add_argument("--steps", type=int, default=1, help="training steps inside the profiled run")
    ap.add_argument("--step-ms", type=float, default=None, help="measured wall ms/step (bench.py)")
    ap.add_argument("--json", action="store_true")
    args = ap.parse_args()
    from scaletorch_amd.models import get_model_config
    from scaletorch_amd.utils.misc import flops_per_token

    cfg = get_model_config(args.model, num_hidden_layers=args.layers)
    b = breakdown(cfg, args.mbs, args.seq, args.tp)
    fl, by = b["flops"], b["bytes"]
    total = sum(fl.values())
    ideal_ms = {k: v / PEAK_BF16 * 1e3 for k, v in fl.items()}
    ideal_ms.update({k: v / HBM_BW * 1e3 for k, v in by.items()})
    model_flops = flops_per_token(cfg.active_params(), cfg.num_hidden_layers, cfg.num_attention_heads,
                                  cfg.head_dim, args.seq) * b["tokens"]
    rep = {"model": args.model, "tokens_per_step": b["tokens"], "executed_tflop": round(total / 1e12, 2),
           "mfu_definition_tflop(6N+12LHdS)": round(model_flops / 1e12, 2),
           "speed_of_light_ms": round(sum(ideal_ms.values()), 1), "components": {}}
    groups = {"gemm_fwd": [k for k in fl if k.endswith("_fwd") and k.startswith("gemm")],
              "gemm_dgrad": [k for k in fl if k.endswith("_dgrad")],
              "gemm_wgrad": [k for k in fl if k.endswith("_wgrad")],
              "attn_fwd": ["attn_fwd"], "attn_bwd": ["attn_bwd"]}
    for g, ks in groups.items():
        rep["components"][g] = {"tflop": round(sum(fl[k] for k in ks) / 1e12, 2),
                                "ideal_ms": round(sum(ideal_ms[k] for k in ks), 2)}
    for k, v in by.items():
        rep["components"][k] = {"gbytes": round(v / 1e9, 2), "ideal_ms": round(ideal_ms[k], 2)}
    if args.stats:
        m = measured(args.stats, args.steps)
        rep["measured_ms"] = {k: round(v, 2) for k, v in sorted(m.items(), key=lambda x: -x[1])}
        gemm_ms = m.get("gemm_hipblaslt", 0) + m.get("gemm_wgrad_hip", 0)
        gemm_fl = sum(v for k, v in fl.items() if k.startswith("gemm"))
        att_ms = m.get("attn_fwd", 0) + m.get("attn_bwd", 0)
        rep["achieved"] = {
            "gemm_tflops": round(gemm_fl / (gemm_ms / 1e3) / 1e12, 1) if gemm_ms else None,
            "attn_fwd_tflops": round(fl["attn_fwd"] / (m["attn_fwd"] / 1e3) / 1e12, 1) if m.get("attn_fwd") else None,
            "attn_bwd_tflops": round(fl["attn_bwd"] / (m["attn_bwd"] / 1e3) / 1e12, 1) if m.get("attn_bwd") else None,
            "adamw_tbps": round(by["adamw"] / (m["adamw"] / 1e3) / 1e12, 2) if m.get("adamw") else None,
            "kernel_ms_per_step": round(sum(m.values()), 1),
            "attention_ms": round(att_ms, 1),
        }
    if args.step_ms:
        rep["mfu_pct"] = round(model_flops / (args.step_ms / 1e3) / PEAK_BF16 * 100, 2)
        rep["executed_flops_utilisation_pct"] = round(total / (args.step_ms / 1e3) / PEAK_BF16 * 100, 2)
    if args.json:
        print(json.dumps(rep))
        return 0
    print(f"{args.model}: {b['tokens']} tokens/step, executed {rep['executed_tflop']} TFLOP "
          f"(MFU definition {rep['mfu_definition_tflop(6N+12LHdS)']} TFLOP), speed-of-light {rep['speed_of_light_ms']} ms")
    for k, v in rep["components"].items():
        print(f"  {k:16s} {json.dumps(v)}")
    for k in ("measured_ms", "achieved"):
        if k in rep:
            print(f"{k}: {json.dumps(rep[k])}")
    if "mfu_pct" in rep:
        print(f"MFU {rep['mfu_pct']} %  (executed-FLOP utilisation {rep['executed_flops_utilisation_pct']} %)")
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Same-process A/B of training-step variants (device clocks differ by up to ~10 %
between MI355X boxes, so cross-run comparisons of a few-% change are noise).

Builds ONE Llama-3-8B trainer (bench.py config) and alternates blocks of steps
between variants, reporting the median ms/step per variant:

  python tools/ab_step.py --variants overlap,serial --rounds 4 --steps 3
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def set_variant(tr, name: str, side) -> None:
    """overlap: side-stream optimizer + backward-time norms; serial: both off;
    ``K=V[+K=V...]``: environment toggles read per call (e.g. ST_WGRAD_KERNEL=0)."""
    if "=" in name:
        for kv in name.split("+"):
            k, v = kv.split("=", 1)
            if k == "TUNABLE":  # TunableOp table lookups on / off (utils/gemm_tuning.py)
                import torch

                torch.cuda.tunable.enable(v == "1")
                continue
            os.environ[k] = v
            if k.startswith("ST_WGRAD"):  # re-run the per-shape wgrad pick under this setting
                from scaletorch_amd.ops import grad as G

                G._WGRAD_CHOICE.clear()
        return
    for k in list(os.environ):
        if k.startswith("ST_WGRAD"):
            del os.environ[k]
    on = name == "overlap"
    tr.optimizer.side_stream = side if on else None
    tr.model.side_stream = side if on else None
    for a in tr.model.arenas:
        a.side_stream = side if on else None
        a.sq_count = 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--variants", default="overlap,serial")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--micro_batch_size", type=int, default=4)
    ap.add_argument("--seq_len", type=int, default=4096)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--fused_head", type=int, default=0, help="1: fused LM head + CE (bench.py default)")
    ap.add_argument("--opt_state_dtype", default="fp32")
    ap.add_argument("--gemm_tuning", default="auto")
    args = ap.parse_args()
    import torch

    from scaletorch_amd.trainer.config import ScaleTorchArguments
    from scaletorch_amd.trainer.engine import Trainer

    a = ScaleTorchArguments(model_name_or_path=args.model, synthetic_data=True, micro_batch_size=args.micro_batch_size,
                            sequence_length=args.seq_len, total_train_steps=10_000, learning_rate=3e-4,
                            lr_scheduler_type="constant", warmup_steps=0, max_grad_norm=1.0, dtype="bfloat16",
                            num_hidden_layers=args.layers, weight_decay=0.1, betas=(0.9, 0.95),
                            fused_lm_head=bool(args.fused_head), optimizer_state_dtype=args.opt_state_dtype,
                            gemm_tuning=args.gemm_tuning)
    tr = Trainer(a)
    side = tr.model.side_stream
    variants = args.variants.split(",")
    times = {v: [] for v in variants}
    for _ in range(2):
        tr.train_step()
    for r in range(args.rounds):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            set_variant(tr, v, side)
            tr.train_step()  # settle the variant
            tr.optimizer.sync()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.train_step()
            tr.optimizer.sync()
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / args.steps * 1e3)
            print(f"round {r} {v}: {times[v][-1]:.2f} ms/step", flush=True)
    from scaletorch_amd.ops import grad as G

    for k, v in G._WGRAD_TIMES.items():
        print("wgrad tune", k[0], k[2], {a: round(b, 3) for a, b in v.items()}, "->",
              {0: "hipblaslt", 1: "hip 4-stage", 2: "hip 8-phase", 17: "hip 4-stage no split",
               18: "hip 8-phase no split", 3: "hipblaslt one-T", 4: "tuned hipblaslt",
               5: "tuned hipblaslt one-T", 6: "hip one-wave-per-SIMD"}.get(G._WGRAD_CHOICE.get(k), "?"))
    print(json.dumps({v: round(statistics.median(t), 2) for v, t in times.items()}))
    return 0


if __name__ == "__main__":
    sys.exit(main())

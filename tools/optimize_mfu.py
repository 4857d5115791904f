#!/usr/bin/env python3
"""Which of the framework's step-level optimisations buys what, on ONE trainer.

Reference: tools/optimize_mfu.py:44-91 (compares 4 strategies incl.
torch.compile on the NPU).  Here the strategies are this framework's own
switches, toggled at run time on one Llama trainer and timed in interleaved
blocks (tools/ab_step.py: device clocks differ by up to ~10 % between boxes, so
only same-process comparisons of few-% effects are meaningful):

  baseline      serial optimizer step after backward, hipBLASLt weight-gradient GEMMs
  +wgrad        + hand-written gfx950 weight-gradient GEMM (per-shape autotuned)
  +overlap      + optimizer / grad-norm on a side stream overlapped with fwd / bwd
  +gc           + activation checkpointing (memory for time: what GC costs)

  python tools/optimize_mfu.py --model llama3-8b --rounds 3 --steps 3
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STRATEGIES = {
    "baseline": dict(env={"ST_WGRAD_KERNEL": "0"}, overlap=False, gc=False),
    "+wgrad": dict(env={"ST_WGRAD_KERNEL": "1"}, overlap=False, gc=False),
    "+overlap": dict(env={"ST_WGRAD_KERNEL": "1"}, overlap=True, gc=False),
    "+gc": dict(env={"ST_WGRAD_KERNEL": "1"}, overlap=True, gc=True),
}


def apply(tr, name: str, side) -> None:
    s = STRATEGIES[name]
    os.environ.update(s["env"])
    st = side if s["overlap"] else None
    tr.optimizer.side_stream = st
    tr.model.side_stream = st
    for a in tr.model.arenas:
        a.side_stream = st
        a.sq_count = 0
    tr.args.gradient_checkpointing = s["gc"]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--strategies", default=",".join(STRATEGIES))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--micro_batch_size", type=int, default=2)
    ap.add_argument("--seq_len", type=int, default=4096)
    ap.add_argument("--layers", type=int, default=None)
    args = ap.parse_args()
    import torch

    from scaletorch_amd.trainer.config import ScaleTorchArguments
    from scaletorch_amd.trainer.engine import Trainer
    from scaletorch_amd.utils.misc import flops_per_token

    a = ScaleTorchArguments(model_name_or_path=args.model, synthetic_data=True, micro_batch_size=args.micro_batch_size,
                            sequence_length=args.seq_len, total_train_steps=10_000, learning_rate=3e-4,
                            lr_scheduler_type="constant", warmup_steps=0, max_grad_norm=1.0, dtype="bfloat16",
                            num_hidden_layers=args.layers, weight_decay=0.1, betas=(0.9, 0.95))
    tr = Trainer(a)
    side = tr.model.side_stream
    names = args.strategies.split(",")
    times = {n: [] for n in names}
    tr.train_step()
    for r in range(args.rounds):
        for n in (names if r % 2 == 0 else names[::-1]):
            apply(tr, n, side)
            tr.train_step()
            tr.optimizer.sync()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.train_step()
            tr.optimizer.sync()
            torch.cuda.synchronize()
            times[n].append((time.perf_counter() - t0) / args.steps * 1e3)
    cfg = tr.model_config
    fpt = flops_per_token(cfg.active_params(), cfg.num_hidden_layers, cfg.num_attention_heads, cfg.head_dim,
                          args.seq_len)
    tok = args.micro_batch_size * args.seq_len
    out = {}
    for n in names:
        ms = statistics.median(times[n])
        out[n] = {"ms_per_step": round(ms, 2), "tokens_per_s": round(tok / ms * 1e3, 1),
                  "mfu_pct": round(tok / ms * 1e3 * fpt / 2.5e15 * 100, 2)}
        print(n, json.dumps(out[n]), flush=True)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())

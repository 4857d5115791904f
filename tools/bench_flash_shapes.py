#!/usr/bin/env python3
"""Flash attention forward / backward at the shapes that decide the BASELINE configs,
default kernels, one JSON line per (shape, pass):

* ``bench``: the Llama-3-8B bench layer (B6 S4096 H32/8 D128 causal), q/k/v as strided
  slices of one fused QKV buffer, exactly as the step calls them;
* ``cp8_32k_r{r}``: one rank of the cp8 @ 32K layout (zig-zag, all-gather CP): its two
  2048-query chunks (c = r and 15 - r) at their global offsets against the gathered
  K/V prefix [0, (c + 1) * 2048) -- the per-rank attention of that BASELINE config.

FLOPs count only the visible (causal) score entries: fwd 4 * d per entry, bwd 10 * d
(recompute S + dP + dV + dK + dQ; reference ring attention: context_parallel.py:266-364).

  python tools/bench_flash_shapes.py [--shapes bench,cp8_32k_r3] [--iters 10] [--no-bwd]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd import ops  # noqa: E402
from scaletorch_amd.ops import _lib  # noqa: E402

H, HKV, D = 32, 8, 128


def visible(sq: int, sk: int, q_off: int, k_off: int) -> int:
    """Count of (query, key) pairs with key_global <= query_global."""
    tot = 0
    for i in range(sq):
        n = q_off + i - k_off + 1
        tot += max(0, min(n, sk))
    return tot


def shape_calls(name: str):
    """[(B, Sq, Sk, q_off, k_off)] attention calls of one shape."""
    if name == "bench":
        return [(6, 4096, 4096, 0, 0)]
    if name.startswith("cp8_32k_r"):
        r, c = int(name.rsplit("r", 1)[1]), 2048
        return [(1, c, (ch + 1) * c, ch * c, 0) for ch in (r, 15 - r)]
    raise ValueError(name)


def run(name: str, iters: int, bwd: bool):
    calls = []
    g = torch.Generator(device="cuda").manual_seed(0)
    for B, Sq, Sk, qo, ko in shape_calls(name):
        qb = torch.randn(B, Sq, H + 2 * HKV, D, device="cuda", dtype=torch.bfloat16, generator=g)
        kv = torch.randn(B, Sk, H + 2 * HKV, D, device="cuda", dtype=torch.bfloat16, generator=g)
        q = qb[:, :, :H]
        k, v = kv[:, :, H:H + HKV], kv[:, :, H + HKV:]
        calls.append((q, k, v, qo, ko, visible(Sq, Sk, qo, ko) * B * H))
    scale = 1 / math.sqrt(D)
    outs = [ops.flash_attn_fwd(q, k, v, scale, True, qo, ko) for q, k, v, qo, ko, _ in calls]
    douts = [torch.randn_like(o) for o, _ in outs]
    pairs = sum(c[-1] for c in calls)

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / iters

    def fwd():
        for q, k, v, qo, ko, _ in calls:
            ops.flash_attn_fwd(q, k, v, scale, True, qo, ko)

    def bwd_():
        for (q, k, v, qo, ko, _), (o, lse), do in zip(calls, outs, douts):
            ops.flash_attn_bwd(do, q, k, v, o, lse, scale, True, qo, ko)

    res = []
    t = timeit(fwd)
    res.append(dict(shape=name, pass_="fwd", ms=round(t, 4), tflops=round(4 * D * pairs / t / 1e9, 1)))
    if bwd:
        t = timeit(bwd_)
        res.append(dict(shape=name, pass_="bwd", ms=round(t, 4), tflops=round(10 * D * pairs / t / 1e9, 1)))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="bench,cp8_32k_r0,cp8_32k_r3")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-bwd", action="store_true")
    a = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    for s in a.shapes.split(","):
        for r in run(s, a.iters, not a.no_bwd):
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

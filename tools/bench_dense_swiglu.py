#!/usr/bin/env python3
"""Dense gate|up projection + SwiGLU at the Llama-3-8B bench shape (T = 6 x 4096 tokens,
h = 4096, 2I = 28672): the current path (hipBLASLt GEMM -> gu, then the SwiGLU kernel
reading gu back) vs csrc/grouped_gemm.hip at G = 1 with the SwiGLU epilogue (gu and
a = silu(g) * u written by the GEMM itself).  Prints one JSON object.

  python tools/bench_dense_swiglu.py [--tokens 24576]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from scaletorch_amd import ops  # noqa: E402
from scaletorch_amd.ops import _lib  # noqa: E402
from scaletorch_amd.utils import gemm_tuning  # noqa: E402


def _time(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    args = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    mode = gemm_tuning.configure("auto")
    T, h, I = args.tokens, args.hidden, args.inter
    x = torch.randn(T, h, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(2 * I, h, device="cuda") * 0.02).to(torch.bfloat16)
    offs = torch.tensor([T], device="cuda", dtype=torch.int32)
    flops = 2.0 * T * h * 2 * I

    def current():
        gu = torch.nn.functional.linear(x, w)
        return gu, ops.swiglu(gu)

    def fused():
        return _lib.ops().grouped_gemm_swiglu(x, w.unsqueeze(0), offs)

    gu_r, a_r = current()
    out = fused()
    assert out, "grouped_gemm_swiglu did not take the shape"
    gu_f, a_f = out
    rel = lambda a, b: float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))  # noqa: E731
    res = {"shape": dict(T=T, h=h, I=I), "gemm_tuning": mode,
           "gu_rel_err": round(rel(gu_f, gu_r), 5), "a_rel_err": round(rel(a_f, a_r), 5)}
    gemm_only = _time(lambda: torch.nn.functional.linear(x, w))
    t_cur = min(_time(current) for _ in range(3))
    t_fused = min(_time(fused) for _ in range(3))
    res.update(gemm_ms=round(gemm_only, 3), gemm_tflops=round(flops / gemm_only / 1e9, 1),
               current_ms=round(t_cur, 3), fused_ms=round(t_fused, 3),
               fused_tflops=round(flops / t_fused / 1e9, 1), fused_vs_current=round(t_cur / t_fused, 3))
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())

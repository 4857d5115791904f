#!/usr/bin/env python3
"""Weight-gradient layouts on Llama-3-8B shapes (T = 24576 tokens, fp32 output):
ours (csrc/wgrad_gemm.hip, both operands token-major) vs hipBLASLt NT (same operands) vs
hipBLASLt with ONE operand made K(token)-contiguous by a transpose (the smaller one),
transpose cost reported separately.  TF/s on random operands.

  python tools/bench_wgrad_layouts.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from scaletorch_amd.ops import _lib  # noqa: E402

T = int(os.environ.get("WG_T", "24576"))
SHAPES = [("qkv", 6144, 4096), ("out", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]


def timeit(fn, iters=6):
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
    assert _lib.load(), _lib.load_error()
    res = {}
    for name, M, N in SHAPES:
        dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        out = torch.zeros(M, N, device="cuda")
        flops = 2.0 * T * M * N
        small_x = N <= M
        xt = x.t().contiguous() if small_x else None
        dyt = None if small_x else dy.t().contiguous()
        arms = {
            "ours": lambda: _lib.ops().wgrad_gemm_(out, dy, x, 0, 0),
            "hipblaslt_NT": lambda: torch.ops.aten.addmm.dtype_out(out, dy.t(), x, torch.float32, beta=0, alpha=1,
                                                                  out=out),
        }
        if small_x:  # C = dY^T (X^T)^T: B K-contiguous
            arms["hipblaslt_one_T"] = lambda: torch.ops.aten.addmm.dtype_out(out, dy.t(), xt.t(), torch.float32,
                                                                             beta=0, alpha=1, out=out)
            tr = lambda: _lib.ops().transpose_(x, xt)  # noqa: E731
        else:  # A K-contiguous
            arms["hipblaslt_one_T"] = lambda: torch.ops.aten.addmm.dtype_out(out, dyt, x, torch.float32, beta=0,
                                                                             alpha=1, out=out)
            tr = lambda: _lib.ops().transpose_(dy, dyt)  # noqa: E731
        # both operands token-contiguous (what producer-written transposed copies would give)
        dyt2 = dy.t().contiguous()
        xt2 = x.t().contiguous()
        arms["hipblaslt_TN"] = lambda: torch.ops.aten.addmm.dtype_out(out, dyt2, xt2.t(), torch.float32, beta=1,
                                                                    alpha=1, out=out)
        arms["tuned_TN"] = lambda: _lib.ops().gemm_(out, dyt2, xt2, False, True, 1.0, 1.0)
        arms["tuned_TN_beta0"] = lambda: _lib.ops().gemm_(out, dyt2, xt2, False, True, 1.0, 0.0)
        arms["ours_8phase"] = lambda: _lib.ops().wgrad_gemm_(out, dy, x, 1, 2)
        r = {}
        for arm, fn in arms.items():
            ms = min(timeit(fn) for _ in range(3))
            r[arm] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}
        r["transpose_ms"] = round(min(timeit(tr) for _ in range(3)), 4)
        res[name] = r
        print(name, json.dumps(r), flush=True)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())

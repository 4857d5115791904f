#!/usr/bin/env python3
"""One-wave-per-SIMD TN GEMM (csrc/gemm4w.hip) vs hipBLASLt (torch, TN on K-contiguous operands)
vs the 8-phase grouped kernel: correctness (rel. error vs fp32) and TF/s on the Llama-3-8B
projection shapes (T = 24,576 rows) and the Mixtral expert shapes (8 x 2,048 rows).

  python tools/bench_gemm4w.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
SHAPES = [  # name, G, rows per group, K, N  (y = x w^T, w [G, N, K])
    ("llama_qkv_fwd", 1, 24576, 4096, 6144),
    ("llama_o_fwd", 1, 24576, 4096, 4096),
    ("llama_gate_up_fwd", 1, 24576, 4096, 28672),
    ("llama_down_fwd", 1, 24576, 14336, 4096),
    ("llama_gate_up_dgrad_TN", 1, 24576, 28672, 4096),
    ("mixtral_gate_up_fwd", 8, 2048, 4096, 28672),
    ("mixtral_down_fwd", 8, 2048, 14336, 4096),
]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


out = {}
for name, G, rows, K, N in SHAPES:
    T = G * rows
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(G, N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    offs = torch.arange(1, G + 1, device="cuda", dtype=torch.int32) * rows
    y = _lib.ops().gemm4w(x, w, offs)
    ref = torch.cat([x[g * rows:(g + 1) * rows].float() @ w[g].float().t() for g in range(G)])
    err = float((y.float() - ref).norm() / ref.norm())
    flops = 2.0 * T * K * N
    arms = {"gemm4w": lambda: _lib.ops().gemm4w(x, w, offs),
            "grouped8": lambda: _lib.ops().grouped_gemm(x, w, offs, False)}
    if G == 1:
        arms["hipblaslt"] = lambda: torch.nn.functional.linear(x, w[0])
    res = {"rel_err": round(err, 5)}
    for arm, fn in arms.items():
        ms = min(timeit(fn) for _ in range(3))
        res[arm] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}
    out[name] = res
    print(name, json.dumps(res), flush=True)
print(json.dumps(out))

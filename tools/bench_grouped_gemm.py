#!/usr/bin/env python3
"""Grouped expert GEMM microbenchmark: csrc/grouped_gemm.hip (one launch, device offsets)
vs torch._grouped_mm (one hipBLASLt GEMM per expert on ROCm) vs a dense hipBLASLt GEMM of
the same total rows (the ceiling), on MoE shapes; prints TF/s per arm.

  python tools/bench_grouped_gemm.py
"""
from __future__ import annotations

import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from scaletorch_amd.ops import _lib  # noqa: E402

SHAPES = [  # name, G, rows per expert, K, N, wn
    ("mixtral_gate_up_fwd", 8, 2048, 4096, 28672, False),
    ("mixtral_down_fwd", 8, 2048, 14336, 4096, False),
    ("mixtral_down_dgrad", 8, 2048, 4096, 14336, True),
    ("mixtral_gate_up_dgrad", 8, 2048, 28672, 4096, True),
    ("mixtral_1gpu_gate_up_fwd", 8, 1024, 4096, 28672, False),
    ("mixtral_1gpu_down_fwd", 8, 1024, 14336, 4096, False),
    ("qwen3moe_gate_up_fwd", 128, 512, 2048, 1536, False),
    ("qwen3moe_down_fwd", 128, 512, 768, 2048, False),
    ("qwen3moe_down_dgrad", 128, 512, 2048, 768, True),
    # dense Llama-3-8B data gradients at micro-batch 6 (G = 1): dX = dY W, W [out, in] = [K][N]
    ("llama_qkv_dgrad", 1, 24576, 6144, 4096, True),
    ("llama_out_dgrad", 1, 24576, 4096, 4096, True),
    ("llama_gate_up_dgrad", 1, 24576, 28672, 4096, True),
    ("llama_down_dgrad", 1, 24576, 4096, 14336, True),
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


def main() -> int:
    assert _lib.load(), _lib.load_error()
    out = {}
    for name, G, rows, K, N, wn in SHAPES:
        T = G * rows
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn((G, K, N) if wn else (G, N, K), device="cuda", dtype=torch.bfloat16) * 0.02
        offs = torch.arange(1, G + 1, device="cuda", dtype=torch.int32) * rows
        flops = 2.0 * T * K * N
        def two_phase(fn):  # the 2-phase kernel (ST_GMM_8PHASE=0, read per launch) for the A/B
            def run():
                os.environ["ST_GMM_8PHASE"] = "0"
                try:
                    return fn()
                finally:
                    os.environ.pop("ST_GMM_8PHASE", None)
            return run

        arms = {
            "hip_grouped": lambda: _lib.ops().grouped_gemm(x, w, offs, wn),
            "hip_grouped_2phase": two_phase(lambda: _lib.ops().grouped_gemm(x, w, offs, wn)),
            "torch_grouped_mm": lambda: torch._grouped_mm(x, w if wn else w.transpose(-2, -1), offs=offs),
            "dense_hipblaslt": lambda: torch.matmul(x, w[0] if wn else w[0].t()),
        }
        if not wn and N % 256 == 0 and K % 64 == 0:  # the one-wave-per-SIMD kernel (csrc/gemm4w.hip)
            def g4(order):
                def run():
                    os.environ["ST_GEMM4W_ORDER"] = order
                    try:
                        return _lib.ops().gemm4w(x, w, offs)
                    finally:
                        os.environ.pop("ST_GEMM4W_ORDER", None)
                return run
            arms["gemm4w_k5_o0"] = g4("0")
            arms["gemm4w_k5_o4"] = g4("4")
        if not wn and "gate_up" in name:  # SwiGLU epilogue: gu and a = silu(g) * u from the GEMM
            arms["hip_grouped_swiglu_epilogue"] = lambda: _lib.ops().grouped_gemm_swiglu(x, w, offs)
            arms["hip_grouped_swiglu_epilogue_2phase"] = two_phase(lambda: _lib.ops().grouped_gemm_swiglu(x, w, offs))
            arms["hip_grouped_then_swiglu"] = lambda: _lib.ops().swiglu_fwd(_lib.ops().grouped_gemm(x, w, offs, wn))
        if wn and G == 1:  # the TN form on a transposed weight copy (what ops/grad.py runs today)
            wt = w[0].t().contiguous()
            arms["dense_hipblaslt_TN_on_WT_copy"] = lambda: torch.nn.functional.linear(x, wt)
        res = {}
        for arm, fn in arms.items():
            ms = min(timeit(fn) for _ in range(3))
            res[arm] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}
        out[name] = res
        print(name, json.dumps(res), flush=True)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())

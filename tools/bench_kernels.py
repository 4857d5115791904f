#!/usr/bin/env python3
"""Micro-benchmarks of the hot ops at Llama-3-8B training shapes on one MI355X.

Times (CUDA events, median of N) our HIP kernels and, for context only, the
vendor paths PyTorch ships (SDPA on ROCm, hipBLASLt GEMMs).  Prints one JSON
object; numbers feed docs/PERF.md.

  python tools/bench_kernels.py [--seq 4096] [--batch 2]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.realpath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


_ITERS = 20


def timeit(fn, iters=None, warmup=3):
    iters = min(iters or _ITERS, _ITERS)
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--only", default="")
    ap.add_argument("--blas", default="", help="torch BLAS backend for the reference GEMMs: hipblaslt | rocblas")
    ap.add_argument("--no-ref", action="store_true", help="skip the vendor reference paths (for counter runs)")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    global _ITERS
    _ITERS = args.iters
    from scaletorch_amd import ops
    from scaletorch_amd.ops import _lib

    assert _lib.load(), _lib.load_error()
    if args.blas:
        torch.backends.cuda.preferred_blas_library(args.blas)
    st = _lib.ops()
    B, S, H, Hkv, D, h, I = args.batch, args.seq, 32, 8, 128, 4096, 14336
    res = {"shape": dict(B=B, S=S, H=H, Hkv=Hkv, D=D)}
    dev = "cuda"
    torch.manual_seed(0)
    scale = 1 / math.sqrt(D)
    flop_mm = 2 * B * H * S * S * D / 2  # one causal QK^T-sized product
    if not args.only or "attn" in args.only:
        q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16)
        k = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
        out, lse = st.flash_fwd(q, k, v, scale, True, 0, 0)
        do = torch.randn_like(out)
        t = timeit(lambda: st.flash_fwd(q, k, v, scale, True, 0, 0))
        res["flash_fwd_ms"] = t
        res["flash_fwd_tflops"] = 2 * flop_mm / t / 1e9
        t = timeit(lambda: st.flash_bwd(do, q, k, v, out, lse, scale, True, 0, 0, None, None, None))
        res["flash_bwd_ms"] = t
        res["flash_bwd_tflops_5mm"] = 5 * flop_mm / t / 1e9
        # vendor SDPA for context (expanded GQA as the reference does)
        qt = None if args.no_ref else q.transpose(1, 2)
        kt = k.transpose(1, 2).repeat_interleave(H // Hkv, 1)
        vt = v.transpose(1, 2).repeat_interleave(H // Hkv, 1)
        try:
            if qt is None:
                raise RuntimeError("skipped (--no-ref)")
            t = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=True))
            res["torch_sdpa_fwd_ms"] = t
            qr, kr, vr = (x.detach().requires_grad_(True) for x in (qt, kt, vt))
            o = F.scaled_dot_product_attention(qr, kr, vr, is_causal=True)
            g = torch.randn_like(o)
            t2 = timeit(lambda: torch.autograd.grad(o, (qr, kr, vr), g, retain_graph=True))
            res["torch_sdpa_bwd_ms"] = t2
        except Exception as e:  # pragma: no cover
            res["torch_sdpa_error"] = str(e)[:200]
    if not args.only or "gemm" in args.only:
        N = B * S
        x = torch.randn(N, h, device=dev, dtype=torch.bfloat16)
        for name, (o_, i_) in {"qkv": (6144, h), "out": (h, h), "gate_up": (2 * I, h), "down": (h, I),
                               "lm_head": (128256, h)}.items():
            w = torch.randn(o_, i_, device=dev, dtype=torch.bfloat16)
            xi = torch.randn(N, i_, device=dev, dtype=torch.bfloat16)
            t = timeit(lambda: F.linear(xi, w))
            res[f"gemm_{name}_fwd_tflops"] = 2 * N * o_ * i_ / t / 1e9
            dy = torch.randn(N, o_, device=dev, dtype=torch.bfloat16)
            t = timeit(lambda: dy.t().mm(xi))
            res[f"gemm_{name}_wgrad_tflops"] = 2 * N * o_ * i_ / t / 1e9
            mg = torch.zeros(o_, i_, device=dev, dtype=torch.float32)
            try:
                t = timeit(lambda: torch.ops.aten.addmm.dtype_out(mg, dy.t(), xi, torch.float32, beta=1, alpha=1,
                                                                 out=mg))
                res[f"gemm_{name}_wgrad_fp32acc_tflops"] = 2 * N * o_ * i_ / t / 1e9
            except Exception as e:
                res["addmm_dtype_error"] = str(e)[:200]
            t = timeit(lambda: mg.add_(dy.t().mm(xi)))
            res[f"gemm_{name}_wgrad_plus_add_tflops"] = 2 * N * o_ * i_ / t / 1e9
    if not args.only or "tgemm" in args.only:
        # autotuned hipBLASLt (st_amd.gemm_) vs torch's default solution, same problems
        N = B * S
        for name, (o_, i_) in {"qkv": (6144, h), "out": (h, h), "gate_up": (2 * I, h), "down": (h, I),
                               "lm_head": (128256, h)}.items():
            w = torch.randn(o_, i_, device=dev, dtype=torch.bfloat16)
            xi = torch.randn(N, i_, device=dev, dtype=torch.bfloat16)
            dy = torch.randn(N, o_, device=dev, dtype=torch.bfloat16)
            fl = 2 * N * o_ * i_ / 1e9
            y = torch.empty(N, o_, device=dev, dtype=torch.bfloat16)
            st.gemm_(y, xi, w, False, True, 1.0, 0.0)
            res[f"tg_{name}_fwd_err"] = ((y.float() - F.linear(xi, w).float()).norm() / y.float().norm()).item()
            res[f"tg_{name}_fwd_tflops"] = fl / timeit(lambda: st.gemm_(y, xi, w, False, True, 1.0, 0.0))
            res[f"torch_{name}_fwd_tflops"] = fl / timeit(lambda: F.linear(xi, w))
            dx = torch.empty(N, i_, device=dev, dtype=torch.bfloat16)
            res[f"tg_{name}_dgrad_tflops"] = fl / timeit(lambda: st.gemm_(dx, dy, w, False, False, 1.0, 0.0))
            res[f"torch_{name}_dgrad_tflops"] = fl / timeit(lambda: dy.mm(w))
            mg = torch.zeros(o_, i_, device=dev, dtype=torch.float32)
            st.gemm_(mg, dy, xi, True, False, 1.0, 1.0)
            res[f"tg_{name}_wgrad_err"] = ((mg - dy.float().t() @ xi.float()).norm() / mg.norm()).item()
            res[f"tg_{name}_wgrad_fp32acc_tflops"] = fl / timeit(lambda: st.gemm_(mg, dy, xi, True, False, 1.0, 1.0))
            res[f"torch_{name}_wgrad_fp32acc_tflops"] = fl / timeit(
                lambda: torch.ops.aten.addmm.dtype_out(mg, dy.t(), xi, torch.float32, beta=1, alpha=1, out=mg))
            # same product with token-contiguous (pre-transposed) operands: the fwd-like layout
            dyT, xT = dy.t().contiguous(), xi.t().contiguous()
            res[f"tg_{name}_wgradT_fp32acc_tflops"] = fl / timeit(
                lambda: st.gemm_(mg, dyT, xT, False, True, 1.0, 1.0))
            res[f"transpose_{name}_ms"] = timeit(lambda: (dy.t().contiguous(), xi.t().contiguous()))
            del w, xi, dy, y, dx, mg, dyT, xT
        rep = st.gemm_tuning_report()
        res["tuning"] = [rep[i:i + 7] for i in range(0, len(rep), 7)]
    if not args.only or "elt" in args.only:
        N = B * S
        x = torch.randn(N, h, device=dev, dtype=torch.bfloat16)
        r = torch.randn_like(x)
        w = torch.ones(h, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: st.rmsnorm_fwd(x, r, w, 1e-5))
        res["rmsnorm_add_fwd_GBps"] = 4 * x.numel() * 2 / t / 1e6
        y, rstd, s = st.rmsnorm_fwd(x, r, w, 1e-5)
        dw = torch.zeros(h, device=dev)
        t = timeit(lambda: st.rmsnorm_bwd(x, s, w, rstd, r, dw))
        res["rmsnorm_bwd_GBps"] = 4 * x.numel() * 2 / t / 1e6
        gu = torch.randn(N, 2 * I, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: st.swiglu_fwd(gu))
        res["swiglu_fwd_GBps"] = 3 * N * I * 2 / t / 1e6
        do = torch.randn(N, I, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: st.swiglu_bwd(do, gu))
        res["swiglu_bwd_GBps"] = 5 * N * I * 2 / t / 1e6
        n = 1 << 28
        m = torch.zeros(n, device=dev)
        vv = torch.zeros(n, device=dev)
        mw = torch.randn(n, device=dev)
        g = torch.randn(n, device=dev)
        p = torch.zeros(n, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: st.adamw_step_(mw, m, vv, g, p, None, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1), iters=5)
        res["adamw_GBps"] = n * 30 / t / 1e6
        logits = torch.randn(N, 128256, device=dev, dtype=torch.bfloat16)
        tgt = torch.randint(0, 128256, (N,), device=dev)
        t = timeit(lambda: st.xent_fwd(logits, tgt, 0), iters=5)
        res["xent_fwd_GBps"] = logits.numel() * 2 / t / 1e6
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Weight-gradient GEMM: hand-written gfx950 kernel (csrc/wgrad_gemm.hip) vs the
hipBLASLt fp32-epilogue GEMM (aten::addmm.dtype_out) on the Llama-3-8B shapes
(T = micro-batch x seq tokens).  Same process, interleaved, random operands."""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (M = out features, N = in features)
    "qkv": (6144, 4096), "out": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
    "lm_head": (128256, 4096),
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import torch

    from scaletorch_amd.ops import _lib

    assert _lib.load(), _lib.load_error()
    T = args.tokens
    res = {}
    for name, (M, N) in SHAPES.items():
        if args.only and name not in args.only.split(","):
            continue
        dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        out0 = torch.zeros(M, N, device="cuda")
        out1 = torch.zeros(M, N, device="cuda")
        ok = _lib.ops().wgrad_gemm_(out0, dy, x, 0)
        torch.ops.aten.addmm.dtype_out(out1, dy.t(), x, torch.float32, beta=0, alpha=1, out=out1)
        err = ((out0 - out1).norm() / out1.norm()).item() if ok else None

        def t_ours():
            _lib.ops().wgrad_gemm_(out0, dy, x, 1)

        def t_p8():
            os.environ["ST_WGRAD_P8"] = "1"
            _lib.ops().wgrad_gemm_(out0, dy, x, 1)
            os.environ["ST_WGRAD_P8"] = "0"

        os.environ["ST_WGRAD_P8"] = "1"
        out2 = torch.zeros(M, N, device="cuda")
        ok8 = _lib.ops().wgrad_gemm_(out2, dy, x, 0)
        os.environ["ST_WGRAD_P8"] = "0"
        err8 = ((out2 - out1).norm() / out1.norm()).item() if ok8 else None
        del out2

        def t_blas():
            torch.ops.aten.addmm.dtype_out(out1, dy.t(), x, torch.float32, beta=1, alpha=1, out=out1)

        fl = 2.0 * T * M * N
        times = {"ours": [], "p8": [], "hipblaslt": []}
        for _ in range(3):
            for k, fn in (("ours", t_ours), ("p8", t_p8), ("hipblaslt", t_blas)):
                if k == "ours" and not ok:
                    continue
                fn()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                for _ in range(args.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[k].append(s.elapsed_time(e) / args.iters)
        row = {"M": M, "N": N, "T": T, "rel_err": err, "rel_err_p8": err8}
        for k, v in times.items():
            if v:
                ms = min(v)
                row[f"{k}_ms"] = round(ms, 4)
                row[f"{k}_tflops"] = round(fl / ms / 1e9, 1)
        res[name] = row
        print(name, json.dumps(row), flush=True)
        del dy, x, out0, out1
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())

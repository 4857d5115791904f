"""Weight-gradient GEMM: tail split on/off vs hipBLASLt on the Llama-3-8B projection
shapes (and their TP=2 shards) at the bench's token count.

    python tools/bench_wgrad_split.py [--tokens 24576] [--iters 10]

Prints one JSON line per shape: TF/s of the 4-stage (v1) and 8-phase (v2) kernels with
ST_WGRAD_SPLIT=0 / auto, and hipBLASLt's fp32-out addmm.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from scaletorch_amd.ops import _lib  # noqa: E402

SHAPES = {  # name: (M = out features, N = in features)
    "qkv": (6144, 4096), "out": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
    "qkv_tp2": (3072, 4096), "out_tp2": (4096, 2048), "gate_up_tp2": (14336, 4096), "down_tp2": (4096, 7168),
}


def timeit(fn, iters):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    T = args.tokens
    for name, (M, N) in SHAPES.items():
        if args.only and name not in args.only.split(","):
            continue
        dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        out = torch.zeros(M, N, device="cuda")
        flops = 2.0 * T * M * N
        res = {"shape": name, "M": M, "N": N, "T": T}
        for rnd in range(3):
            for v in (1, 2):
                for sp in ("0", "auto"):
                    if sp == "auto":
                        os.environ.pop("ST_WGRAD_SPLIT", None)
                    else:
                        os.environ["ST_WGRAD_SPLIT"] = sp
                    if not _lib.ops().wgrad_gemm_(out, dy, x, 1, v):
                        continue
                    ms = timeit(lambda: _lib.ops().wgrad_gemm_(out, dy, x, 1, v), args.iters)
                    k = f"v{v}_split_{sp}"
                    res[k] = max(res.get(k, 0.0), round(flops / ms / 1e9, 1))
            os.environ.pop("ST_WGRAD_SPLIT", None)
            ms = timeit(lambda: torch.ops.aten.addmm.dtype_out(out, dy.t(), x, torch.float32, beta=1, alpha=1,
                                                               out=out), args.iters)
            res["hipblaslt"] = max(res.get("hipblaslt", 0.0), round(flops / ms / 1e9, 1))
        print(json.dumps(res), flush=True)
        del dy, x, out


if __name__ == "__main__":
    main()

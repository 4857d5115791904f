#!/usr/bin/env python3
"""Data-gradient GEMM layout A/B on one MI355X (Llama-3-8B projection shapes).

dX = dY W with W row-major [out, in] is an NN GEMM for hipBLASLt; with a
K-contiguous copy W^T [in, out] it becomes the TN form F.linear(dY, W^T) the
forward pass runs.  Times both (interleaved rounds in one process, random
data), plus the cost of producing W^T with csrc/transpose.hip vs torch.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (6144, 4096), "out": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(fn, iters=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from scaletorch_amd.ops import _lib

    assert _lib.load(), _lib.load_error()
    T = args.tokens
    res = {}
    for name, (o, i) in SHAPES.items():
        W = torch.empty(o, i, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        dy = torch.empty(T, o, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        Wt = torch.empty(i, o, device="cuda", dtype=torch.bfloat16)
        _lib.ops().transpose_(W, Wt)
        assert torch.equal(Wt, W.t().contiguous()), name
        ref = dy.float() @ W.float() if o * i <= 6144 * 4096 else None
        a = dy.matmul(W)
        b = F.linear(dy, Wt)
        if ref is not None:
            ea = ((a.float() - ref).norm() / ref.norm()).item()
            eb = ((b.float() - ref).norm() / ref.norm()).item()
            assert eb < 1e-2, (name, eb)
            res[f"{name}_rel_err_nn_tn"] = [ea, eb]
        nn, tn, tr_ours, tr_torch = [], [], [], []
        for _ in range(args.rounds):
            nn.append(timeit(lambda: dy.matmul(W)))
            tn.append(timeit(lambda: F.linear(dy, Wt)))
            tr_ours.append(timeit(lambda: _lib.ops().transpose_(W, Wt)))
            tr_torch.append(timeit(lambda: W.t().contiguous()))
        fl = 2.0 * T * o * i
        m = statistics.median
        res[name] = dict(nn_ms=m(nn), tn_ms=m(tn), nn_tflops=fl / m(nn) / 1e9, tn_tflops=fl / m(tn) / 1e9,
                         transpose_ms=m(tr_ours), transpose_tbps=4 * o * i / m(tr_ours) / 1e9,
                         torch_transpose_ms=m(tr_torch))
        print(name, json.dumps(res[name]), flush=True)
        del W, dy, Wt, a, b
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

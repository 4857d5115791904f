"""Expert forward / data-gradient GEMMs: torch._grouped_mm (device offsets) vs one
hipBLASLt GEMM per expert (host-known counts), Mixtral-8x7B shapes, ragged counts.

    python tools/probe_expert_gemm.py [--tokens 16384]

Prints TF/s of x @ W_gu^T ([T,4096] x [E,28672,4096]) and h @ W_dn^T per path.
"""
from __future__ import annotations

import argparse
import json

import torch


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--experts", type=int, default=8)
    args = ap.parse_args()
    E, T, h, inter = args.experts, args.tokens, 4096, 14336
    g = torch.Generator().manual_seed(0)
    w = torch.rand(E, generator=g) + 0.5
    counts = (w / w.sum() * T).long()
    counts[-1] += T - counts.sum()
    cl = counts.tolist()
    offs = torch.cumsum(counts.to("cuda", torch.int32), 0, dtype=torch.int32)
    x = torch.randn(T, h, device="cuda", dtype=torch.bfloat16)
    hh = torch.randn(T, inter, device="cuda", dtype=torch.bfloat16)
    wgu = torch.randn(E, 2 * inter, h, device="cuda", dtype=torch.bfloat16) * 0.02
    wdn = torch.randn(E, h, inter, device="cuda", dtype=torch.bfloat16) * 0.02
    for name, a, wt, n_out in (("gate_up", x, wgu, 2 * inter), ("down", hh, wdn, h)):
        k = a.shape[1]
        flops = 2.0 * T * k * n_out

        def grouped():
            return torch._grouped_mm(a, wt.transpose(-2, -1), offs=offs)

        out = torch.empty(T, n_out, device="cuda", dtype=torch.bfloat16)

        def loop():
            o = 0
            for e, n in enumerate(cl):
                if n:
                    torch.mm(a[o:o + n], wt[e].t(), out=out[o:o + n])
                o += n
            return out

        ref = grouped()
        got = loop()
        err = ((ref.float() - got.float()).norm() / ref.float().norm()).item()
        res = {"gemm": name, "counts": cl, "rel_err": err}
        for k_, fn in (("grouped_mm", grouped), ("per_expert_mm", loop)):
            res[k_ + "_TFps"] = round(flops / timeit(fn) / 1e9, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

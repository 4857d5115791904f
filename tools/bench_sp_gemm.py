#!/usr/bin/env python3
"""Sequence-parallel GEMM pieces vs the unsplit GEMM at the tp2pp2dp2 preset shapes
(Llama-3-8B, tp 2, mbs 4, S 4096: shard Sp = 2048 in c = 2 sub-chunks of 1024).

The pipelined SP linears (parallel/tensor_parallel.py) cut each projection into
(peer, sub-chunk) pieces so the all-gather / reduce-scatter overlaps them.  This
times, per projection, (a) ONE GEMM over all B*S rows, (b) the round-3 split
(one [Sc, K] GEMM per batch element and piece) and (c) the round-4 split (one
[B*Sc, K] GEMM per piece over all B sequences, input gathered / output copied when
strided: ``_bmm_into`` "fold"), with no communication, and prints one JSON object
(rates in TFLOP/s and the ratios to (a)).
"""
from __future__ import annotations

import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

from scaletorch_amd.parallel.tensor_parallel import _bmm_into  # noqa: E402


def _time(fn, iters=20):
    for _ in range(3):
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
    dev = torch.device("cuda")
    B, S, ws, c = 4, 4096, 2, 2
    Sp, Sc = S // ws, S // ws // c
    h, I, kvh = 4096, 14336, 1024
    shapes = {  # name: (kind, K, N)
        "qkv_col": ("col", h, (h + 2 * kvh) // ws),
        "gate_up_col": ("col", h, 2 * I // ws),
        "o_row_fwd": ("row", h // ws, h),
        "down_row_fwd": ("row", I // ws, h),
        "o_row_dgrad": ("dgrad", h, h // ws),
        "down_row_dgrad": ("dgrad", h, I // ws),
    }
    out = {"config": dict(B=B, S=S, tp=ws, sub_chunks=c, Sp=Sp, Sc=Sc)}
    for name, (kind, K, N) in shapes.items():
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        wt = w.t()
        flops = 2.0 * B * S * K * N
        if kind == "col":
            x = torch.randn(B, Sp, K, device=dev, dtype=torch.bfloat16)          # own shard
            g = [torch.randn(ws * B, Sc, K, device=dev, dtype=torch.bfloat16) for _ in range(c)]  # gathered
            y = torch.empty(B, S, N, device=dev, dtype=torch.bfloat16)
            xf = torch.randn(B * S, K, device=dev, dtype=torch.bfloat16)
            yf = torch.empty(B * S, N, device=dev, dtype=torch.bfloat16)

            def unsplit():
                torch.matmul(xf, wt, out=yf)

            def run(mode):
                _bmm_into(x, wt, y[:, :Sp], mode)
                for q in range(c):
                    _bmm_into(g[q][B:2 * B], wt, y[:, Sp + q * Sc: Sp + (q + 1) * Sc], mode)
        elif kind == "row":
            x = torch.randn(B, S, K, device=dev, dtype=torch.bfloat16)
            bufs = [torch.empty(ws * B, Sc, N, device=dev, dtype=torch.bfloat16) for _ in range(c)]
            xf = x.view(B * S, K)
            yf = torch.empty(B * S, N, device=dev, dtype=torch.bfloat16)

            def unsplit():
                torch.matmul(xf, wt, out=yf)

            def run(mode):
                for q in range(c):
                    for j in range(ws):
                        _bmm_into(x[:, j * Sp + q * Sc: j * Sp + (q + 1) * Sc], wt, bufs[q][j * B:(j + 1) * B], mode)
        else:  # row backward: dX[B, S, K'] = dY W, own shard + gathered peer shard
            Kd, Nd = K, N  # dY [.., h] @ W [h, in/tp]
            wd = torch.randn(Kd, Nd, device=dev, dtype=torch.bfloat16) * 0.02  # = W [out, in] row-major
            wdt = wd.t().contiguous()  # the W^T copy
            b2 = wdt.t()
            dys = torch.randn(B, Sp, Kd, device=dev, dtype=torch.bfloat16)
            buf = torch.randn(ws * B, Sp, Kd, device=dev, dtype=torch.bfloat16)
            dx = torch.empty(B, S, Nd, device=dev, dtype=torch.bfloat16)
            xf = torch.randn(B * S, Kd, device=dev, dtype=torch.bfloat16)
            yf = torch.empty(B * S, Nd, device=dev, dtype=torch.bfloat16)
            flops = 2.0 * B * S * Kd * Nd

            def unsplit():
                torch.matmul(xf, b2, out=yf)

            def run(mode):
                _bmm_into(dys, b2, dx[:, :Sp], mode)
                _bmm_into(buf[B:2 * B], b2, dx[:, Sp:], mode)
        # correctness of the folded pieces against the per-element loop
        run("loop")
        torch.cuda.synchronize()
        ref = (y if kind == "col" else (torch.cat(bufs) if kind == "row" else dx)).clone()
        run("fold")
        torch.cuda.synchronize()
        got = y if kind == "col" else (torch.cat(bufs) if kind == "row" else dx)
        err = ((got.float() - ref.float()).norm() / ref.float().norm()).item()
        t = {k: _time(f) for k, f in (("unsplit", unsplit), ("per_element", lambda: run("loop")),
                                      ("folded", lambda: run("fold")))}
        out[name] = {k + "_tflops": round(flops / v / 1e9, 1) for k, v in t.items()}
        out[name]["folded_vs_unsplit"] = round(t["unsplit"] / t["folded"], 3)
        out[name]["per_element_vs_unsplit"] = round(t["unsplit"] / t["per_element"], 3)
        out[name]["rel_err_fold_vs_loop"] = err
        print(name, json.dumps(out[name]), flush=True)
    # the SP MLP in the gathered layout (tensor_parallel._SPMLPFn): every piece is a contiguous
    # 2-D GEMM -- gate|up over [B*Sc] rows per (q, own / peer block), down over [ws*B*Sc] per q
    I2, Il = 2 * I // ws, I // ws
    wgu = torch.randn(I2, h, device=dev, dtype=torch.bfloat16) * 0.02
    wdn = torch.randn(h, Il, device=dev, dtype=torch.bfloat16) * 0.02
    xg = torch.randn(c, ws, B * Sc, h, device=dev, dtype=torch.bfloat16)
    gu = torch.empty(c, ws, B * Sc, I2, device=dev, dtype=torch.bfloat16)
    a = torch.randn(c, ws * B * Sc, Il, device=dev, dtype=torch.bfloat16)
    rs = torch.empty(c, ws * B * Sc, h, device=dev, dtype=torch.bfloat16)
    xf = xg.view(-1, h)
    guf = torch.empty(B * S, I2, device=dev, dtype=torch.bfloat16)
    af = a.view(-1, Il)
    yf = torch.empty(B * S, h, device=dev, dtype=torch.bfloat16)

    def mlp_pieces():
        for q in range(c):
            torch.matmul(xg[q, 0], wgu.t(), out=gu[q, 0])            # own rows
            torch.matmul(xg[q, 1:].reshape(-1, h), wgu.t(), out=gu[q, 1:].view(-1, I2))  # peers
            torch.matmul(a[q], wdn.t(), out=rs[q])                    # down: one GEMM per sub-chunk

    def mlp_unsplit():
        torch.matmul(xf, wgu.t(), out=guf)
        torch.matmul(af, wdn.t(), out=yf)

    flops = 2.0 * B * S * h * (I2 + Il)
    t = {"unsplit": _time(mlp_unsplit), "gathered_layout": _time(mlp_pieces)}
    out["mlp_gathered_layout"] = {k + "_tflops": round(flops / v / 1e9, 1) for k, v in t.items()}
    out["mlp_gathered_layout"]["pieces_vs_unsplit"] = round(t["unsplit"] / t["gathered_layout"], 3)
    print("mlp_gathered_layout", json.dumps(out["mlp_gathered_layout"]), flush=True)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Mixtral EP8 expert FFN, op by op, at the rows one expert receives per micro-batch (G = 1):
every kernel this framework can run each of the six GEMMs on, in isolation, TF/s per arm.

The step chooses one kernel per op (models/moe.py ``_ExpertFFNFn``); this table is what the
choice rests on ("use the slice to decide the kernel per transport").

  python tools/bench_ep8_expert.py [--rows 8192,8544,16384]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from scaletorch_amd.models.moe import _gmm_tail_split  # noqa: E402
from scaletorch_amd.ops import _lib  # noqa: E402


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="8192,8544,16384")
    ap.add_argument("--ops", default="", help="comma list of ops to time (default all)")
    ap.add_argument("--h", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    a = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    ops = _lib.ops()
    h, I = a.h, a.inter
    torch.manual_seed(0)
    w_gu = torch.randn(1, 2 * I, h, device="cuda", dtype=torch.bfloat16) * 0.02
    w_dn = torch.randn(1, h, I, device="cuda", dtype=torch.bfloat16) * 0.02
    w_gu_t = w_gu[0].t().contiguous()  # [h, 2I]: TN dgrad on a transposed copy
    w_dn_t = w_dn[0].t().contiguous()  # [I, h]
    mg_gu = torch.zeros(1, 2 * I, h, device="cuda", dtype=torch.float32)
    mg_dn = torch.zeros(1, h, I, device="cuda", dtype=torch.float32)
    out = {}
    for R in [int(r) for r in a.rows.split(",")]:
        offs = torch.tensor([R], device="cuda", dtype=torch.int32)
        x = torch.randn(R, h, device="cuda", dtype=torch.bfloat16)
        gu = torch.randn(R, 2 * I, device="cuda", dtype=torch.bfloat16)
        act = torch.randn(R, I, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(R, h, device="cuda", dtype=torch.bfloat16)
        dgu = torch.randn(R, 2 * I, device="cuda", dtype=torch.bfloat16)
        f_gu, f_dn = 2.0 * R * h * 2 * I, 2.0 * R * h * I
        arms = {
            "gate_up_fwd": (f_gu, {
                "gemm4w_swiglu": lambda: ops.gemm4w_swiglu_grouped(x, w_gu, offs),
                "grouped_swiglu": lambda: ops.grouped_gemm_swiglu(x, w_gu, offs),
                "hipblaslt+swiglu": lambda: ops.swiglu_fwd(torch.matmul(x, w_gu[0].t()), offs),
                "hipblaslt": lambda: torch.matmul(x, w_gu[0].t()),
            }),
            "down_fwd": (f_dn, {
                "gemm4w": lambda: ops.gemm4w(act, w_dn, offs),
                "grouped": lambda: ops.grouped_gemm(act, w_dn, offs, False),
                "hipblaslt": lambda: torch.matmul(act, w_dn[0].t()),
                "bands+hipblaslt_tail": lambda: _gmm_tail_split(act, w_dn, offs, False, False),
            }),
            "down_dgrad_dswiglu": (f_dn, {
                "grouped_dswiglu": lambda: ops.grouped_gemm_dswiglu(dy, w_dn, offs, gu),
                "grouped+swiglu_bwd": lambda: ops.swiglu_bwd(ops.grouped_gemm(dy, w_dn, offs, True), gu, offs),
                "hipblaslt_NN+swiglu_bwd": lambda: ops.swiglu_bwd(torch.matmul(dy, w_dn[0]), gu, offs),
                "hipblaslt_TN_on_WT+swiglu_bwd": lambda: ops.swiglu_bwd(torch.nn.functional.linear(dy, w_dn_t), gu,
                                                                        offs),
            }),
            "gate_up_dgrad": (f_gu, {
                "grouped": lambda: ops.grouped_gemm(dgu, w_gu, offs, True),
                "hipblaslt_NN": lambda: torch.matmul(dgu, w_gu[0]),
                "hipblaslt_TN_on_WT": lambda: torch.nn.functional.linear(dgu, w_gu_t),
                "bands+hipblaslt_tail": lambda: _gmm_tail_split(dgu, w_gu, offs, True, False),
            }),
            "gate_up_wgrad_acc": (f_gu, {
                "wgrad4_grouped": lambda: ops.wgrad_grouped_(mg_gu, dgu, x, offs, 1),
                "hipblaslt_fp32": lambda: torch.ops.aten.addmm.dtype_out(mg_gu[0], dgu.t(), x, torch.float32,
                                                                         beta=1, alpha=1, out=mg_gu[0]),
            }),
            "down_wgrad_acc": (f_dn, {
                "wgrad4_grouped": lambda: ops.wgrad_grouped_(mg_dn, dy, act, offs, 1),
                "hipblaslt_fp32": lambda: torch.ops.aten.addmm.dtype_out(mg_dn[0], dy.t(), act, torch.float32,
                                                                         beta=1, alpha=1, out=mg_dn[0]),
            }),
        }
        res = {}
        for op, (flops, fns) in arms.items():
            if a.ops and op not in a.ops.split(","):
                continue
            r = {}
            for arm, fn in fns.items():
                try:
                    ms = min(timeit(fn) for _ in range(3))
                    r[arm] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}
                except Exception as e:  # noqa: BLE001 -- an arm the binding refuses is reported, not fatal
                    r[arm] = {"error": repr(e)[:120]}
            res[op] = r
            print(R, op, json.dumps(r), flush=True)
        out[R] = res
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())

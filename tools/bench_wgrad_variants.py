#!/usr/bin/env python3
"""Weight-gradient kernel variants on the Llama-3-8B projection shapes at mbs 6
(T = 24,576 tokens): 1 = the 4-stage kernel, 2 = the 8-phase kernel (+16: without the
tail split), against hipBLASLt.  Checks each against an fp32 product of the same bf16
operands, then times them interleaved in one process (csrc/wgrad_gemm.hip).  With
ST_WGRAD_PROBE=1/3/4 the 8-phase arms run the timing probes (no DMA / DMA never waited
for / DMA from an L2-hot tile; wrong results): profiles/r03/wgrad_ring.md."""
import os as _os; _os.environ.setdefault("ST_KERNEL_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "build", "variants", "probes.so"))  # noqa: E401,E702 -- timing probes exist only in the diagnostic library (python -m scaletorch_amd._build --probes)
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"qkv": (6144, 4096), "out": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import torch

    from scaletorch_amd.ops import _lib

    assert _lib.load(), _lib.load_error()
    ops = _lib.ops()
    T = args.tokens
    arms = {"four_stage": 1, "p8": 2, "p8_nosplit": 18}
    res = {}
    for name, (M, N) in SHAPES.items():
        if args.only and name not in args.only.split(","):
            continue
        torch.manual_seed(0)
        dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        ref = dy.float().t().mm(x.float())
        out = torch.zeros(M, N, device="cuda")
        row = {"M": M, "N": N, "T": T}

        def run(arm, beta):
            return ops.wgrad_gemm_(out, dy, x, beta, arms[arm])

        for arm in arms:
            ok = run(arm, 0)
            torch.cuda.synchronize()
            row[f"{arm}_err"] = ((out - ref).norm() / ref.norm()).item() if ok else None
        del ref
        times = {a: [] for a in arms}
        times["hipblaslt"] = []
        for _ in range(args.rounds):
            for arm in times:
                fn = ((lambda: torch.ops.aten.addmm.dtype_out(out, dy.t(), x, torch.float32, beta=1, alpha=1, out=out))
                      if arm == "hipblaslt" else (lambda arm=arm: run(arm, 1)))
                fn()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                for _ in range(args.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[arm].append(s.elapsed_time(e) / args.iters)
        fl = 2.0 * T * M * N
        for arm, v in times.items():
            ms = min(v)
            row[f"{arm}_ms"] = round(ms, 4)
            row[f"{arm}_tflops"] = round(fl / ms / 1e9, 1)
        res[name] = row
        print(name, json.dumps(row), flush=True)
        del dy, x, out
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())

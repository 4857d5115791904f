#!/usr/bin/env python3
"""Fused AdamW kernel alone (csrc/adamw.hip), 256 M parameters: fp32 vs bf16 moments (the bf16
ones with stochastic rounding), flat and W^T-writing variants; prints ms and effective TB/s
(bytes read + written per parameter: fp32 moments 30 / 32 with W^T, bf16 22 / 24).

  python tools/bench_adamw.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
st = _lib.ops()
R, C = 16384, 16384  # 268 M parameters, one weight
n = R * C
out = {}
for sd, nbytes in ((torch.float32, 30), (torch.bfloat16, 22)):
    w = torch.randn(n, device="cuda")
    m = torch.zeros(n, device="cuda", dtype=sd)
    v = torch.zeros(n, device="cuda", dtype=sd)
    g = torch.randn(n, device="cuda")
    p = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    wt = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    for name, fn, b in (("flat", lambda: st.adamw_step_(w, m, v, g, p, None, 1e-4, 0.9, 0.95, 1e-8, 0.1, 3), nbytes),
                        ("wt", lambda: st.adamw_wt_step_(w, m, v, g, p.view(R, C), wt, None, 1e-4, 0.9, 0.95, 1e-8,
                                                         0.1, 3), nbytes + 2)):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                fn()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) / 3)
        key = f"{'bf16' if sd == torch.bfloat16 else 'fp32'}_moments_{name}"
        out[key] = {"ms": round(best, 3), "TBps": round(n * b / best / 1e9, 2)}
        print(key, out[key], flush=True)
    del w, m, v, g, p, wt
    torch.cuda.empty_cache()
print(json.dumps(out))

"""Gradient-norm pass (csrc/adamw.hip sumsq_kernel) on one 470 MB fp32 bucket (the size the
headline step reduces, 66 per step) and a bf16 one: ms and TB/s, plus the value vs torch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load()
res = {}
for dt in (torch.float32, torch.bfloat16):
    g = torch.randn(117_440_512, device="cuda").to(dt)
    out = torch.zeros(1, device="cuda")
    best = 1e9
    for _ in range(5):
        _lib.ops().sumsq_(g, out)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            _lib.ops().sumsq_(g, out)
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / 10)
    out.zero_()
    _lib.ops().sumsq_(g, out)
    ref = g.float().pow(2).sum().item()
    res[str(dt)] = {"ms": round(best, 4), "tb_s": round(g.numel() * g.element_size() / best / 1e9, 2),
                    "rel_err": abs(out.item() - ref) / ref}
print(json.dumps(res))

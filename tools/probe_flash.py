#!/usr/bin/env python3
"""Flash-attention timing probes at the bench shape (B4 S4096 H32/8 D128, causal):
full forward + backward vs the VALU-skipped bwd probe (ST_FLASH_PROBE=1, wrong
results), interleaved in one process.  Run under rocprofv3 --kernel-trace --stats
for the per-kernel split."""
import os as _os; _os.environ.setdefault("ST_KERNEL_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "build", "variants", "probes.so"))  # noqa: E401,E702 -- timing probes exist only in the diagnostic library (python -m scaletorch_amd._build --probes)
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd import ops  # noqa: E402
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
B, S, H, Hkv, D = 4, 4096, 32, 8, 128
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
fl_fwd = 4 * B * H * S * S * D / 2
res = {}
for rnd in range(3 if len(sys.argv) <= 1 else 1):
    for arm in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("full", "probe_novalu")):
        os.environ["ST_FLASH_PROBE"] = "1" if "probe" in arm else "0"
        o = ops.flash_attn(q, k, v, causal=True)
        o.backward(g)
        torch.cuda.synchronize()
        s0, s1, e = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        s0.record()
        for _ in range(5):
            o = ops.flash_attn(q, k, v, causal=True)
        s1.record()
        for _ in range(5):
            torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
        e.record()
        torch.cuda.synchronize()
        fwd, bwd = s0.elapsed_time(s1) / 5, s1.elapsed_time(e) / 5
        r = res.setdefault(arm, {"fwd_ms": 1e9, "bwd_ms": 1e9})
        r["fwd_ms"], r["bwd_ms"] = min(r["fwd_ms"], fwd), min(r["bwd_ms"], bwd)
for arm, r in res.items():
    print(arm, f"fwd {r['fwd_ms']:.3f} ms ({fl_fwd / r['fwd_ms'] / 1e9:.0f} TF/s)  "
               f"bwd {r['bwd_ms']:.3f} ms ({2.5 * fl_fwd / r['bwd_ms'] / 1e9:.0f} TF/s 5-matmul)", flush=True)

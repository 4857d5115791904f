#!/usr/bin/env python3
"""Flash forward/backward at the bench shape on contiguous [B,S,H,D] q/k/v vs the
in-step layout (strided views into one fused QKV GEMM output [B,S,(H+2Hkv)*D])."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd import ops  # noqa: E402

B, S, H, Hkv, D = 4, 4096, 32, 8, 128
qkv = torch.randn(B, S, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
arms = {
    "contiguous": [t.contiguous() for t in (qkv[..., :H * D].view(B, S, H, D), qkv[..., H * D:(H + Hkv) * D].view(B, S, Hkv, D),
                                           qkv[..., (H + Hkv) * D:].view(B, S, Hkv, D))],
    "fused_qkv_views": [qkv[..., :H * D].view(B, S, H, D), qkv[..., H * D:(H + Hkv) * D].view(B, S, Hkv, D),
                        qkv[..., (H + Hkv) * D:].view(B, S, Hkv, D)],
}
g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
best = {}
for rnd in range(3):
    for name, (q, k, v) in arms.items():
        q, k, v = (t.detach().requires_grad_(True) for t in (q, k, v))
        o = ops.flash_attn(q, k, v, causal=True)
        torch.autograd.grad(o, (q, k, v), g)
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
        f, b = s0.elapsed_time(s1) / 5, s1.elapsed_time(e) / 5
        r = best.setdefault(name, [1e9, 1e9])
        best[name] = [min(r[0], f), min(r[1], b)]
for name, (f, b) in best.items():
    print(f"{name}: fwd {f:.3f} ms  bwd {b:.3f} ms", flush=True)

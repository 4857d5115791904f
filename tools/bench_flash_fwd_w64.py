"""Flash forward at the bench layer shape (Llama-3-8B mbs 6: B6 S4096 H32/8 D128 causal):
the default 4-wave kernel (32 queries per wave) vs flash_fwd_w64_kernel (ST_FLASH_FWD_W64=1,
64 queries per wave), each with the XCD-aware order on / off.  Interleaved rounds, best ms."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd import ops  # noqa: E402
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 6
S = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
H, Hkv, D = 32, 8, 128
torch.manual_seed(0)
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
scale = 1 / math.sqrt(D)
fl = 4 * B * H * S * S * D / 2
arms = {"w32_xcd": ("0", "1"), "w32": ("0", "0"), "w64_xcd": ("1", "1"), "w64": ("1", "0")}
best, outs = {}, {}
for rnd in range(5):
    for name, (w64, xcd) in arms.items():
        os.environ["ST_FLASH_FWD_W64"], os.environ["ST_FLASH_XCD"] = w64, xcd
        outs[name] = ops.flash_attn_fwd(q, k, v, scale, True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            ops.flash_attn_fwd(q, k, v, scale, True)
        e.record()
        e.synchronize()
        best[name] = min(best.get(name, 1e9), s.elapsed_time(e) / 5)
o0, l0 = outs["w32_xcd"]
o1, l1 = outs["w64_xcd"]
print(json.dumps({"shape": [B, S, H, Hkv, D], "ms": {k2: round(v2, 4) for k2, v2 in best.items()},
                  "tflops": {k2: round(fl / v2 / 1e9, 1) for k2, v2 in best.items()},
                  "rel_o_w64_vs_w32": ((o1.float() - o0.float()).norm() / o0.float().norm()).item(),
                  "max_dlse": (l1 - l0).abs().max().item()}))

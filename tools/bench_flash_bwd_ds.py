#!/usr/bin/env python3
"""Flash-attention backward A/B at the bench layer shape (Llama-3-8B, micro-batch 6:
B6 S4096 H32/8 D128, causal): the recompute dQ kernel beside dK/dV (ST_FLASH_BWD_DS=0,
concurrent streams; "recompute_serial": the same on one stream) vs the dS-materialising
backward (ST_FLASH_BWD_DS=1: dK/dV stores dS^T tiles, dQ = dS K from them).
PROBE_STORES=1 adds a timing arm with the dS stores skipped (wrong dQ).  Interleaved rounds in one process; prints one JSON
line with the best time per arm and the rel. difference of the two arms' gradients.

  python tools/bench_flash_bwd_ds.py [B] [S]
"""
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
out, lse = ops.flash_attn_fwd(q, k, v, scale, True)
dout = torch.randn_like(out)
fl_fwd = 4 * B * H * S * S * D / 2
arms = {"recompute": ("0", "1", "0"), "recompute_serial": ("0", "0", "0"), "ds": ("1", "1", "0")}
if os.environ.get("PROBE_STORES") == "1":  # dS path with the dK/dV kernel's dS stores skipped (wrong dQ)
    arms["ds_nostore_probe"] = ("1", "1", "2")
best, grads = {}, {}
for rnd in range(5):
    for name, (ds, conc, probe) in arms.items():
        os.environ["ST_FLASH_BWD_DS"], os.environ["ST_FLASH_BWD_CONCURRENT"] = ds, conc
        os.environ["ST_FLASH_PROBE"] = probe
        grads[name] = ops.flash_attn_bwd(dout, q, k, v, out, lse, scale, True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            ops.flash_attn_bwd(dout, q, k, v, out, lse, scale, True)
        e.record()
        e.synchronize()
        best[name] = min(best.get(name, 1e9), s.elapsed_time(e) / 5)


# forward at the same shape, interleaved: 2 query heads per workgroup (opt-in), 1 head
# (default), 1 head without the XCD-aware order (ST_FLASH_FWD_HP, ST_FLASH_XCD)
fwd = {}
for rnd in range(5):
    for xcd in ("1", "h1", "0"):
        os.environ["ST_FLASH_XCD"] = "0" if xcd == "0" else "1"
        os.environ["ST_FLASH_FWD_HP"] = "2" if xcd == "1" else "1"
        ops.flash_attn_fwd(q, k, v, scale, True)
        torch.cuda.synchronize()
        fs, fe = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fs.record()
        for _ in range(5):
            ops.flash_attn_fwd(q, k, v, scale, True)
        fe.record()
        fe.synchronize()
        fwd[xcd] = min(fwd.get(xcd, 1e9), fs.elapsed_time(fe) / 5)
os.environ["ST_FLASH_XCD"], os.environ["ST_FLASH_FWD_HP"] = "1", "1"
fwd_ms = fwd["h1"]


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


res = {"shape": [B, S, H, Hkv, D], "fwd_ms": round(fwd_ms, 4), "fwd_tflops": round(fl_fwd / fwd_ms / 1e9, 1),
       "fwd_ms_2heads": round(fwd["1"], 4), "fwd_ms_xcd_off": round(fwd["0"], 4),
       "bwd_ms": {k2: round(v2, 4) for k2, v2 in best.items()},
       "tflops_5matmul": {k2: round(2.5 * fl_fwd / v2 / 1e9, 1) for k2, v2 in best.items()},
       "rel_diff": {n: rel(a, b) for n, a, b in zip(("dq", "dk", "dv"), grads["ds"], grads["recompute"])}}
print(json.dumps(res), flush=True)

#!/usr/bin/env python3
"""CP backward per chunk shape: the dS-materialising two-phase path (flash_bwd_kv, dS^T
workspace, then dQ = dS K: flash_bwd_q_ds -- what parallel/context_parallel.py runs) vs the
one-shot backward (dK/dV + the recompute dQ kernel, no workspace) at the per-rank zig-zag
chunk shapes of cp8 @ 32K (Llama-3-8B: B 1, H 32 / 8, D 128; chunk c = S / 2cp queries at
global offset g0 against keys [0, g0 + c)).  Interleaved rounds in one process; one JSON
line per chunk shape with both times, the workspace bytes and the faster path.

  python tools/bench_cp_flash_bwd.py [S] [cp]
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
S = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
cp = int(sys.argv[2]) if len(sys.argv) > 2 else 8
B, H, Hkv, D = 1, 32, 8, 128
c = S // (2 * cp)
scale = 1 / math.sqrt(D)
torch.manual_seed(0)
k_all = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
v_all = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
offsets = sorted({r * c for r in range(cp)} | {(2 * cp - 1 - r) * c for r in range(cp)})
rows = []
for g0 in offsets:
    kend = g0 + c
    q = torch.randn(B, c, H, D, device="cuda", dtype=torch.bfloat16)
    k, v = k_all[:, :kend], v_all[:, :kend]
    out, lse = ops.flash_attn_fwd(q, k, v, scale, True, g0, 0)
    dout = torch.randn_like(out)

    def two_phase():
        dk, dv, ws = _lib.ops().flash_bwd_kv(dout, q, k, v, out, lse, scale, True, g0, 0)
        if ws.numel() == 0:
            return None
        dq = _lib.ops().flash_bwd_q_ds(q, k, ws, scale, True, g0, 0)
        return dq, dk, dv, ws.numel() * ws.element_size()

    def one_shot():
        os.environ["ST_FLASH_BWD_DS"] = "0"
        try:
            return ops.flash_attn_bwd(dout, q, k, v, out, lse, scale, True, g0, 0)
        finally:
            os.environ.pop("ST_FLASH_BWD_DS", None)

    probe = two_phase()
    if probe is None:
        rows.append({"q_offset": g0, "keys": kend, "two_phase": "declined"})
        print(json.dumps(rows[-1]), flush=True)
        continue
    ws_bytes = probe[3]
    ref = one_shot()
    err = max(float((a.float() - b.float()).norm() / (b.float().norm() + 1e-6)) for a, b in zip(probe[:3], ref))
    best = {}
    for _ in range(4):
        for name, fn in (("two_phase", two_phase), ("one_shot", one_shot)):
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                fn()
            e.record()
            e.synchronize()
            best[name] = min(best.get(name, 1e9), s.elapsed_time(e) / 3)
    rows.append({"q_offset": g0, "keys": kend, "queries": c, "ws_gb": round(ws_bytes / 1e9, 3),
                 "two_phase_ms": round(best["two_phase"], 4), "one_shot_ms": round(best["one_shot"], 4),
                 "faster": min(best, key=best.get), "rel_diff": round(err, 5)})
    print(json.dumps(rows[-1]), flush=True)
tot = {k: round(sum(r.get(k + "_ms", 0) for r in rows), 3) for k in ("two_phase", "one_shot")}
tot["best_per_shape"] = round(sum(min(r.get("two_phase_ms", 1e9), r.get("one_shot_ms", 1e9)) for r in rows
                                  if "one_shot_ms" in r), 3)
print(json.dumps({"S": S, "cp": cp, "chunk": c, "totals_ms": tot}))

#!/usr/bin/env python3
"""What the zig-zag reorder of the gathered K/V costs in the CP all-gather transport
(parallel/context_parallel.py ``_CPAttnFn``) at the cp8 @ 32K layout, next to the
attention work it serves.

The gathered [K|V] arrives in rank order; one ``index_select`` puts it in global
order (forward) and one puts dK/dV back (backward).  Splitting the gather by zig-zag
half instead would avoid both copies but cost two more flash launches and LSE merges
per chunk.  This prints one JSON object: the reorder time and the flash forward /
backward times of the two local query chunks of a cp = 8 rank (4K queries in two
2K chunks, keys up to 32K), per layer.
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from scaletorch_amd import ops  # noqa: E402
from scaletorch_amd.parallel.context_parallel import _global_order_index, zigzag_chunk_starts  # noqa: E402


def _time(fn, iters=10):
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
    S, cp, H, Hkv, D = 32768, 8, 32, 8, 128
    rank = 3  # a middle rank: chunk starts 6K and 26K
    dev = torch.device("cuda")
    kv = torch.randn(1, S, 2 * Hkv, D, device=dev, dtype=torch.bfloat16)
    idx = _global_order_index(S, cp, dev)
    t_reorder = _time(lambda: kv.index_select(1, idx))
    a, b, c = zigzag_chunk_starts(S, cp, rank)
    q = torch.randn(1, 2 * c, H, D, device=dev, dtype=torch.bfloat16)
    scale = D ** -0.5
    kf, vf = kv[:, :, :Hkv], kv[:, :, Hkv:]
    outs = []

    def fwd():
        outs.clear()
        for off, g0 in ((0, a), (c, b)):
            outs.append(ops.flash_attn_fwd(q[:, off:off + c], kf[:, :g0 + c], vf[:, :g0 + c], scale, True, g0, 0))

    t_fwd = _time(fwd)
    dout = torch.randn_like(q)

    def bwd():
        for (off, g0), (o, lse) in zip(((0, a), (c, b)), outs):
            ops.flash_attn_bwd(dout[:, off:off + c], q[:, off:off + c], kf[:, :g0 + c], vf[:, :g0 + c], o, lse,
                               scale, True, g0, 0)

    t_bwd = _time(bwd)
    res = {"shape": dict(S=S, cp=cp, H=H, Hkv=Hkv, D=D, rank=rank), "reorder_ms": round(t_reorder, 4),
           "reorder_GBps": round(2 * kv.numel() * 2 / t_reorder / 1e6, 1),
           "flash_fwd_ms": round(t_fwd, 3), "flash_bwd_ms": round(t_bwd, 3),
           "reorder_share_of_attention_pct": round(100 * 2 * t_reorder / (t_fwd + t_bwd), 2)}
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())

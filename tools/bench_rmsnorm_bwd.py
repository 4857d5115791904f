#!/usr/bin/env python3
"""RMSNorm (+ residual) backward at the Llama-3-8B bench shape (6 x 4096 rows, h 4096):
kernel time and HBM rate of csrc/rmsnorm.hip's backward.  The block cap is read once per
process (ST_RMSNORM_BWD_BLOCKS), so compare caps with one process each:

  for b in 256 512 1024; do ST_RMSNORM_BWD_BLOCKS=$b python tools/bench_rmsnorm_bwd.py; done
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from scaletorch_amd import ops  # noqa: E402
from scaletorch_amd.ops import _lib  # noqa: E402


def main() -> int:
    assert _lib.load(), _lib.load_error()
    rows, h = 6 * 4096, 4096
    x = torch.randn(rows, h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(rows, h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y, s = ops.add_rms_norm(x, r, w, 1e-5)
    gy, gs = torch.randn_like(y), torch.randn_like(s)

    def bwd():
        torch.autograd.grad((y, s), (x, w), (gy, gs), retain_graph=True)

    bwd()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        a.record()
        for _ in range(10):
            bwd()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / 10)
    nbytes = 4 * rows * h * 2  # dy, s, dres read + ds written (bf16)
    print(json.dumps({"blocks_cap": os.environ.get("ST_RMSNORM_BWD_BLOCKS", "default"),
                      "prefetch": os.environ.get("ST_RMSNORM_BWD_PF", "0"), "bwd_ms": round(best, 4),
                      "TBps_rows": round(nbytes / best / 1e9, 2)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""gemm4w kind 5 diagnostic build (ST_GEMM4W_PROBE=7): shader-cycle stamps per segment of the
steady-state K-tile step, averaged over every wave of every workgroup.
Segments: MFMA 0-BAR (sub-step 1 reads), the barrier wait, BAR-63 (DMA issue), 64-127 (sub-step 0
reads of the next tile + DMA).  The MFMA floor is 16 cycles per 16x16x32 MFMA."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load()
SHAPES = {"gate_up": (24576, 4096, 28672), "down": (24576, 14336, 4096), "qkv": (24576, 4096, 6144)}
os.environ["ST_GEMM4W_KIND"] = "5"
for name, (T, K, N) in SHAPES.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(1, N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    offs = torch.tensor([T], device="cuda", dtype=torch.int32)
    out = {}
    for order, sched in (("0", "0"), ("0", "4"), ("4", "4")):
        os.environ["ST_GEMM4W_ORDER"], os.environ["ST_GEMM4W_SCHED"] = order, sched
        os.environ["ST_GEMM4W_PROBE"] = "0"
        _lib.ops().gemm4w(x, w, offs)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            _lib.ops().gemm4w(x, w, offs)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / 3
        os.environ["ST_GEMM4W_PROBE"] = "7"
        y = _lib.ops().gemm4w(x, w, offs)
        torch.cuda.synchronize()
        yi = y.view(torch.int64)  # [T, N / 4]
        v = yi.view(T // 256, 256, N // 256, 64)[:, :4, :, :5].reshape(-1, 5).double()
        steps = v[:, 4].clamp(min=1)
        seg = (v[:, :4] / steps[:, None]).mean(0).tolist()
        out[f"s{sched}o{order}"] = {"ms": round(ms, 3), "tflops": round(2.0 * T * K * N / ms / 1e9, 1),
                            "cycles_per_step": {k: round(c, 1) for k, c in zip(
                                ("mfma0_to_bar", "barrier_wait", "bar_to_63", "mfma64_to_127"), seg)},
                            "total": round(sum(seg), 1), "mfma_floor": 128 * 16}
    os.environ["ST_GEMM4W_PROBE"] = "0"
    print(name, json.dumps(out), flush=True)

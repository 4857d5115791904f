"""wgrad4 diagnostic build (ST_WGRAD4_PROBE=7): shader-cycle stamps per segment of the steady-state
K-tile step (64 tokens, 128 16x16x32 MFMAs per wave: floor 2,048 cycles), averaged over every wave.
Segments: MFMA 0-20 (sub-step-1 reads + A-image release wait), the m=20 barrier, 20-63 (A DMAs),
the m=63 publish barrier (vmcnt + barrier), 63-127 (B DMAs + next tile's sub-step-0 reads)."""
import os as _os; _os.environ.setdefault("ST_KERNEL_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "build", "variants", "probes.so"))  # noqa: E401,E702 -- timing probes exist only in the diagnostic library (python -m scaletorch_amd._build --probes)
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load()
os.environ["ST_WGRAD4_SPLIT"] = "1"
SHAPES = {"o": (24576, 4096, 4096), "gate_up": (24576, 28672, 4096), "down": (24576, 4096, 14336)}
names = ("mfma0_20", "bar20_wait", "mfma20_63", "bar63_wait", "mfma63_127")
for (name, (T, M, N)), kd in [(it, kd) for it in SHAPES.items() for kd in ("0", "1")]:
    os.environ["ST_WGRAD4_KDESC"] = kd  # 1: per-K-tile descriptors (the ragged / grouped path)
    dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    out = torch.zeros(M, N, device="cuda")
    os.environ["ST_WGRAD4_PROBE"] = "0"
    _lib.ops().wgrad_gemm_(out, dy, x, 0, 6)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        _lib.ops().wgrad_gemm_(out, dy, x, 0, 6)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / 3
    os.environ["ST_WGRAD4_PROBE"] = "7"
    out.zero_()
    _lib.ops().wgrad_gemm_(out, dy, x, 0, 6)
    torch.cuda.synchronize()
    os.environ["ST_WGRAD4_PROBE"] = "0"
    v = out.view(torch.int64)[:1024, :6].double()  # rows 4 b + w, u64 words
    v = v[v[:, 5] > 0]
    per = (v[:, :5] / v[:, 5:6]).mean(0).tolist()
    print(f"{name} kdesc={kd}", json.dumps({"ms": round(ms, 3), "pflops": round(2.0 * T * M * N / ms / 1e12, 3),
                            "cycles_per_step": {k: round(c, 1) for k, c in zip(names, per)},
                            "total": round(sum(per), 1), "mfma_floor": 2048, "waves": int(v.shape[0])}), flush=True)
    del dy, x, out

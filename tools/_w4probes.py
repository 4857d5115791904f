"""wgrad4 timing probes (ST_WGRAD4_PROBE 1 / 2 / 3: the K-loop without its DMA / fragment reads /
barriers -- wrong results, timing only) vs the real kernel, Llama-3-8B wgrad shapes, no tail split."""
import os as _os; _os.environ.setdefault("ST_KERNEL_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "build", "variants", "probes.so"))  # noqa: E401,E702 -- timing probes exist only in the diagnostic library (python -m scaletorch_amd._build --probes)
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load()
os.environ["ST_WGRAD4_SPLIT"] = "1"
SHAPES = {"o": (24576, 4096, 4096), "gate_up": (24576, 28672, 4096)}
for name, (T, M, N) in SHAPES.items():
    dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    out = torch.zeros(M, N, device="cuda")
    res = {}
    for rnd in range(3):
        for pv in ("0", "1", "2", "3"):
            os.environ["ST_WGRAD4_PROBE"] = pv
            _lib.ops().wgrad_gemm_(out, dy, x, 0, 6)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                _lib.ops().wgrad_gemm_(out, dy, x, 0, 6)
            e.record()
            e.synchronize()
            res[pv] = min(res.get(pv, 1e9), s.elapsed_time(e) / 3)
    os.environ["ST_WGRAD4_PROBE"] = "0"
    fl = 2.0 * T * M * N
    print(name, json.dumps({{"0": "real", "1": "no_dma", "2": "no_reads", "3": "no_barriers"}[k]:
                            {"ms": round(v, 3), "pflops": round(fl / v / 1e12, 3)} for k, v in res.items()}), flush=True)
    del dy, x, out

"""Grouped (MoE expert) weight gradient: csrc/wgrad4.hip st_wgrad4_grouped (ST_WGRAD_GROUPED4=1)
vs csrc/wgrad_gemm.hip's 4-stage grouped kernel (=0), at the Mixtral 1-GPU proxy and Qwen3-30B-A3B
expert shapes with ragged per-expert counts (+-25 % around the mean).  Best ms per arm."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load()
SHAPES = [  # name, experts, mean rows per expert, M (dY features), N (X features)
    ("mixtral_gate_up_wgrad", 8, 4096, 28672, 4096),
    ("mixtral_down_wgrad", 8, 4096, 4096, 14336),
    ("qwen3moe_gate_up_wgrad", 128, 512, 1536, 2048),
    ("qwen3moe_down_wgrad", 128, 512, 2048, 768),
]
g = torch.Generator().manual_seed(0)
for name, G, rows, M, N in SHAPES:
    counts = (rows * (0.75 + 0.5 * torch.rand(G, generator=g))).int()
    T = int(counts.sum())
    offs = torch.cumsum(counts, 0, dtype=torch.int32).cuda()
    dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    out = torch.zeros(G, M, N, device="cuda")
    res, outs = {}, {}
    for rnd in range(3):
        for arm in ("1", "0"):
            os.environ["ST_WGRAD_GROUPED4"] = arm
            assert _lib.ops().wgrad_grouped_(out, dy, x, offs, 0)
            outs[arm] = out.clone()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                _lib.ops().wgrad_grouped_(out, dy, x, offs, 1)
            e.record()
            e.synchronize()
            res[arm] = min(res.get(arm, 1e9), s.elapsed_time(e) / 3)
    fl = 2.0 * T * M * N
    d = ((outs["1"] - outs["0"]).norm() / outs["0"].norm()).item()
    print(name, json.dumps({"wgrad4": {"ms": round(res["1"], 3), "pflops": round(fl / res["1"] / 1e12, 3)},
                            "4stage": {"ms": round(res["0"], 3), "pflops": round(fl / res["0"] / 1e12, 3)},
                            "rel_diff": d}), flush=True)
    del dy, x, out, outs

"""Flash-attention backward with the dK/dV query-range and dQ key-range splits off / auto on short grids
(the single-device Qwen3 rows of BASELINE.md) and on the Llama-3-8B bench shape.

    python tools/bench_flash_split.py

One JSON line per shape: backward ms with ST_FLASH_{DKDV,DQ}_SPLIT=1 (off) and unset (auto).
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from scaletorch_amd import ops  # noqa: E402
from scaletorch_amd.ops import _lib  # noqa: E402

SHAPES = [  # B, S, H, Hkv
    (2, 2048, 16, 8),   # Qwen3-0.6B mbs 2 x 2048
    (1, 2048, 16, 8),   # Qwen3-1.7B mbs 1 x 2048
    (1, 8192, 16, 8),   # Qwen3-0.6B / 1.7B 1 x 8192
    (1, 2048, 32, 8),   # Qwen3-4B 1 x 2048
    (4, 4096, 32, 8),   # Llama-3-8B bench shape (grid long enough: split stays off)
]


def main():
    assert _lib.load(), _lib.load_error()
    D = 128
    for B, S, H, Hkv in SHAPES:
        q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
        o = ops.flash_attn(q, k, v, causal=True)
        res = {"B": B, "S": S, "H": H, "Hkv": Hkv}
        grads = {}
        for _ in range(3):
            for arm in ("off", "auto"):
                for knob in ("ST_FLASH_DKDV_SPLIT", "ST_FLASH_DQ_SPLIT"):
                    if arm == "off":
                        os.environ[knob] = "1"
                    else:
                        os.environ.pop(knob, None)
                grads[arm] = torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                for _ in range(10):
                    torch.autograd.grad(o, (q, k, v), g, retain_graph=True)
                e.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(e) / 10
                res[f"bwd_ms_{arm}"] = round(min(res.get(f"bwd_ms_{arm}", 1e9), ms), 4)
        os.environ.pop("ST_FLASH_DKDV_SPLIT", None)
        os.environ.pop("ST_FLASH_DQ_SPLIT", None)
        # the splits change only the fp32 summation order of dQ / dK / dV
        res["max_abs_diff_dk"] = float((grads["off"][1].float() - grads["auto"][1].float()).abs().max())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""Weight-gradient GEMM arms at the Llama-3-8B wgrad shapes (T 24,576): csrc/wgrad4.hip (variant 6)
vs the 8-phase / 4-stage HIP kernels (2 / 1) and hipBLASLt (fp32 out, accumulate), and without the
tail split-K, plus a numerics check of variant 6 against fp32.  Prints ms and PF/s per arm (min over rounds)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load()
torch.manual_seed(0)
# numerics: beta 0 then beta 1 accumulate, several tiles per persistent workgroup
T, M, N = 512, 4096, 4352
dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
out = torch.full((M, N), 7.0, device="cuda")
assert _lib.ops().wgrad_gemm_(out, dy, x, 0, 6)
ref = dy.float().t() @ x.float()
e0 = ((out - ref).norm() / ref.norm()).item()
assert _lib.ops().wgrad_gemm_(out, dy, x, 1, 6)
e1 = ((out - 2 * ref).norm() / (2 * ref).norm()).item()
print("numerics", json.dumps({"rel_err_beta0": e0, "rel_err_beta1": e1}), flush=True)
for rs in ("1",):  # spread-read schedule (ST_WGRAD4_RS)
    os.environ["ST_WGRAD4_RS"] = rs
    out.fill_(7.0)
    assert _lib.ops().wgrad_gemm_(out, dy, x, 0, 6)
    r0 = ((out - ref).norm() / ref.norm()).item()
    assert _lib.ops().wgrad_gemm_(out, dy, x, 1, 6)
    r1 = ((out - 2 * ref).norm() / (2 * ref).norm()).item()
    os.environ.pop("ST_WGRAD4_RS")
    print(f"numerics rs={rs}", json.dumps({"rel_err_beta0": r0, "rel_err_beta1": r1}), flush=True)
    assert r0 < 1e-5 and r1 < 1e-5

ORDERS = [o for o in os.environ.get("W4_ORDERS", "").split(",") if o]  # XCD-grouped tile orders to time
SHAPES = {"qkv": (24576, 6144, 4096), "o": (24576, 4096, 4096), "gate_up": (24576, 28672, 4096),
          "down": (24576, 4096, 14336), "lm_head_chunk": (4096, 128256, 4096)}
for name, (T, M, N) in SHAPES.items():
    dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    out = torch.zeros(M, N, device="cuda")
    arms = {f"hip_v{v}": (lambda v=v: _lib.ops().wgrad_gemm_(out, dy, x, 1, v)) for v in (6, 2, 1)}
    def v6_nosplit():
        os.environ["ST_WGRAD4_SPLIT"] = "1"
        _lib.ops().wgrad_gemm_(out, dy, x, 1, 6)
        os.environ.pop("ST_WGRAD4_SPLIT")

    arms["hip_v6_nosplit"] = v6_nosplit

    def v6_rs1():
        os.environ["ST_WGRAD4_RS"] = "1"
        _lib.ops().wgrad_gemm_(out, dy, x, 1, 6)
        os.environ.pop("ST_WGRAD4_RS")

    arms["hip_v6_rs1"] = v6_rs1
    for gm in ORDERS:
        def v6_order(gm=gm):
            os.environ["ST_WGRAD4_ORDER"] = gm
            _lib.ops().wgrad_gemm_(out, dy, x, 1, 6)
            os.environ.pop("ST_WGRAD4_ORDER")
        arms[f"hip_v6_order{gm}"] = v6_order
    arms["hipblaslt"] = lambda: torch.ops.aten.addmm.dtype_out(out, dy.t(), x, torch.float32, beta=1, alpha=1, out=out)
    res = {}
    for rnd in range(3):
        for k, fn in arms.items():
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                fn()
            e.record()
            e.synchronize()
            res[k] = min(res.get(k, 1e9), s.elapsed_time(e) / 3)
    fl = 2.0 * T * M * N
    print(name, json.dumps({k: {"ms": round(v, 3), "pflops": round(fl / v / 1e12, 3)} for k, v in res.items()}), flush=True)
    del dy, x, out

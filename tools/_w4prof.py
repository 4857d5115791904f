"""Kernels for PMC passes over the weight gradient at the Llama-3-8B gate|up shape (T 24,576, dY
[T, 28672], X [T, 4096]): csrc/wgrad4.hip (variant 6), the 8-phase kernel (variant 2) and hipBLASLt
(fp32 out, beta 1).  3 dispatches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load()
T, M, N = 24576, 28672, 4096
dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
out = torch.zeros(M, N, device="cuda")
for v in (6, 2):
    for _ in range(3):
        _lib.ops().wgrad_gemm_(out, dy, x, 1, v)
    torch.cuda.synchronize()
for _ in range(3):
    torch.ops.aten.addmm.dtype_out(out, dy.t(), x, torch.float32, beta=1, alpha=1, out=out)
torch.cuda.synchronize()

"""Kernels for PMC passes: gemm4w slot-major, gemm4w XCD-grouped, hipBLASLt (dense gate|up shape)."""
import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib
assert _lib.load()
T, K, N = 24576, 4096, 28672
x = torch.randn(T, K, device='cuda', dtype=torch.bfloat16)
w = torch.randn(1, N, K, device='cuda', dtype=torch.bfloat16) * 0.02
offs = torch.tensor([T], device='cuda', dtype=torch.int32)
os.environ["ST_GEMM4W_KIND"] = "0"
for order in ("0", "4"):
    os.environ["ST_GEMM4W_ORDER"] = order
    for _ in range(3):
        _lib.ops().gemm4w(x, w, offs)
    torch.cuda.synchronize()
for _ in range(3):
    torch.matmul(x, w[0].t())
torch.cuda.synchronize()

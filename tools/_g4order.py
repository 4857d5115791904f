"""gemm4w: kernel kind x tile order sweep on the dense gate|up and down shapes (timing only)."""
import sys, os, torch, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib
assert _lib.load()
shapes = {"gate_up": (24576, 4096, 28672), "down": (24576, 14336, 4096), "qkv": (24576, 4096, 6144)}
for name, (T, K, N) in shapes.items():
    x = torch.randn(T, K, device='cuda', dtype=torch.bfloat16)
    w = torch.randn(1, N, K, device='cuda', dtype=torch.bfloat16) * 0.02
    offs = torch.tensor([T], device='cuda', dtype=torch.int32)
    flops = 2.0 * T * K * N
    res = {}
    for rnd in range(3):
        for kind in ("0", "1", "4"):
            for order in ("0", "4"):
                os.environ["ST_GEMM4W_KIND"], os.environ["ST_GEMM4W_ORDER"] = kind, order
                _lib.ops().gemm4w(x, w, offs)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    _lib.ops().gemm4w(x, w, offs)
                e.record(); e.synchronize()
                key = f"k{kind}o{order}"
                res[key] = min(res.get(key, 1e9), s.elapsed_time(e) / 5)
    bl = torch.empty(T, N, device='cuda', dtype=torch.bfloat16)
    w2 = w[0]
    torch.matmul(x, w2.t(), out=bl)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        torch.matmul(x, w2.t(), out=bl)
    e.record(); e.synchronize()
    res["hipblaslt"] = s.elapsed_time(e) / 5
    print(name, json.dumps({k: round(flops / v / 1e9, 1) for k, v in res.items()}), flush=True)
    del x, w, bl

"""gemm4w: kernel kind x tile order sweep on the dense gate|up and down shapes (timing only)."""
import sys, os, torch, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib
assert _lib.load()
shapes = {  # name: (T, K, N) -- forward projections and the TN data gradients on W^T copies
    "gate_up": (24576, 4096, 28672), "down": (24576, 14336, 4096), "qkv": (24576, 4096, 6144),
    "o": (24576, 4096, 4096), "down_dgrad": (24576, 4096, 14336), "lm_head_chunk": (4096, 4096, 128256),
    "gate_up_dgrad": (24576, 28672, 4096), "qkv_dgrad": (24576, 6144, 4096)}
if len(sys.argv) > 1:
    shapes = {k: v for k, v in shapes.items() if k in sys.argv[1].split(",")}
for name, (T, K, N) in shapes.items():
    x = torch.randn(T, K, device='cuda', dtype=torch.bfloat16)
    w = torch.randn(1, N, K, device='cuda', dtype=torch.bfloat16) * 0.02
    offs = torch.tensor([T], device='cuda', dtype=torch.int32)
    flops = 2.0 * T * K * N
    res = {}
    for rnd in range(3):
        for kind in os.environ.get("G4_KINDS", "5,6").split(","):
            for order, sched in [(o, sc) for o in os.environ.get("G4_ORDERS", "0,4,8").split(",")
                                 for sc in os.environ.get("G4_SCHEDS", "0").split(",")]:
                os.environ["ST_GEMM4W_KIND"], os.environ["ST_GEMM4W_ORDER"] = kind, order
                os.environ["ST_GEMM4W_SCHED"] = sched
                _lib.ops().gemm4w(x, w, offs)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    _lib.ops().gemm4w(x, w, offs)
                e.record(); e.synchronize()
                key = f"k{kind}s{sched}o{order}"
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

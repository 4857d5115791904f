import sys, os, torch, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib
assert _lib.load()
T, K, N = 24576, 4096, 28672
x = torch.randn(T, K, device='cuda', dtype=torch.bfloat16)
w = torch.randn(1, N, K, device='cuda', dtype=torch.bfloat16) * 0.02
offs = torch.tensor([T], device='cuda', dtype=torch.int32)
kinds = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1", "2"]
flops = 2.0 * T * K * N
for kind in kinds:
    os.environ["ST_GEMM4W_KIND"] = kind
    res = {}
    for rnd in range(3):
        for probe in ("0", "1", "2", "3", "4", "5", "6"):
            os.environ["ST_GEMM4W_PROBE"] = probe
            _lib.ops().gemm4w(x, w, offs)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                _lib.ops().gemm4w(x, w, offs)
            e.record(); e.synchronize()
            ms = s.elapsed_time(e) / 5
            res[probe] = min(res.get(probe, 1e9), ms)
    print("kind", kind, json.dumps({k: {"ms": round(v, 3), "tflops": round(flops / v / 1e9, 1)} for k, v in res.items()}), flush=True)
os.environ["ST_GEMM4W_PROBE"] = "0"

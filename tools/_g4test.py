import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib
assert _lib.load()
torch.manual_seed(0)
# ragged groups (an empty one, a partial tile), K not a multiple of 128, every kernel kind
for K, counts, N in ((128, [37, 0, 300], 512), (192, [256, 1, 511], 512), (4096, [700, 300], 512),
                     (192, [3000, 0, 1999, 1], 4096), (1024, [4999, 1], 4096)):  # > 256 tiles: several per persistent WG
    c = torch.tensor(counts, device='cuda', dtype=torch.int32)
    offs = torch.cumsum(c, 0, dtype=torch.int32)
    T, G = int(c.sum()), len(counts)
    x = torch.randn(T, K, device='cuda', dtype=torch.bfloat16)
    w = torch.randn(G, N, K, device='cuda', dtype=torch.bfloat16)
    for kind, sched in (("0", "0"), ("4", "0"), ("5", "5"), ("6", "5")):
        os.environ["ST_GEMM4W_KIND"], os.environ["ST_GEMM4W_SCHED"] = kind, sched
        y = _lib.ops().gemm4w(x, w, offs)
        torch.cuda.synchronize()
        off, errs = 0, []
        for e, n in enumerate(counts):
            if n:
                ref = x[off:off + n].float() @ w[e].float().t()
                errs.append(round(float((y[off:off + n].float() - ref).norm() / ref.norm()), 5))
            off += n
        print("K", K, "kind", kind, "sched", sched, errs, flush=True)

import torch, time
print(torch.__version__, hasattr(torch, "_grouped_mm"))
dev = "cuda"
E, K, N = 8, 4096, 14336
counts = torch.tensor([900, 1100, 1000, 1024, 980, 1050, 990, 1148], device=dev)
M = int(counts.sum())
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
w = torch.randn(E, N, K, device=dev, dtype=torch.bfloat16)
offs = torch.cumsum(counts, 0).to(torch.int32)
try:
    y = torch._grouped_mm(x, w.transpose(-2, -1), offs=offs)
    ref = torch.cat([x[o - c:o] @ w[e].t() for e, (o, c) in enumerate(zip(offs.tolist(), counts.tolist()))])
    print("grouped ok", y.shape, ((y.float() - ref.float()).norm() / ref.float().norm()).item())
    for fn, name in ((lambda: torch._grouped_mm(x, w.transpose(-2, -1), offs=offs), "grouped"),
                     (lambda: [x[o - c:o] @ w[e].t() for e, (o, c) in enumerate(zip(offs.tolist(), counts.tolist()))], "loop")):
        for _ in range(3): fn()
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(10): fn()
        torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 10
        print(name, dt * 1e3, "ms", 2 * M * N * K / dt / 1e12, "TF/s")
except Exception as e:
    print("grouped_mm failed:", type(e).__name__, str(e)[:300])

import torch, time
dev = "cuda"
E, T, h, I2 = 8, 16384, 4096, 28672
x = torch.randn(T, h, device=dev, dtype=torch.bfloat16)
dy = torch.randn(T, I2, device=dev, dtype=torch.bfloat16)
offs = torch.cumsum(torch.full((E,), T // E, dtype=torch.int32, device=dev), 0, dtype=torch.int32)
for od in (None, torch.float32):
    try:
        out = torch._grouped_mm(dy.t(), x, offs=offs, out_dtype=od)  # [E, I2, h]
        torch.cuda.synchronize()
        ref = (dy[:T // E].float().t() @ x[:T // E].float())
        err = (out[0].float() - ref).abs().max().item() / ref.abs().max().item()
        t0 = time.perf_counter()
        for _ in range(5):
            out = torch._grouped_mm(dy.t(), x, offs=offs, out_dtype=od)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        print("out_dtype", od, out.dtype, tuple(out.shape), f"rel err {err:.2e}", f"{dt*1e3:.2f} ms", f"{2*T*h*I2/dt/1e15:.2f} PF/s", flush=True)
    except Exception as e:
        print("out_dtype", od, "FAILED", repr(e)[:300], flush=True)

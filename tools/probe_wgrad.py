import os as _os; _os.environ.setdefault("ST_KERNEL_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "build", "variants", "probes.so"))  # noqa: E401,E702 -- timing probes exist only in the diagnostic library (python -m scaletorch_amd._build --probes)
import os, sys, torch, json
sys.path.insert(0, os.getcwd())
from scaletorch_amd.ops import _lib
assert _lib.load()
T = 16384
res = {}
for name, (M, N) in {"gate_up": (28672, 4096), "down": (4096, 14336), "out": (4096, 4096)}.items():
    dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16); x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    out = torch.zeros(M, N, device="cuda")
    for rnd in range(3):
        for arm in ["p8", "p8_nodma", "p8_noread", "old", "old_nodma"]:
            os.environ["ST_WGRAD_P8"] = "1" if arm.startswith("p8") else "0"
            os.environ["ST_WGRAD_PROBE"] = "1" if "nodma" in arm else ("2" if "noread" in arm else "0")
            _lib.ops().wgrad_gemm_(out, dy, x, 1)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(); s.record()
            for _ in range(10): _lib.ops().wgrad_gemm_(out, dy, x, 1)
            e.record(); torch.cuda.synchronize()
            t = s.elapsed_time(e) / 10
            k = f"{name}_{arm}"
            res[k] = min(res.get(k, 1e9), round(2 * T * M * N / t / 1e9, 1))
    print(name, {k: v for k, v in res.items() if k.startswith(name)}, flush=True)

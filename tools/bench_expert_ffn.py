"""Expert FFN forward + backward (scaletorch_amd/models/moe.py ``_ExpertFFNFn``): the one-launch
HIP grouped kernels vs one hipBLASLt GEMM per expert (host-known counts), at the per-rank expert
shapes of the MoE presets -- 1-GPU proxies (all experts local) and EP 8 (Mixtral: 1 local
expert, Qwen3-30B-A3B: 16).  Prints ms per fwd+bwd and the GEMM TF/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.models.moe import _ExpertFFNFn  # noqa: E402

SHAPES = {  # name: (local experts, rows per expert, hidden, moe intermediate)
    "mixtral_1gpu_mbs1": (8, 1024, 4096, 14336),
    "mixtral_ep8_rank": (1, 8192, 4096, 14336),
    "qwen3moe_1gpu_mbs2": (128, 512, 2048, 768),
    "qwen3moe_ep8_rank": (16, 4096, 2048, 768),
}


def run(G, n, h, I, host, reps=5):
    counts = [n] * G
    offs = torch.cumsum(torch.tensor(counts, device="cuda", dtype=torch.int32), 0, dtype=torch.int32)
    x = torch.randn(G * n, h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w_gu = torch.nn.Parameter(torch.randn(G, 2 * I, h, device="cuda", dtype=torch.bfloat16) * 0.02)
    w_dn = torch.nn.Parameter(torch.randn(G, h, I, device="cuda", dtype=torch.bfloat16) * 0.02)
    for w in (w_gu, w_dn):
        w.main_grad = torch.zeros(w.shape, device="cuda")
    dy = torch.randn(G * n, h, device="cuda", dtype=torch.bfloat16)

    def once():
        for w in (w_gu, w_dn):
            w._st_fresh = True
        y = _ExpertFFNFn.apply(x, offs, w_gu, w_dn, counts if host else None)
        y.backward(dy)
        x.grad = None

    once()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        once()
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / reps
    flops = 3 * 2 * G * n * h * 3 * I  # 3 GEMMs (gate|up 2I, down I) x (fwd, dgrad, wgrad)
    return ms, flops / ms / 1e9


def main():
    out = {}
    for name, (G, n, h, I) in SHAPES.items():
        r = {}
        for rnd in range(2):
            for host in (False, True):
                ms, tf = run(G, n, h, I, host)
                k = "per_expert_hipblaslt" if host else "grouped_hip"
                if k not in r or ms < r[k]["ms"]:
                    r[k] = {"ms": round(ms, 3), "tflops": round(tf, 1)}
        out[name] = r
        print(name, json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

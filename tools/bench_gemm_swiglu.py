"""gate|up GEMM + SwiGLU at the Llama-3-8B bench shape (T 24,576, K 4,096, I 14,336): hipBLASLt
GEMM + csrc/swiglu.hip pass vs ONE csrc/gemm4w.hip kernel with the SwiGLU epilogue (both tile
orders), and the plain kind-5 GEMM.  Prints ms per call (min over rounds)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaletorch_amd.ops import _lib  # noqa: E402

assert _lib.load()


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    T, K, I = 24576, 4096, 14336
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(2 * I, K, device="cuda", dtype=torch.bfloat16) * 0.02
    offs = torch.tensor([T], device="cuda", dtype=torch.int32)
    res = {}

    def unfused():
        gu = torch.matmul(x, w.t())
        return _lib.ops().swiglu_fwd(gu)

    def gemm_only():
        return torch.matmul(x, w.t())

    def fused():
        return _lib.ops().gemm_swiglu(x, w)

    def plain5():
        return _lib.ops().gemm4w(x, w.unsqueeze(0), offs)

    for rnd in range(3):
        for name, fn, env in (("hipblaslt_gemm", gemm_only, {}), ("hipblaslt_gemm+swiglu", unfused, {}),
                              ("fused_o0", fused, {"ST_GEMM4W_ORDER": "0"}),
                              ("fused_o4", fused, {"ST_GEMM4W_ORDER": "4"}),
                              ("gemm4w_k5_o0", plain5, {"ST_GEMM4W_ORDER": "0"}),
                              ("gemm4w_k5_o4", plain5, {"ST_GEMM4W_ORDER": "4"})):
            os.environ.update(env)
            ms = timeit(fn)
            for k in env:
                os.environ.pop(k, None)
            res[name] = min(res.get(name, 1e9), ms)
    gu_ref = torch.matmul(x, w.t())
    gu, h = _lib.ops().gemm_swiglu(x, w)
    err = ((gu.float() - gu_ref.float()).norm() / gu_ref.float().norm()).item()
    print(json.dumps({"ms": {k: round(v, 3) for k, v in res.items()},
                      "gemm_tflops": {k: round(2.0 * T * K * 2 * I / v / 1e9, 1) for k, v in res.items()},
                      "rel_err_gu_vs_hipblaslt": err, "h_equals_swiglu_kernel": bool(torch.equal(h, _lib.ops().swiglu_fwd(gu)))}))


if __name__ == "__main__":
    main()

"""Weight-gradient plumbing shared by every fused op.

When a parameter carries ``main_grad`` (an fp32 view into the flat gradient
arena owned by :class:`scaletorch_amd.parallel.data_parallel.GradArena`), fused
backward passes accumulate the weight gradient straight into it -- for linear
layers with ONE GEMM whose epilogue adds into the fp32 buffer (beta = 1,
bf16 x bf16 -> fp32), so no bf16 ``.grad`` tensor is ever materialised and no
separate accumulation kernel runs.  The parameter's ``_st_grad_ready`` hook
(installed by the DP bucket manager) is then called so the bucket holding the
parameter can start its all-reduce while the rest of backward runs.

Without ``main_grad`` (plain autograd use, unit tests) the gradient is returned
normally and autograd accumulates ``.grad``.
"""
from __future__ import annotations

import os

import torch

_ADDMM_DTYPE_OK: bool | None = None
# per-shape winner of the weight-gradient GEMM: 1 / 2 = csrc/wgrad_gemm.hip 4-stage / 8-phase, 0 = hipBLASLt
_WGRAD_CHOICE: dict = {}
_WGRAD_TIMES: dict = {}  # tuning measurements (ms for two calls), for tools/ab_step.py
_TUNE_MAX_BYTES = 512 << 20


# ---------------------------------------------------------------- data-gradient GEMM layout
# dX = dY W on a row-major weight is an NN GEMM; hipBLASLt runs the TN form
# F.linear(dY, W^T) 14-19 % faster on MI355X for every Llama-3-8B projection
# (profiles/r02/dgrad_layout.json: 1.32-1.37 -> 1.54-1.62 PF/s).  So each arena
# weight gets a persistent K-contiguous copy W^T, produced ONCE per optimizer
# step by csrc/transpose.hip (5-6.6 TB/s) on a side stream during the forward
# pass -- hidden under the forward GEMMs -- and consumed by the backward.
_WT_EPOCH = [0]
_WT_STREAMS: dict = {}


def bump_weight_epoch() -> None:
    """Weights may have changed (new step / load): W^T copies must be refreshed."""
    _WT_EPOCH[0] += 1


def invalidate_wt(params) -> None:
    """The weights were overwritten outside the optimizer (checkpoint / HF load): drop
    their W^T copies, including one the fused AdamW pass left pending."""
    for w in params:
        w._st_wt_pending = None
        w._st_wt_epoch = -1


def _wt_enabled(w: torch.Tensor) -> bool:
    return (w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.shape[0] % 64 == 0
            and w.shape[1] % 64 == 0 and getattr(w, "main_grad", None) is not None
            and os.environ.get("ST_DGRAD_WT", "1") == "1")


def prepare_dgrad_weight(w: torch.Tensor) -> None:
    """Launch (once per weight epoch) the side-stream transpose W -> W^T.  Call from
    a forward, after the weight's bucket wait, so the copy sees the updated weight."""
    if not _wt_enabled(w):
        return
    from . import _lib

    if not _lib.use_native(w):
        return
    if getattr(w, "_st_wt_epoch", -1) == _WT_EPOCH[0]:
        return
    pending = getattr(w, "_st_wt_pending", None)
    if pending is not None:
        # the side-stream AdamW pass already wrote W^T with the updated weight
        # (optim.py ``_step_overlapped``, csrc/adamw.hip adamw_wt_kernel): adopt it
        w._st_wt_pending = None
        w._st_wt_done = pending
        w._st_wt_epoch = _WT_EPOCH[0]
        return
    if getattr(w, "_st_wt", None) is not None and _lib.probe_env("ST_DGRAD_WT_PROBE_STALE"):
        # timing probe of the diagnostic library only (WRONG gradients): reuse the previous
        # step's W^T, no transpose
        w._st_wt_epoch = _WT_EPOCH[0]
        return
    buf = getattr(w, "_st_wt", None)
    if buf is None or buf.shape != (w.shape[1], w.shape[0]):
        buf = torch.empty(w.shape[1], w.shape[0], dtype=w.dtype, device=w.device)
        w._st_wt = buf
    if os.environ.get("ST_DGRAD_WT_STREAM", "side") == "main":  # serialised into the forward (A/B)
        _lib.ops().transpose_(w.detach(), buf)
        done = torch.cuda.Event()
        done.record()
        w._st_wt_done = done
        w._st_wt_epoch = _WT_EPOCH[0]
        return
    st = _WT_STREAMS.get(w.device.index)
    if st is None:
        # ST_WT_STREAM_PRIORITY: HIP priority of the W^T stream (0 default, -1 high)
        st = _WT_STREAMS[w.device.index] = torch.cuda.Stream(
            device=w.device, priority=int(os.environ.get("ST_WT_STREAM_PRIORITY", "0")))
    ready = torch.cuda.Event()
    ready.record()
    with torch.cuda.stream(st):
        st.wait_event(ready)
        _lib.ops().transpose_(w.detach(), buf)
        done = torch.cuda.Event()
        done.record(st)
    w._st_wt_done = done
    w._st_wt_epoch = _WT_EPOCH[0]


def dgrad(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dX = dY W, on the TN layout when a current W^T copy exists."""
    if getattr(w, "_st_wt_epoch", -1) == _WT_EPOCH[0] and dy.is_cuda:
        torch.cuda.current_stream().wait_event(w._st_wt_done)
        return torch.nn.functional.linear(dy, w._st_wt)
    return dy.matmul(w)


def dgrad_into(dy2: torch.Tensor, w: torch.Tensor, out: torch.Tensor) -> None:
    """``out = dY W`` for 2-D ``dy2`` / ``out`` (a row block of a larger dX), TN layout
    when a current W^T copy exists."""
    if getattr(w, "_st_wt_epoch", -1) == _WT_EPOCH[0] and dy2.is_cuda:
        torch.cuda.current_stream().wait_event(w._st_wt_done)
        torch.matmul(dy2, w._st_wt.t(), out=out)
        return
    torch.matmul(dy2, w, out=out)


# ---------------------------------------------------------------- weight-gradient GEMM layout
# dW = dY^T X with both operands token-major is an "NT" GEMM (neither operand
# K-contiguous); hipBLASLt's TN kernels on token-contiguous copies dY^T [out, T]
# and X^T [in, T] run 1.25-1.38 PF/s vs 1.0-1.17 for the NT path and for the
# hand-written csrc/wgrad_gemm.hip (profiles/gemm_microbench.json "wgradT").
# The two transposes (csrc/transpose.hip, ~5.5 TB/s) are issued on a side
# stream BEFORE the layer's data-gradient GEMM.  Measured in-step on MI355X it LOSES
# (735 vs 713 ms/step, profiles/r02/wgrad_tn_ab.log): off by default (ST_WGRAD_TN=1 on).
_WG_STREAMS: dict = {}


def _wgrad_tn_ok(dy2d: torch.Tensor, x2d: torch.Tensor) -> bool:
    return (dy2d.is_cuda and dy2d.dtype == torch.bfloat16 and x2d.dtype == torch.bfloat16
            and dy2d.shape[0] % 64 == 0 and dy2d.shape[1] % 64 == 0 and x2d.shape[1] % 64 == 0
            and dy2d.stride(1) == 1 and x2d.stride(1) == 1 and dy2d.stride(0) % 8 == 0 and x2d.stride(0) % 8 == 0
            and dy2d.data_ptr() % 16 == 0 and x2d.data_ptr() % 16 == 0
            and os.environ.get("ST_WGRAD_TN", "0") == "1"
            and dy2d.shape[1] >= float(os.environ.get("ST_WGRAD_TN_MIN_RATIO", "0")) * x2d.shape[1])


class WgradOperands:
    """Token-contiguous copies of (dY, X) being produced on a side stream."""

    __slots__ = ("dyt", "xt", "done")

    def __init__(self, dyt, xt, done):
        self.dyt, self.xt, self.done = dyt, xt, done


def prefetch_wgrad(param: torch.Tensor, dy2d: torch.Tensor, x2d: torch.Tensor):
    """Start the dY^T / X^T transposes for ``param``'s weight gradient on a side
    stream (call before the data-gradient GEMM so they overlap it); None when the
    TN path does not apply."""
    mg = getattr(param, "main_grad", None)
    if mg is None or mg.dtype != torch.float32 or not _wgrad_tn_ok(dy2d, x2d):
        return None
    from . import _lib

    if not _lib.use_native(dy2d):
        return None
    T = dy2d.shape[0]
    dyt = torch.empty(dy2d.shape[1], T, dtype=dy2d.dtype, device=dy2d.device)
    xt = torch.empty(x2d.shape[1], T, dtype=x2d.dtype, device=x2d.device)
    if os.environ.get("ST_WGRAD_TN_STREAM", "side") == "main":
        st = torch.cuda.current_stream(dy2d.device)
    else:
        st = _WG_STREAMS.get(dy2d.device.index)
        if st is None:
            st = _WG_STREAMS[dy2d.device.index] = torch.cuda.Stream(device=dy2d.device)
    ready = torch.cuda.Event()
    ready.record()
    with torch.cuda.stream(st):
        st.wait_event(ready)
        _lib.ops().transpose_(dy2d, dyt)
        _lib.ops().transpose_(x2d, xt)
        done = torch.cuda.Event()
        done.record(st)
    return WgradOperands(dyt, xt, done)


def _grad_ready(param: torch.Tensor) -> None:
    hook = getattr(param, "_st_grad_ready", None)
    if hook is not None:
        hook(param)


def take_fresh(param: torch.Tensor) -> bool:
    """True (once per step) if ``param.main_grad`` holds last step's values.

    The arena does not zero its fp32 gradients between steps (a 4-byte/param
    fill pass); instead every parameter is marked fresh and its FIRST gradient
    write of the step overwrites (GEMM beta = 0, copy) rather than accumulates.
    Parameters nobody wrote are zeroed before their bucket is reduced
    (data_parallel.GradArena.zero_fresh)."""
    if getattr(param, "_st_fresh", False):
        param._st_fresh = False
        return True
    return False


def accumulate_grad(param: torch.Tensor, grad: torch.Tensor):
    """Add ``grad`` into ``param.main_grad`` (returns None) or return it for autograd."""
    mg = getattr(param, "main_grad", None)
    if mg is None:
        return grad.to(param.dtype) if grad.dtype != param.dtype else grad
    if take_fresh(param):
        mg.copy_(grad.view_as(mg))
    else:
        mg.add_(grad.view_as(mg))
    _grad_ready(param)
    return None


def _one_t_ok(dy2d: torch.Tensor, x2d: torch.Tensor) -> bool:
    T = dy2d.shape[0]
    return (T % 64 == 0 and dy2d.shape[1] % 64 == 0 and x2d.shape[1] % 64 == 0 and dy2d.stride(1) == 1
            and x2d.stride(1) == 1 and dy2d.stride(0) % 8 == 0 and x2d.stride(0) % 8 == 0
            and dy2d.data_ptr() % 16 == 0 and x2d.data_ptr() % 16 == 0)


def _wgrad_one_t(out: torch.Tensor, dy2d: torch.Tensor, x2d: torch.Tensor, beta: int, tuned: bool = False) -> None:
    """out = beta out + dY^T X with the SMALLER operand first transposed to token-contiguous
    (csrc/transpose.hip, ~5.5 TB/s), so hipBLASLt reads one operand K-contiguous: on the
    gate|up shape (dY 28672 wide, X 4096) 1390 vs 1292 TF/s for the HIP kernel, transpose
    included (profiles/r03/wgrad_layouts.log).  ``tuned``: the GEMM runs on csrc/gemm.cpp's
    autotuned hipBLASLt call (every heuristic candidate timed once per shape) instead of
    PyTorch's first heuristic.  Picked per shape by ``_wgrad_pick``."""
    from . import _lib

    T = dy2d.shape[0]
    if x2d.shape[1] <= dy2d.shape[1]:
        xt = torch.empty(x2d.shape[1], T, dtype=x2d.dtype, device=x2d.device)
        _lib.ops().transpose_(x2d, xt)
        if tuned:
            _lib.ops().gemm_(out, dy2d, xt, True, True, 1.0, float(beta))
        else:
            torch.ops.aten.addmm.dtype_out(out, dy2d.t(), xt.t(), torch.float32, beta=beta, alpha=1, out=out)
    else:
        dyt = torch.empty(dy2d.shape[1], T, dtype=dy2d.dtype, device=dy2d.device)
        _lib.ops().transpose_(dy2d, dyt)
        if tuned:
            _lib.ops().gemm_(out, dyt, x2d, False, False, 1.0, float(beta))
        else:
            torch.ops.aten.addmm.dtype_out(out, dyt, x2d, torch.float32, beta=beta, alpha=1, out=out)


def _wgrad_pick(dy2d: torch.Tensor, x2d: torch.Tensor) -> int:
    """First call per (shape, strides): time the two HIP kernels (1: 4-stage ring,
    2: 8-phase ping-pong, csrc/wgrad_gemm.hip; each with and without the tail split), 3: hipBLASLt
    on the smaller operand transposed to token-contiguous (``_wgrad_one_t``), against the hipBLASLt fp32-epilogue
    GEMM on a scratch output (5 rounds x 2 calls, same stream, interleaved) and keep
    the fastest -- 0 = hipBLASLt.  On gfx950 none wins every projection shape
    (tools/probe_wgrad.py: the 8-phase kernel +3-13 % on out/down, -1-2 % on
    gate_up/qkv)."""
    from . import _lib

    key = (tuple(dy2d.shape), dy2d.stride(0), tuple(x2d.shape), x2d.stride(0), dy2d.device.index)
    got = _WGRAD_CHOICE.get(key)
    if got is not None:
        return got
    M, N = dy2d.shape[1], x2d.shape[1]
    if os.environ.get("ST_WGRAD_TUNE", "1") != "1":
        _WGRAD_CHOICE[key] = 1
        return 1
    if M * N * 4 > _TUNE_MAX_BYTES:
        # output too large for a scratch copy (the untied LM head: 128256 x 4096 fp32 = 2.1 GB):
        # time the arms on a column slice of dY -- the first Ms output rows -- instead
        Ms = max(256, (_TUNE_MAX_BYTES // (N * 4)) // 256 * 256)
        if Ms >= M or Ms * N * 4 > _TUNE_MAX_BYTES or os.environ.get("ST_WGRAD_TUNE_LARGE", "1") != "1":
            _WGRAD_CHOICE[key] = 1
            return 1
        dy2d = dy2d[:, :Ms]
        M = Ms
    scratch = torch.zeros(M, N, dtype=torch.float32, device=dy2d.device)
    # +16: the same kernel without the tail split (csrc/wgrad_gemm.hip), where the last
    # partial round of tiles is left partly idle instead of being cut into token ranges
    # 6: the one-wave-per-SIMD kernel (csrc/wgrad4.hip)
    hip_arms = (1, 2, 6, 17, 18, 22) if os.environ.get("ST_WGRAD4", "1") == "1" else (1, 2, 17, 18)
    arms = {v: (lambda v=v: _lib.ops().wgrad_gemm_(scratch, dy2d, x2d, 1, v)) for v in hip_arms
            if _lib.ops().wgrad_gemm_(scratch, dy2d, x2d, 0, v)}
    if not arms:
        _WGRAD_CHOICE[key] = 0
        return 0
    if _one_t_ok(dy2d, x2d) and os.environ.get("ST_WGRAD_ONE_T", "1") == "1":
        # 3: hipBLASLt on the smaller operand made token-contiguous (transpose timed in);
        # 5: the same on the autotuned hipBLASLt call (csrc/gemm.cpp)
        arms[3] = lambda: _wgrad_one_t(scratch, dy2d, x2d, 1)
        if os.environ.get("ST_WGRAD_TUNED", "1") == "1":
            arms[5] = lambda: _wgrad_one_t(scratch, dy2d, x2d, 1, tuned=True)
    if os.environ.get("ST_WGRAD_TUNED", "1") == "1":
        # 4: the fp32-epilogue GEMM on the autotuned hipBLASLt call, operands as stored
        arms[4] = lambda: _lib.ops().gemm_(scratch, dy2d, x2d, True, False, 1.0, 1.0)

    def blas():
        torch.ops.aten.addmm.dtype_out(scratch, dy2d.t(), x2d, torch.float32, beta=1, alpha=1, out=scratch)

    arms[0] = blas
    best = {}
    try:
        blas()
        for _ in range(5):
            for name, fn in arms.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn()
                fn()
                e.record()
                e.synchronize()
                best[name] = min(best.get(name, 1e30), s.elapsed_time(e))
        choice = min(best, key=best.get)
    except (RuntimeError, NotImplementedError):
        choice = 1
    del scratch
    _WGRAD_CHOICE[key] = choice
    _WGRAD_TIMES[key] = best
    return choice


_WGRAD_SIDE: dict = {}


def wgrad_side_stream(device: torch.device):
    """The stream linear weight gradients run on when ``ST_WGRAD_STREAM=side`` (else None):
    the dW GEMM then overlaps the backward's next data-gradient GEMM and its memory-bound
    elementwise kernels instead of following them on one stream.  Readers of main_grad
    (DP bucket launches, the post-backward join) wait for this stream.  Measured at
    Llama-3-8B mbs 6 it is 3x SLOWER (2981 vs 1002 ms/step, profiles/r03/wgrad_side_stream_ab.log):
    dY / X stay allocated until the side stream catches up (record_stream), and at 271 GB
    of 288 the caching allocator then frees and re-allocates synchronously.  Kept opt-in for
    configurations with memory to spare."""
    import os

    if device.type != "cuda" or os.environ.get("ST_WGRAD_STREAM", "main") != "side":
        return None
    st = _WGRAD_SIDE.get(device.index)
    if st is None:
        st = _WGRAD_SIDE[device.index] = torch.cuda.Stream(device=device)
    return st


def accumulate_linear_wgrad(param: torch.Tensor, dy2d: torch.Tensor, x2d: torch.Tensor, pre=None):
    """dW = dy^T x, accumulated into ``param.main_grad`` in fp32 when present.

    On GPU the product runs on the hand-written gfx950 weight-gradient GEMM
    (csrc/wgrad_gemm.hip: both operands token-major, read with LDS transpose
    reads, fp32 epilogue accumulating into main_grad); shapes it does not tile
    go to ``aten::addmm.dtype_out`` (hipBLASLt, bf16 operands, fp32 C/D).
    ``ST_WGRAD_KERNEL=0`` forces the hipBLASLt path (A/B).  Preferred on GPU: the
    TN GEMM on token-contiguous copies (``prefetch_wgrad``; opt-in ``ST_WGRAD_TN=1``).
    """
    mg = getattr(param, "main_grad", None)
    if mg is None:
        return dy2d.t().mm(x2d)
    if pre is None and mg.dtype == torch.float32:
        pre = prefetch_wgrad(param, dy2d, x2d)
    beta = 0 if take_fresh(param) else 1
    if pre is not None:
        torch.cuda.current_stream().wait_event(pre.done)
        m2 = mg.view(mg.shape[0], -1)
        torch.ops.aten.addmm.dtype_out(m2, pre.dyt, pre.xt.t(), torch.float32, beta=beta, alpha=1, out=m2)
        _grad_ready(param)
        return None
    ws = wgrad_side_stream(dy2d.device) if mg.dtype == torch.float32 else None
    if ws is not None:
        ready = torch.cuda.Event()
        ready.record()
        ws.wait_event(ready)
        with torch.cuda.stream(ws):
            wgrad_into(mg.view(mg.shape[0], -1), dy2d, x2d, beta)
        dy2d.record_stream(ws)  # autograd frees them when this node returns
        x2d.record_stream(ws)
    else:
        wgrad_into(mg.view(mg.shape[0], -1), dy2d, x2d, beta)
    _grad_ready(param)
    return None


def wgrad_into(out: torch.Tensor, dy2d: torch.Tensor, x2d: torch.Tensor, beta: int,
               variant: int | None = None) -> None:
    """``out = beta * out + dy2d^T x2d`` for a 2-D ``out`` (fp32 accumulator or the
    operands' dtype), on the per-shape faster of csrc/wgrad_gemm.hip and hipBLASLt.
    ``variant`` (0 hipBLASLt, 1 / 2 the HIP kernels) skips the per-shape pick: for
    token counts that change every step (MoE experts) timing each new shape would
    cost more than it saves."""
    global _ADDMM_DTYPE_OK
    if out.dtype == dy2d.dtype:
        out.addmm_(dy2d.t(), x2d, beta=beta)
        return
    if (out.dtype == torch.float32 and dy2d.is_cuda and dy2d.dtype == torch.bfloat16
            and x2d.dtype == torch.bfloat16 and os.environ.get("ST_WGRAD_KERNEL", "1") == "1"):
        from . import _lib

        if _lib.use_native(dy2d):
            forced = os.environ.get("ST_WGRAD_VARIANT", "")  # 0-6 / 17 / 18 overrides the pick (A/B)
            if forced in ("0", "1", "2", "3", "4", "5", "6", "17", "18"):
                variant = int(forced)
            elif variant is None:
                variant = _wgrad_pick(dy2d, x2d)
            if variant in (3, 5) and _one_t_ok(dy2d, x2d):
                _wgrad_one_t(out, dy2d, x2d, beta, tuned=variant == 5)
                return
            if variant == 4:
                _lib.ops().gemm_(out, dy2d, x2d, True, False, 1.0, float(beta))
                return
            if variant and variant not in (3, 4, 5) and _lib.ops().wgrad_gemm_(out, dy2d, x2d, beta, variant):
                return
    if _ADDMM_DTYPE_OK is not False and dy2d.is_cuda and os.environ.get("ST_WGRAD_FP32_GEMM", "1") == "1":
        try:
            torch.ops.aten.addmm.dtype_out(out, dy2d.t(), x2d, out.dtype, beta=beta, alpha=1, out=out)
            _ADDMM_DTYPE_OK = True
            return
        except (RuntimeError, NotImplementedError):
            _ADDMM_DTYPE_OK = False
    prod = dy2d.t().mm(x2d)
    if beta == 0:
        out.copy_(prod)
    else:
        out.add_(prod)

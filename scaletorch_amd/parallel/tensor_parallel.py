"""Megatron-style tensor parallelism (+ sequence parallelism) for MI355X.

Reference: scaletorch/parallel/tensor_parallel/{tensor_parallel.py,tp_comms.py}
and scaletorch/parallel/sequence_parallel/sp_comms.py.  What differs:

* layers are built TP-sharded from the start (no post-hoc module swap), and the
  Q/K/V projections and the gate/up projections are each ONE column-parallel
  GEMM (``FusedColumnParallelLinear``): the backward grad-input all-reduce runs
  2x per decoder layer instead of 5x, and each GEMM is larger
  (better MFMA utilisation);
* the column-parallel backward overlaps its grad-input all-reduce (issued
  async on RCCL's stream) with the weight-gradient GEMM, which accumulates
  straight into the fp32 ``main_grad`` arena;
* sequence parallelism is real: activations between TP regions are sharded on
  the sequence dim, column-parallel inputs are all-gathered (backward:
  reduce-scatter) and row-parallel outputs reduce-scattered (backward:
  all-gather) -- the reference never wired SP into Qwen3;
* the LM head stays vocab-sharded; the loss is the vocab-parallel
  cross-entropy (ops/xent.py) -- no [b, S, V] all-gather.
Checkpoints split the fused layers back into the reference's
``q_proj/k_proj/v_proj`` and ``gate_proj/up_proj`` names (per-TP-rank shards,
models/base.py ``reference_state_dict``), so they keep the reference layout.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..dist import collectives as C
from ..ops.grad import (accumulate_grad, accumulate_linear_wgrad, dgrad, dgrad_into, prefetch_wgrad,
                        prepare_dgrad_weight)
from . import mesh


# ====================================================================== comm autograd functions
def _ws(group) -> int:
    return C.get_world_size(group)


# TP transport: "rccl" or "xgmi" (dist/xgmi.py: one-shot / two-shot all-reduce, all-gather,
# reduce-scatter over IPC-mapped peer buffers; messages a kernel does not take go to RCCL).
# One communicator per TP group.  ``_TP_XGMI_OPS``: which collectives take the xGMI path --
# the start-up self-test keeps each only where it beat RCCL at the run's real message size.
_TP_COMM = "rccl"
_XGMI: dict = {}
_TP_XGMI_OPS = {"all_reduce": True, "all_gather": True, "reduce_scatter": True}


def set_tp_comm(kind: str, ops: dict | None = None) -> None:
    global _TP_COMM
    if kind not in ("rccl", "xgmi"):
        raise ValueError(f"tp_comm must be rccl or xgmi, got {kind!r}")
    _TP_COMM = kind
    for op in _TP_XGMI_OPS:
        _TP_XGMI_OPS[op] = kind == "xgmi" and (ops is None or bool(ops.get(op, False)))
    TRANSPORT["tp"] = kind
    TRANSPORT["ops"] = [op for op, on in _TP_XGMI_OPS.items() if on] if kind == "xgmi" else []


_PAIR: list = [None]  # dist/xgmi.PairPath of a 2-rank TP group (multipath SP collectives)


def setup_tp_pair_path(group) -> None:
    """Collective over the WORLD at start-up (--tp_comm xgmi, tp = 2 on one node): the SP
    all-gather / reduce-scatter of the 2-rank TP group then runs over the direct link
    plus 2-hop relays through the other GPUs (dist/xgmi.py pair collectives)."""
    from ..dist.xgmi import setup_pair_path

    _PAIR[0] = setup_pair_path(group)


TRANSPORT: dict = {"tp": "rccl", "ops": [], "selftest": None}  # chosen TP transport (bench JSON reports it)


def _tp_area_bytes(msg_bytes: int | None) -> int:
    """IPC data area of a TP-group communicator: the run's largest TP message (the
    all-reduce / reduce-scatter input [B, S, h] bf16) rounded up to 8 MiB, at least 16 MiB;
    ST_XGMI_TP_MAX_MB overrides (shared-GPU rehearsals and tests set it small)."""
    import os

    env = os.environ.get("ST_XGMI_TP_MAX_MB")
    if env:
        return int(float(env) * (1 << 20))
    m = int(msg_bytes or (64 << 20))
    return max(16 << 20, -(-m // (8 << 20)) * (8 << 20))


def _close_tp_xgmi() -> None:
    """Release every TP-side IPC area (a losing self-test keeps no dead HBM)."""
    for comm in list(_XGMI.values()):
        comm.close()
    _XGMI.clear()
    if _PAIR[0] is not None:
        _PAIR[0].comm.close()
    _PAIR[0] = None


def select_tp_transport(group, requested: str = "auto", probe_mb: int = 64, msg_bytes: int | None = None) -> str:
    """Pick the TP transport at start-up; collective over the WORLD (every rank calls it).

    ``requested`` "rccl" / "xgmi" are taken as given.  "auto", every TP size on one node:
      * tp = 2: the 7-link pair path (dist/xgmi.py ``setup_pair_path``) self-tested against
        RCCL -- a ``probe_mb`` MiB all-gather and reduce-scatter (AG bitwise, RS within one
        bf16 rounding), kept only if faster on both;
      * tp > 2 (4 / 8: the reference's TP4 / TP8 rows): a communicator over the TP group
        whose all-reduce (one-shot <= 512 KiB, two-shot above), all-gather and
        reduce-scatter are each timed against RCCL at the run's REAL message size
        ``msg_bytes`` (the [B, S, h] activation a row-parallel linear all-reduces) --
        all-gather bitwise equal to RCCL's, all-reduce / reduce-scatter within one bf16
        rounding of an fp32 sum of the gathered inputs; each collective keeps xGMI only
        where it is correct AND faster.
    Every verdict is MIN-reduced over the world, so all ranks route identically; anything
    that fails falls back to RCCL and the losing communicators are closed (their IPC areas
    freed).  Reference transport: NCCL/HCCL only (tp_comms.py:117-166, :288-315;
    sp_comms.py:31-94)."""
    import torch.distributed as dist

    ws = _ws(group)
    if requested in ("rccl", "xgmi"):
        set_tp_comm(requested)
        if requested == "xgmi" and ws == 2:
            setup_tp_pair_path(group)
        return requested
    if requested != "auto":
        raise ValueError(f"tp_comm must be auto, rccl or xgmi, got {requested!r}")
    names = list(_TP_XGMI_OPS)
    flags, info = [0] * len(names), {}
    import os

    # the pair path's node-wide communicator opens every peer's 512 MiB IPC areas: with more
    # than two ranks time-slicing ONE GPU (ST_GPU_OVERSUBSCRIBE rehearsals) that setup hung
    # (8-rank tp2pp2dp2 / tp2 x dp4 rehearsals, round 6; dist/xgmi.py _max_bytes_default), so
    # such runs keep RCCL unless the area is set explicitly (ST_XGMI_MAX_MB)
    shared_many = (os.environ.get("ST_GPU_OVERSUBSCRIBE", "0") == "1" and dist.is_initialized()
                   and dist.get_world_size() > 2 and "ST_XGMI_MAX_MB" not in os.environ)
    if ws == 2 and shared_many:
        info = {"skipped": "tp = 2 pair path on > 2 ranks sharing one GPU (set ST_XGMI_MAX_MB to force)"}
    elif ws >= 2 and torch.cuda.is_available():
        try:
            if ws == 2:
                setup_tp_pair_path(group)
                pair = _PAIR[0]
                if pair is not None:
                    ok, info = _pair_selftest(pair, group, probe_mb)
                    # the pair path carries the SP gathers / scatters; all-reduces stay on the
                    # 2-rank communicator's kernels only when the pair path is on
                    flags = [ok] * len(names)
            else:
                from ..dist.xgmi import XgmiAllReduce

                comm = _XGMI[id(group)] = XgmiAllReduce(group, max_bytes=_tp_area_bytes(msg_bytes))
                per_op, info = _tp_selftest(comm, group, msg_bytes or (probe_mb << 20))
                flags = [per_op.get(n, 0) for n in names]
        except Exception as e:  # noqa: BLE001 -- fall back, but every rank still joins the vote
            flags, info = [0] * len(names), {"error": repr(e)[:200]}
    voted = _vote(names, flags)
    choice = "xgmi" if any(voted.values()) else "rccl"
    if choice == "rccl":
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()  # no peer still reads an area we are about to free
        _close_tp_xgmi()
    set_tp_comm(choice, voted)
    TRANSPORT.update(selftest=info)
    return choice


def _vote(names: list, flags: list) -> dict:
    """MIN of every rank's per-collective verdict over the world: a collective keeps the xGMI
    path only if it passed on EVERY rank (one all-reduce; gloo-safe on CPU)."""
    import torch.distributed as dist

    on_gpu = torch.cuda.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"
    flag = torch.tensor(flags, dtype=torch.int32, device="cuda" if on_gpu else "cpu")
    if dist.is_initialized():
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return {n: bool(int(v)) for n, v in zip(names, flag.tolist())}


def _tp_selftest(comm, group, msg_bytes: int):
    """Per-collective verdicts ({op: 1 if correct and faster than RCCL else 0}, timings) of a
    TP-group communicator at ``msg_bytes`` (capped by its area)."""
    ws, r = _ws(group), C.get_rank(group)
    n = max(8 * ws, min(int(msg_bytes), comm.cap) // 2 // (8 * ws) * (8 * ws))  # bf16 elements
    g = torch.Generator(device="cuda").manual_seed(4321 + r)
    x = torch.randn(n, device="cuda", dtype=torch.bfloat16, generator=g)
    part = x[: n // ws].contiguous()

    def timed(fn, iters=5):
        out = fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        return out, s.elapsed_time(e) / iters

    everyone = C.all_gather(x, group=group).view(ws, n).float()   # fp32 reference sum
    ref = everyone.sum(0)
    ar_x, t_ar_x = timed(lambda: comm.all_reduce(x, out=torch.empty_like(x)))
    _, t_ar_r = timed(lambda: C.all_reduce(x.clone(), group=group))
    ag_x, t_ag_x = timed(lambda: comm.all_gather(part))
    ag_r, t_ag_r = timed(lambda: C.all_gather(part, group=group))
    rs_x, t_rs_x = timed(lambda: comm.reduce_scatter(x))
    rs_r, t_rs_r = timed(lambda: C.reduce_scatter(x, group=group))
    # the one-shot kernel (messages <= 512 KiB: vocab-parallel CE and norm all-reduces) is a
    # different code path from the two-shot one the run-size probe exercises: check it too
    ns = min(n, (256 << 10) // 2 // (8 * ws) * (8 * ws))
    xs = x[:ns].contiguous()
    ar_s = comm.all_reduce(xs, out=torch.empty_like(xs))
    ref_s = everyone[:, :ns].sum(0)
    comm.check()
    tol = ref.abs() * 2.0 ** -8 + 1e-6  # one bf16 rounding of the exact (fp32) sum
    ar_ok = bool(((ar_x.float() - ref).abs() <= tol).all())
    ar_ok = ar_ok and bool(((ar_s.float() - ref_s).abs() <= ref_s.abs() * 2.0 ** -8 + 1e-6).all())
    chunk = n // ws
    rs_ok = bool(((rs_x.float() - ref[r * chunk:(r + 1) * chunk]).abs() <= tol[r * chunk:(r + 1) * chunk]).all())
    ag_ok = bool(torch.equal(ag_x, ag_r))
    # ranks sharing ONE GPU (ST_GPU_OVERSUBSCRIBE=1: rehearsals / tests) time-slice it, so
    # neither timing means anything there: the verdict is correctness alone
    import os

    shared = os.environ.get("ST_GPU_OVERSUBSCRIBE", "0") == "1"
    per_op = {"all_reduce": int(ar_ok and (shared or t_ar_x < t_ar_r)),
              "all_gather": int(ag_ok and (shared or t_ag_x < t_ag_r)),
              "reduce_scatter": int(rs_ok and (shared or t_rs_x < t_rs_r))}
    info = {"msg_mb": round(2 * n / (1 << 20), 2), "world": ws,
            "ar_ms": [round(t_ar_x, 3), round(t_ar_r, 3)], "ag_ms": [round(t_ag_x, 3), round(t_ag_r, 3)],
            "rs_ms": [round(t_rs_x, 3), round(t_rs_r, 3)],
            "small_ar_kib": round(2 * ns / 1024, 1),
            "correct": {"all_reduce": ar_ok, "all_gather": ag_ok, "reduce_scatter": rs_ok}, "local": per_op,
            "timing": "ignored (ranks share one GPU)" if shared else "xgmi kept only where faster"}
    return per_op, info


def _pair_selftest(pair, group, probe_mb: int):
    """(1 if the pair path is correct and faster than RCCL else 0, timings)."""
    n = (probe_mb << 20) // 2
    r = C.get_rank(group)
    g = torch.Generator(device="cuda").manual_seed(1234 + r)
    x = torch.randn(n // 2, device="cuda", dtype=torch.bfloat16, generator=g)
    big = torch.randn(n, device="cuda", dtype=torch.bfloat16, generator=g)

    def timed(fn, iters=5):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            out = fn()
        e.record()
        e.synchronize()
        return out, s.elapsed_time(e) / iters

    ag_x, t_ag_x = timed(lambda: pair.all_gather(x))
    ag_r, t_ag_r = timed(lambda: C.all_gather(x, group=group))
    rs_x, t_rs_x = timed(lambda: pair.reduce_scatter(big))
    rs_r, t_rs_r = timed(lambda: C.reduce_scatter(big, group=group))
    pair.comm.check()
    same_ag = bool(torch.equal(ag_x, ag_r))
    err_rs = float(((rs_x.float() - rs_r.float()).abs() / (rs_r.float().abs() + 1e-3)).max())
    info = {"probe_mb": probe_mb, "ag_ms": [round(t_ag_x, 3), round(t_ag_r, 3)],
            "rs_ms": [round(t_rs_x, 3), round(t_rs_r, 3)], "ag_bitwise": same_ag, "rs_max_rel_err": round(err_rs, 5)}
    good = same_ag and err_rs < 1e-2 and t_ag_x < t_ag_r and t_rs_x < t_rs_r
    return (1 if good else 0), info


class _StreamWork:
    """Async handle for an all-reduce issued on a side stream."""

    def __init__(self, stream):
        self.ev = torch.cuda.Event()
        self.ev.record(stream)

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


def _tp_all_reduce(x: torch.Tensor, group, async_op: bool = False):
    """Sum over the TP group; returns a handle with ``wait()`` when ``async_op``."""
    from ..dist import trace

    comm = _xgmi_comm(group, "all_reduce") if x.is_cuda else None
    if comm is not None and not comm.supports(x):
        comm = None  # too large for the IPC area / unaligned: RCCL
    trace.record("tp.all_reduce", x, group_size=_ws(group), transport="xgmi" if comm is not None else "rccl",
                 overlapped=async_op)
    if comm is not None:
        # every xGMI collective of the process runs on ONE stream (``_on_comm_stream``); an
        # async one (the column-parallel dX all-reduce) runs there under the dW GEMM
        work = _on_comm_stream(lambda t: comm.all_reduce(t), x)[1]
        if not async_op:
            work.wait()
            return None
        return work
    return C.all_reduce(x, group=group, async_op=async_op)


def _xgmi_comm(group, op: str | None = None):
    """The xGMI communicator of ``group`` when the xGMI TP transport is active and (``op``
    given) that collective kept the xGMI path at start-up; else None (RCCL)."""
    if _TP_COMM != "xgmi" or group is None or _ws(group) == 1:
        return None
    if op is not None and not _TP_XGMI_OPS.get(op, False):
        return None
    from ..dist.xgmi import XgmiAllReduce

    comm = _XGMI.get(id(group))
    if comm is None:
        comm = _XGMI[id(group)] = XgmiAllReduce(group)
    return comm


def check_xgmi() -> None:
    """Raise if any xGMI collective of this process timed out (one host sync per
    communicator; the trainer polls it at logging steps -- ADVICE r1)."""
    for comm in list(_XGMI.values()):
        comm.check()
    if _PAIR[0] is not None:
        _PAIR[0].comm.check()


class CopyToTensorParallelRegion(torch.autograd.Function):
    """Megatron ``f``: identity forward, all-reduce backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        if _ws(ctx.group) > 1:
            g = g.contiguous()
            _tp_all_reduce(g, ctx.group)
        return g, None


class ReduceFromTensorParallelRegion(torch.autograd.Function):
    """Megatron ``g``: all-reduce forward, identity backward."""

    @staticmethod
    def forward(ctx, x, group):
        if _ws(group) == 1:
            return x
        x = x.contiguous()
        _tp_all_reduce(x, group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class GatherFromTensorParallelRegion(torch.autograd.Function):
    """All-gather along the last dim forward, keep own slice backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        ws = _ws(group)
        if ws == 1:
            return x
        parts = C.all_gather(x.contiguous(), group=group, as_list=True)
        return torch.cat(parts, dim=-1)

    @staticmethod
    def backward(ctx, g):
        ws = _ws(ctx.group)
        if ws == 1:
            return g, None
        return g.chunk(ws, dim=-1)[C.get_rank(ctx.group)].contiguous(), None


class ScatterToTensorParallelRegion(torch.autograd.Function):
    """Keep own last-dim slice forward, all-gather backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        ws = _ws(group)
        if ws == 1:
            return x
        return x.chunk(ws, dim=-1)[C.get_rank(group)].contiguous()

    @staticmethod
    def backward(ctx, g):
        ws = _ws(ctx.group)
        if ws == 1:
            return g, None
        return torch.cat(C.all_gather(g.contiguous(), group=ctx.group, as_list=True), dim=-1), None


def _trace(op: str, x: torch.Tensor, ws: int, transport: str | None = None) -> None:
    from ..dist import trace

    trace.record(op, x, group_size=ws, transport=transport)


def _gather_seq(x: torch.Tensor, group) -> torch.Tensor:
    """[B, S/tp, ...] -> [B, S, ...] (one all_gather_into_tensor; zero-copy when B == 1)."""
    ws = _ws(group)
    if ws == 1:
        return x
    xg = _xgmi_comm(group, "all_gather") if x.is_cuda else None
    pair = _PAIR[0] if (xg is not None and ws == 2) else None
    if pair is not None and pair.fits(x.numel(), x):
        xg = pair  # multipath: direct link + 2-hop relays
    _trace("sp.all_gather", x, ws, "xgmi" if xg is not None and (xg is pair or xg.supports(x)) else None)
    gather = _synced(xg.all_gather) if xg is not None else (lambda t: C.all_gather(t, group=group))
    if x.shape[0] == 1:
        return gather(x[0].contiguous()).unsqueeze(0)
    xt = x.transpose(0, 1).contiguous()  # [S/tp, B, ...]
    return gather(xt).transpose(0, 1).contiguous()


def _reduce_scatter_seq(x: torch.Tensor, group) -> torch.Tensor:
    """[B, S, ...] summed over ranks -> [B, S/tp, ...]."""
    ws = _ws(group)
    if ws == 1:
        return x
    xg = _xgmi_comm(group, "reduce_scatter") if x.is_cuda else None
    pair = _PAIR[0] if (xg is not None and ws == 2) else None
    if pair is not None and pair.fits(x.numel() // 2, x):
        xg = pair  # multipath: direct link + 2-hop relays
    _trace("sp.reduce_scatter", x, ws, "xgmi" if xg is not None and (xg is pair or xg.supports(x)) else None)
    scatter = _synced(xg.reduce_scatter) if xg is not None else (lambda t: C.reduce_scatter(t, group=group))
    if x.shape[0] == 1:
        return scatter(x[0].contiguous()).unsqueeze(0)
    xt = x.transpose(0, 1).contiguous()
    return scatter(xt).transpose(0, 1).contiguous()


def _gather_seq_async(x: torch.Tensor, group):
    """Issue the sequence all-gather; returns ``finish() -> [B, S, ...]`` (waits on first call).
    RCCL async, or the xGMI pair path on its comm side stream (``_sp_gather_async``)."""
    ws = _ws(group)
    if ws == 1:
        return lambda: x
    B = x.shape[0]
    xt = x[0].contiguous() if B == 1 else x.transpose(0, 1).contiguous()
    out, work = _sp_gather_async(xt, group)

    def finish():
        work.wait()
        return out.unsqueeze(0) if B == 1 else out.transpose(0, 1).contiguous()
    return finish


def _reduce_scatter_seq_async(x: torch.Tensor, group):
    """Issue the sequence reduce-scatter; returns ``finish() -> [B, S/tp, ...]``."""
    ws = _ws(group)
    if ws == 1:
        return lambda: x
    B = x.shape[0]
    xt = x[0].contiguous() if B == 1 else x.transpose(0, 1).contiguous()
    out, work = _sp_reduce_scatter_async(xt, group)

    def finish():
        work.wait()
        return out.unsqueeze(0) if B == 1 else out.transpose(0, 1).contiguous()
    return finish


def _split_seq(x: torch.Tensor, group) -> torch.Tensor:
    ws = _ws(group)
    if ws == 1:
        return x
    return x.chunk(ws, dim=1)[C.get_rank(group)].contiguous()


class AllGatherFromSequenceParallelRegion(torch.autograd.Function):
    """All-gather along seq forward, reduce-scatter backward (reference sp_comms.py:31-61)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _gather_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return _reduce_scatter_seq(g, ctx.group), None


class ReduceScatterToSequenceParallelRegion(torch.autograd.Function):
    """Reduce-scatter along seq forward, all-gather backward (reference sp_comms.py:64-94)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _reduce_scatter_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return _gather_seq(g, ctx.group), None


class ScatterToSequenceParallelRegion(torch.autograd.Function):
    """Split along seq forward (no comm), all-gather backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _split_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return _gather_seq(g, ctx.group), None


# ====================================================================== linear with overlapped TP grad all-reduce
class _ColumnParallelFn(torch.autograd.Function):
    """y = x W^T (+b) where x is replicated on the TP group.

    Backward: dX = dY W is all-reduced over TP asynchronously while the dW GEMM
    (accumulated into ``main_grad``) runs -- reference LinearWithAsyncAllReduce,
    scaletorch/parallel/tensor_parallel/tp_comms.py:229-320.
    """

    @staticmethod
    def forward(ctx, x, weight, bias, group, link=None):
        ctx.save_for_backward(x, weight)
        ctx.group, ctx.bias, ctx.link = group, bias, link
        if x.requires_grad:
            prepare_dgrad_weight(weight)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        link = ctx.link
        if link is not None and link.event is not None:
            return _ColumnParallelFn._backward_split(ctx, dy, dy2, x2, weight, link)
        pre = prefetch_wgrad(weight, dy2, x2) if ctx.needs_input_grad[1] else None  # overlaps the dgrad GEMM
        dx = dgrad(dy, weight)
        handle = None
        if _ws(ctx.group) > 1:
            handle = _tp_all_reduce(dx, ctx.group, async_op=True)
        dw = accumulate_linear_wgrad(weight, dy2, x2, pre) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.bias is not None and ctx.needs_input_grad[2]:
            db = accumulate_grad(ctx.bias, dy2.float().sum(0))
        if handle is not None:
            handle.wait()
        return dx, dw, db, None, None

    @staticmethod
    def _backward_split(ctx, dy, dy2, x2, weight, link):
        """QKV projection backward while the attention's dQ pass still runs on a side
        stream (ops.attention.DQLink, TP = 1): the k/v columns' data gradient and weight
        gradient first, then wait for dQ and add the q columns' (same bf16 GEMMs and fp32
        main_grad epilogues as the one-shot path, split at a column boundary)."""
        from ..ops.grad import _WT_EPOCH, _grad_ready, take_fresh, wgrad_into

        c = link.split
        wt = weight._st_wt if (getattr(weight, "_st_wt_epoch", -1) == _WT_EPOCH[0] and dy.is_cuda) else None
        if wt is not None:
            torch.cuda.current_stream().wait_event(weight._st_wt_done)
        mg = getattr(weight, "main_grad", None)
        want_w = ctx.needs_input_grad[1]
        beta = (0 if take_fresh(weight) else 1) if (want_w and mg is not None) else None

        def dgrad_part(lo, hi, out=None):
            b = wt[:, lo:hi].t() if wt is not None else weight[lo:hi]  # TN on the W^T copy's column block
            return out.addmm_(dy2[:, lo:hi], b) if out is not None else dy2[:, lo:hi] @ b

        def wgrad_part(lo, hi):
            if beta is not None:
                wgrad_into(mg.view(mg.shape[0], -1)[lo:hi], dy2[:, lo:hi], x2, beta)

        n = dy2.shape[1]
        dx = dgrad_part(c, n)
        wgrad_part(c, n)
        link.wait()  # dQ (and its inverse RoPE) landed
        dgrad_part(0, c, out=dx)
        wgrad_part(0, c)
        dw = None
        if want_w:
            if mg is not None:
                _grad_ready(weight)
            else:
                dw = dy2.t().mm(x2)
        db = None
        if ctx.bias is not None and ctx.needs_input_grad[2]:
            db = accumulate_grad(ctx.bias, dy2.float().sum(0))
        return dx.view(*dy.shape[:-1], dx.shape[-1]), dw, db, None, None


def _sp_overlap(x: torch.Tensor) -> bool:
    """Pipelined SP forward (ST_SP_OVERLAP=0: one blocking collective + one GEMM, A/B).
    Composes with the xGMI pair path: its collectives run on a comm side stream."""
    import os

    return os.environ.get("ST_SP_OVERLAP", "1") == "1"


def _sp_chunks(Sp: int, tokens: int) -> int:
    """Sequence sub-chunks of a rank's shard in the pipelined SP forward (ST_SP_CHUNKS overrides)."""
    import os

    env = os.environ.get("ST_SP_CHUNKS")
    c = max(1, int(env)) if env else (2 if tokens >= 8192 else 1)
    while c > 1 and Sp % c:
        c -= 1
    return c


def _rows_gemm(x2: torch.Tensor, weight: torch.Tensor, out: torch.Tensor) -> None:
    torch.matmul(x2, weight.t(), out=out)


def _bmm_into(x3: torch.Tensor, b2: torch.Tensor, out3: torch.Tensor, mode: str | None = None) -> None:
    """``out3[b] = x3[b] @ b2`` for every batch element; ``x3`` [B, M, K] and ``out3`` [B, M, N]
    may be sequence slices of larger [B, S, .] tensors (batch stride != M * row stride).

    ``fold`` (default): ONE [B*M, K] x [K, N] GEMM -- the input slice is gathered into a
    contiguous buffer when it is strided, the output written in place when contiguous,
    else through one strided copy; ``loop``: one 2-D GEMM per batch element straight
    on the strided views (the round-3 form).  ``tools/bench_sp_gemm.py`` times both
    against the unsplit GEMM at the tp2pp2dp2 shapes (profiles/r04/).  Only plain 2-D
    GEMMs are issued: a strided-batched torch.bmm with a stride-0 weight and a strided
    output faulted on ROCm 7 here (illegal address), so it is not used."""
    import os

    B, M, K = x3.shape
    if B == 1:
        torch.matmul(x3[0], b2, out=out3[0])
        return
    mode = mode or os.environ.get("ST_SP_GEMM", "fold")
    if mode == "loop":
        for b in range(B):
            torch.matmul(x3[b], b2, out=out3[b])
        return
    x2 = x3.reshape(B * M, K)
    if out3.is_contiguous():
        torch.matmul(x2, b2, out=out3.view(B * M, out3.shape[-1]))
    else:
        out3.copy_(torch.matmul(x2, b2).view(B, M, out3.shape[-1]))


def _dgrad_b2(weight: torch.Tensor) -> torch.Tensor:
    """[out, in] right operand of dX = dY W: the TN view of the current W^T copy when
    one exists (ops/grad.py ``prepare_dgrad_weight``), else the weight itself."""
    from ..ops.grad import _WT_EPOCH

    if getattr(weight, "_st_wt_epoch", -1) == _WT_EPOCH[0] and weight.is_cuda:
        torch.cuda.current_stream().wait_event(weight._st_wt_done)
        return weight._st_wt.t()
    return weight


def _sp_gather_async(part: torch.Tensor, group):
    """Issue the all-gather of one SP sub-chunk ([B, Sc, h] -> [ws*B, Sc, h], rank-major);
    returns (buffer, work).  Over the xGMI pair path (tp = 2, --tp_comm xgmi) it runs on
    the comm side stream, so it overlaps the GEMMs exactly like the RCCL one."""
    ws = _ws(group)
    pair = _pair_for(group, part.numel(), part)
    if pair is not None:
        return _on_comm_stream(pair.all_gather, part)
    xg = _xgmi_comm(group, "all_gather") if (part.is_cuda and ws > 2) else None
    if xg is not None and xg.supports(part):  # tp 4 / 8: all 7 links, on the comm side stream
        _trace("sp.all_gather", part, ws, "xgmi")
        return _on_comm_stream(xg.all_gather, part.contiguous())
    _trace("sp.all_gather", part, ws)
    return C.all_gather(part, group=group, async_op=True)


def _sp_reduce_scatter_async(buf: torch.Tensor, group):
    """Issue the reduce-scatter of one SP sub-chunk ([ws*B, Sc, o] -> [B, Sc, o]);
    returns (output, work) -- xGMI pair path on the comm side stream, else RCCL."""
    ws = _ws(group)
    pair = _pair_for(group, buf.numel() // 2, buf)
    if pair is not None:
        return _on_comm_stream(pair.reduce_scatter, buf)
    xg = _xgmi_comm(group, "reduce_scatter") if (buf.is_cuda and ws > 2) else None
    if xg is not None and buf.is_contiguous() and xg.supports(buf) and buf.shape[0] % ws == 0:
        _trace("sp.reduce_scatter", buf, ws, "xgmi")
        return _on_comm_stream(xg.reduce_scatter, buf)
    _trace("sp.reduce_scatter", buf, ws)
    return C.reduce_scatter(buf, group=group, async_op=True)


def _pair_for(group, n_elems: int, t: torch.Tensor):
    """The 2-rank xGMI multipath transport for this SP message, or None (RCCL)."""
    if not t.is_cuda or _ws(group) != 2 or _xgmi_comm(group, "all_gather") is None:
        return None
    pair = _PAIR[0]
    if pair is None or not pair.fits(n_elems, t):
        return None
    from ..dist import trace

    trace.record("sp.pair", t, group_size=2, transport="xgmi-pair")
    return pair


_COMM_STREAMS: dict = {}


def _comm_stream(device: torch.device):
    """(side stream of the xGMI SP collectives, event of the current stream's position):
    the collective starts once the producer of its input has finished."""
    st = _COMM_STREAMS.get(device.index)
    if st is None:
        st = _COMM_STREAMS[device.index] = torch.cuda.Stream(device=device)
    ready = torch.cuda.Event()
    ready.record()
    return st, ready


def _on_comm_stream(fn, t: torch.Tensor):
    """Run the xGMI collective ``fn(t)`` on the comm stream once the current stream has
    produced ``t``; returns (output, work).  EVERY xGMI collective of the process (TP
    all-reduce, SP all-gather / reduce-scatter, pair path, sync or async) goes through
    this one stream: the IPC protocol's epoch-parity buffers assume the group's
    collectives run one after another in issue order, which two streams would not keep
    (an async reduce-scatter still in flight beside a synchronous all-gather issued on
    the compute stream deadlocked the pair path)."""
    st, ready = _comm_stream(t.device)
    with torch.cuda.stream(st):
        st.wait_event(ready)
        out = fn(t)
    t.record_stream(st)
    if isinstance(out, torch.Tensor) and out.data_ptr() != t.data_ptr():
        out.record_stream(torch.cuda.current_stream())
    return out, _StreamWork(st)


def _synced(fn):
    """``fn`` (an xGMI collective) on the comm stream, the current stream waiting for it."""
    def run(t):
        out, work = _on_comm_stream(fn, t)
        work.wait()
        return out
    return run


def _sp_column_forward(x_shard: torch.Tensor, weight: torch.Tensor, group) -> torch.Tensor:
    """y[B, S, out] = all_gather_seq(x_shard) W^T with the gather hidden behind GEMMs:
    the sequence all-gathers are issued first (async, in ``c`` sub-chunks), the rows of
    this rank's OWN shard are multiplied while they are in flight, then each sub-chunk's
    peer rows as soon as that sub-chunk has landed.  Every GEMM is ONE strided-batched
    product over all B sequences writing its rows of y in place (no assembly copy).
    Reference: AllGatherFromSequenceParallelRegion + a column linear,
    scaletorch/parallel/sequence_parallel/sp_comms.py:31-61 (serialised)."""
    ws, r = _ws(group), C.get_rank(group)
    B, Sp, _ = x_shard.shape
    c = _sp_chunks(Sp, B * Sp * ws)
    Sc = Sp // c
    xs = x_shard.contiguous()
    gathers = []
    for q in range(c):
        part = xs[:, q * Sc:(q + 1) * Sc]
        part = part.contiguous() if (c > 1 and B > 1) else part
        gathers.append(_sp_gather_async(part, group))  # [ws*B, Sc, h], rank-major
    y = torch.empty(B, Sp * ws, weight.shape[0], dtype=x_shard.dtype, device=x_shard.device)
    wt = weight.t()
    _bmm_into(xs, wt, y[:, r * Sp:(r + 1) * Sp])  # own rows: no communication needed
    for q, (buf, work) in enumerate(gathers):
        work.wait()
        for j in range(ws):
            if j != r:
                _bmm_into(buf[j * B:(j + 1) * B], wt, y[:, j * Sp + q * Sc: j * Sp + (q + 1) * Sc])
    return y


class _SPColumnParallelFn(torch.autograd.Function):
    """Sequence-parallel column linear: all-gather x along seq, GEMM -- pipelined
    (``_sp_column_forward``).

    Backward (every collective async, each hidden behind a GEMM): the re-gather
    of x is issued first and runs under the dX = dY W GEMM; the reduce-scatter
    of dX is issued next and runs under the dW GEMM (accumulated into
    main_grad).  The gathered input is NOT saved (Megatron's memory/traffic
    trade-off: an all-gather of [B,S,h] in backward instead of keeping it).
    Reference: sp_comms.py:31-61 + tp_comms.py:288-311 (which serialised them).
    """

    @staticmethod
    def forward(ctx, x_shard, weight, bias, group):
        ctx.save_for_backward(x_shard, weight)
        ctx.group, ctx.bias = group, bias
        if x_shard.requires_grad:
            prepare_dgrad_weight(weight)
        if _ws(group) > 1 and _sp_overlap(x_shard):
            y = _sp_column_forward(x_shard, weight, group)
            return y + bias if bias is not None else y
        xg = _gather_seq(x_shard, group)
        return F.linear(xg, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x_shard, weight = ctx.saved_tensors
        gather = _gather_seq_async(x_shard, ctx.group) if ctx.needs_input_grad[1] else None
        dx_full = dgrad(dy, weight)                           # overlaps the all-gather
        scatter = _reduce_scatter_seq_async(dx_full, ctx.group)
        dy2 = dy.reshape(-1, dy.shape[-1])
        dw = None
        if gather is not None:
            xg = gather()
            dw = accumulate_linear_wgrad(weight, dy2, xg.reshape(-1, xg.shape[-1]))  # overlaps the RS
        db = None
        if ctx.bias is not None and ctx.needs_input_grad[2]:
            db = accumulate_grad(ctx.bias, dy2.float().sum(0))
        return scatter(), dw, db, None


def _swiglu_fwd(gu: torch.Tensor) -> torch.Tensor:
    from ..ops import _lib

    if gu.is_cuda and _lib.use_native(gu) and gu.dtype == torch.bfloat16:
        return _lib.ops().swiglu_fwd(gu.contiguous())
    g, u = gu.chunk(2, dim=-1)
    return F.silu(g) * u


def _swiglu_bwd(da: torch.Tensor, gu: torch.Tensor) -> torch.Tensor:
    from ..ops import _lib

    if gu.is_cuda and _lib.use_native(gu) and gu.dtype == torch.bfloat16:
        return _lib.ops().swiglu_bwd(da.contiguous(), gu.contiguous())
    g, u = gu.float().chunk(2, dim=-1)
    sg = torch.sigmoid(g)
    d = da.float()
    return torch.cat([d * u * (sg + g * sg * (1 - sg)), d * g * sg], dim=-1).to(gu.dtype)


def _peer_ranges(ws: int, r: int) -> list[tuple[int, int]]:
    """Contiguous ranges of peer ranks (everyone but r): at most two."""
    return [(a, b) for a, b in ((0, r), (r + 1, ws)) if b > a]


def _wgrad_pieces(weight: torch.Tensor, pieces) -> torch.Tensor | None:
    """dW = sum_p dy_p^T x_p straight into ``weight.main_grad`` (the first piece overwrites a
    fresh accumulator, the rest add; ONE grad-ready signal), or returned for autograd."""
    from ..ops.grad import _grad_ready, take_fresh, wgrad_into

    mg = getattr(weight, "main_grad", None)
    if mg is None:
        dw = None
        for dy2, x2 in pieces:
            p = dy2.t().mm(x2)
            dw = p if dw is None else dw + p
        return dw
    fresh = take_fresh(weight)
    m2 = mg.view(mg.shape[0], -1)
    for i, (dy2, x2) in enumerate(pieces):
        wgrad_into(m2, dy2, x2, 0 if (fresh and i == 0) else 1)
    _grad_ready(weight)
    return None


class _SPMLPFn(torch.autograd.Function):
    """The whole sequence-parallel SwiGLU MLP (gate|up column GEMM -> SwiGLU -> down row
    GEMM) in the GATHERED layout: the intermediate rows are kept in the order the
    sequence all-gather delivers them, [sub-chunk q][rank j][sequence b][Sc rows],
    instead of [b][S].  Every GEMM piece is then one contiguous 2-D product over all B
    sequences -- the gate|up rows of (q, j) land in one block, the down projection of
    sub-chunk q is ONE [ws*B*Sc] GEMM that writes its reduce-scatter buffer directly --
    with no strided writes, no per-sequence loops and no layout copies; only the [B, Sp]
    shard at the ends is in sequence order.  The gather of sub-chunk q+1 and the
    reduce-scatter of sub-chunk q overlap the GEMMs (RCCL async, or the xGMI pair path on
    its comm side stream).  Backward re-gathers x and gathers dY per sub-chunk (same
    layout), runs dgrad -> SwiGLU backward -> dgrad per sub-chunk with each dX
    reduce-scatter in flight under the next, and accumulates both weight gradients over
    the sub-chunks into main_grad.  Reference: the Llama MLP with
    AllGather/ReduceScatterFromSequenceParallelRegion around it,
    scaletorch/models/llama.py:236-249, scaletorch/parallel/sequence_parallel/sp_comms.py:31-94."""

    @staticmethod
    def forward(ctx, x_shard, w_gu, w_dn, group):
        ws, r = _ws(group), C.get_rank(group)
        B, Sp, h = x_shard.shape
        c = _sp_chunks(Sp, B * Sp * ws)
        Sc = Sp // c
        n2, I = w_gu.shape[0], w_dn.shape[1]
        if x_shard.requires_grad:
            prepare_dgrad_weight(w_gu)
            prepare_dgrad_weight(w_dn)
        xs = x_shard.contiguous()
        parts = [xs[:, q * Sc:(q + 1) * Sc].contiguous() if c > 1 else xs for q in range(c)]
        gathers = [_sp_gather_async(p, group) for p in parts]  # [ws*B, Sc, h] each, rank-major
        gu = torch.empty(c, ws, B * Sc, n2, dtype=xs.dtype, device=xs.device)
        wgu_t, wdn_t = w_gu.t(), w_dn.t()
        for q in range(c):  # own rows while the gathers are in flight
            torch.matmul(parts[q].view(B * Sc, h), wgu_t, out=gu[q, r])
        y = torch.empty(B, Sp, h, dtype=xs.dtype, device=xs.device)
        scatters, acts = [], []
        for q, (buf, work) in enumerate(gathers):
            work.wait()
            for j0, j1 in _peer_ranges(ws, r):
                torch.matmul(buf[j0 * B:j1 * B].reshape(-1, h), wgu_t, out=gu[q, j0:j1].view(-1, n2))
            a_q = _swiglu_fwd(gu[q]).view(-1, I)  # [ws*B*Sc, I]: kept for the down weight gradient
            acts.append(a_q)
            rs_in = torch.matmul(a_q, wdn_t).view(ws * B, Sc, h)
            scatters.append(_sp_reduce_scatter_async(rs_in, group))  # -> [B, Sc, h]
        for q, (out, work) in enumerate(scatters):
            work.wait()
            y[:, q * Sc:(q + 1) * Sc] = out
        ctx.save_for_backward(xs, gu, w_gu, w_dn, *acts)
        ctx.group, ctx.c = group, c
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, gu, w_gu, w_dn = ctx.saved_tensors[:4]
        acts = ctx.saved_tensors[4:]
        group, c = ctx.group, ctx.c
        ws = _ws(group)
        B, Sp, h = xs.shape
        Sc = Sp // c
        n2, I = w_gu.shape[0], w_dn.shape[1]
        dys = dy.contiguous()
        dgathers = [_sp_gather_async(dys[:, q * Sc:(q + 1) * Sc].contiguous() if c > 1 else dys, group)
                    for q in range(c)]
        xgathers = [_sp_gather_async(xs[:, q * Sc:(q + 1) * Sc].contiguous() if c > 1 else xs, group)
                    for q in range(c)]
        b_dn, b_gu = _dgrad_b2(w_dn), _dgrad_b2(w_gu)  # [h, I] and [2I, h] right operands
        dx = torch.empty(B, Sp, h, dtype=dys.dtype, device=dys.device)
        scatters, dn_pieces, dgus = [], [], []
        for q, (dbuf, work) in enumerate(dgathers):
            work.wait()
            dY = dbuf.reshape(-1, h)
            da = torch.matmul(dY, b_dn)  # [ws*B*Sc, I]
            dgu_q = _swiglu_bwd(da, gu[q].view(-1, n2))
            dgus.append(dgu_q)
            dn_pieces.append((dY, acts[q]))
            dxf = torch.matmul(dgu_q, b_gu).view(ws * B, Sc, h)
            scatters.append(_sp_reduce_scatter_async(dxf, group))
        dw_dn = _wgrad_pieces(w_dn, dn_pieces) if ctx.needs_input_grad[2] else None
        gu_pieces = []
        for q, (xbuf, work) in enumerate(xgathers):
            work.wait()
            gu_pieces.append((dgus[q], xbuf.reshape(-1, h)))
        dw_gu = _wgrad_pieces(w_gu, gu_pieces) if ctx.needs_input_grad[1] else None
        for q, (out, work) in enumerate(scatters):
            work.wait()
            dx[:, q * Sc:(q + 1) * Sc] = out
        return dx, dw_gu, dw_dn, None


def sp_mlp_applies(mlp, x: torch.Tensor) -> bool:
    """The gathered-layout SP MLP takes this call: TP > 1 with sequence parallelism,
    bias-free projections, a [B, Sp, h] shard, training with gradients
    (``ST_SP_MLP=0``: the per-projection SP path, A/B)."""
    import os

    gu, dn = mlp.gate_up_proj, mlp.down_proj
    return (gu.tp > 1 and gu.sequence_parallel and dn.sequence_parallel and gu.bias is None and dn.bias is None
            and x.dim() == 3 and torch.is_grad_enabled() and os.environ.get("ST_SP_MLP", "1") == "1"
            and _sp_overlap(x))


def sp_mlp(x_shard: torch.Tensor, w_gu: torch.Tensor, w_dn: torch.Tensor, group) -> torch.Tensor:
    return _SPMLPFn.apply(x_shard, w_gu, w_dn, group)


class _SPRowParallelFn(torch.autograd.Function):
    """Sequence-parallel row linear: y_shard = reduce_scatter_seq(x W^T), pipelined.

    Forward: the output sequence is cut into ``c`` sub-chunks per rank shard; the
    GEMMs of sub-chunk q (every rank's rows of it) write straight into that
    sub-chunk's reduce-scatter buffer and its reduce-scatter is issued async, so it
    runs while sub-chunk q+1's GEMMs compute -- only the last one is exposed.
    Backward: the all-gather of dY is issued async and dX for this rank's OWN rows
    is computed from the local shard under it; the peer rows follow, then dW over
    the whole sequence into main_grad.  Reference: ReduceScatterToSequenceParallelRegion
    after RowParallelLinear (sp_comms.py:64-94, tensor_parallel.py:352-362)."""

    @staticmethod
    def forward(ctx, x, weight, group):
        ctx.save_for_backward(x, weight)
        ctx.group = group
        if x.requires_grad:
            prepare_dgrad_weight(weight)
        ws = _ws(group)
        B, S, _ = x.shape
        Sp = S // ws
        c = _sp_chunks(Sp, B * S)
        Sc = Sp // c
        out_f = weight.shape[0]
        x = x.contiguous()
        wt = weight.t()
        pending = []
        for q in range(c):
            buf = torch.empty(ws * B, Sc, out_f, dtype=x.dtype, device=x.device)
            for j in range(ws):  # every sequence's rows of (peer j, sub-chunk q): one batched GEMM
                _bmm_into(x[:, j * Sp + q * Sc: j * Sp + (q + 1) * Sc], wt, buf[j * B:(j + 1) * B])
            pending.append(_sp_reduce_scatter_async(buf, group))  # -> [B, Sc, out]
        if c == 1:
            out, work = pending[0]
            work.wait()
            return out
        y = torch.empty(B, Sp, out_f, dtype=x.dtype, device=x.device)
        for q, (out, work) in enumerate(pending):
            work.wait()
            y[:, q * Sc:(q + 1) * Sc] = out
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        group = ctx.group
        ws, r = _ws(group), C.get_rank(group)
        B, Sp, out_f = dy.shape
        S = Sp * ws
        dys = dy.contiguous()
        buf, work = _sp_gather_async(dys, group)  # [ws*B, Sp, out], rank-major
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(B, S, weight.shape[1], dtype=dy.dtype, device=dy.device)
            b2 = _dgrad_b2(weight)
            _bmm_into(dys, b2, dx[:, r * Sp:(r + 1) * Sp])  # own rows under the gather
        work.wait()
        if dx is not None:
            for j in range(ws):
                if j != r:
                    _bmm_into(buf[j * B:(j + 1) * B], b2, dx[:, j * Sp:(j + 1) * Sp])
        dw = None
        if ctx.needs_input_grad[1]:
            if B == 1:
                dyf = buf.view(S, out_f)  # rank-major == sequence order
            else:
                dyf = buf.view(ws, B, Sp, out_f).transpose(0, 1).reshape(B * S, out_f)
            dw = accumulate_linear_wgrad(weight, dyf, x.reshape(-1, x.shape[-1]))
        return dx, dw, None


def _ar_chunks(tokens: int) -> int:
    """Token chunks of the row-parallel forward (ST_TP_AR_CHUNKS overrides)."""
    import os

    env = os.environ.get("ST_TP_AR_CHUNKS")
    if env:
        return max(1, int(env))
    return 4 if tokens >= 8192 else (2 if tokens >= 2048 else 1)


class _RowParallelFn(torch.autograd.Function):
    """y = all_reduce(x W^T) over TP with the all-reduce PIPELINED against the GEMM:
    the tokens are split into chunks, and chunk i's all-reduce (async, RCCL
    stream / xGMI side stream) runs while chunk i+1's GEMM computes, so only the
    last chunk's all-reduce is exposed.  Backward needs no communication (dY is
    replicated): dX = dY W and dW = dY^T X into main_grad.
    Reference: RowParallelLinear + ReduceFromModelParallelRegion
    (tensor_parallel.py:352-362, tp_comms.py:140-153), a blocking all-reduce."""

    @staticmethod
    def forward(ctx, x, weight, group):
        ctx.save_for_backward(x, weight)
        if x.requires_grad:
            prepare_dgrad_weight(weight)
        x2 = x.reshape(-1, x.shape[-1])
        T = x2.shape[0]
        n = _ar_chunks(T)
        y = torch.empty(T, weight.shape[0], dtype=x.dtype, device=x.device)
        works = []
        bounds = [T * i // n for i in range(n + 1)]
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            if hi > lo:
                yc = y[lo:hi]
                torch.matmul(x2[lo:hi], weight.t(), out=yc)
                works.append(_tp_all_reduce(yc, group, async_op=True))
        for w in works:
            if w is not None:
                w.wait()
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        pre = prefetch_wgrad(weight, dy2, x2) if ctx.needs_input_grad[1] else None  # overlaps the dgrad GEMM
        dx = dgrad(dy, weight) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            dw = accumulate_linear_wgrad(weight, dy2, x2, pre)
        return dx, dw, None


def _init_shard_(weight: torch.Tensor, init: str, std: float, fan_in: int) -> None:
    with torch.no_grad():
        if init == "normal":
            weight.normal_(0.0, std)
        else:  # reference _init_weights: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (attention_utils.py:160-167)
            bound = 1.0 / math.sqrt(fan_in)
            weight.uniform_(-bound, bound)


class ColumnParallelLinear(nn.Module):
    """Output features split over TP: weight [out/tp, in] (reference tensor_parallel.py:147-261)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False, gather_output: bool = False,
                 sequence_parallel: bool = False, init: str = "uniform", init_std: float = 0.02,
                 group=None):
        super().__init__()
        self.group = group if group is not None else mesh.tp_group()
        self.tp = _ws(self.group) if self.group is not None else 1
        if out_features % self.tp:
            raise ValueError(f"out_features {out_features} not divisible by tp {self.tp}")
        self.in_features, self.out_features = in_features, out_features
        self.out_per_rank = out_features // self.tp
        self.gather_output, self.sequence_parallel = gather_output, sequence_parallel
        self.init, self.init_std = init, init_std
        self.weight = nn.Parameter(torch.empty(self.out_per_rank, in_features))
        self.bias = nn.Parameter(torch.zeros(self.out_per_rank)) if bias else None
        self.reset_parameters()

    def _row_pieces(self) -> list[int]:
        return [self.out_features]

    def reset_parameters(self) -> None:
        from .init import init_full

        key = getattr(self, "_st_init_key", None)
        if key is None:
            _init_shard_(self.weight, self.init, self.init_std, self.in_features)
        else:
            full = init_full((self.out_features, self.in_features), self.init, self.init_std, self.in_features,
                             key, self.weight.device)
            r = C.get_rank(self.group) if self.tp > 1 else 0
            shards = [p.chunk(self.tp, dim=0)[r] for p in full.split(self._row_pieces(), dim=0)]
            with torch.no_grad():
                self.weight.copy_(torch.cat(shards, dim=0))
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, x: torch.Tensor, labels: torch.Tensor | None = None, chunk: int | None = None,
                grad_scale: float | None = None, act: str | None = None) -> torch.Tensor:
        """Logits shard ``[..., out/tp]``; with ``labels`` (LM head use) the mean
        vocab-parallel cross-entropy instead, fused and chunked so the logits are
        never materialised (ops/fused_head.py).  ``act="swiglu"`` (a fused gate|up weight,
        the caller checked ``ops.mlp.gate_up_swiglu_ok``): silu(gate) * up from ONE kernel.
        All run as a module call so the forward pre-hook (optimizer-bucket wait) precedes
        every read of the weight."""
        if act == "swiglu":
            from ..ops.mlp import gate_up_swiglu

            return gate_up_swiglu(x, self.weight)
        if labels is not None:
            from ..ops.fused_head import fused_linear_cross_entropy

            if self.bias is not None:
                raise ValueError("fused LM head + cross-entropy takes a bias-free projection")
            if self.sequence_parallel and self.tp > 1:
                x = AllGatherFromSequenceParallelRegion.apply(x, self.group)
            elif self.tp > 1:
                x = CopyToTensorParallelRegion.apply(x, self.group)
            vocab_start = C.get_rank(self.group) * self.out_per_rank if self.tp > 1 else 0
            return fused_linear_cross_entropy(x, self.weight, labels, vocab_start,
                                              group=self.group if self.tp > 1 else None, chunk=chunk,
                                              grad_scale=grad_scale)
        if self.sequence_parallel and self.tp > 1:
            y = _SPColumnParallelFn.apply(x, self.weight, self.bias, self.group)
        elif self.tp > 1 or getattr(self.weight, "main_grad", None) is not None:
            # _st_link: an attention that finishes dQ in this node's backward (ops.attention.DQLink)
            y = _ColumnParallelFn.apply(x, self.weight, self.bias, self.group, getattr(self, "_st_link", None))
        else:
            y = F.linear(x, self.weight, self.bias)
        if self.gather_output and self.tp > 1:
            y = GatherFromTensorParallelRegion.apply(y, self.group)
        return y


class RowParallelLinear(nn.Module):
    """Input features split over TP: weight [out, in/tp]; output all-reduced
    (or reduce-scattered along seq under SP) (reference tensor_parallel.py:264-372)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False, input_is_parallel: bool = True,
                 sequence_parallel: bool = False, init: str = "uniform", init_std: float = 0.02, group=None):
        super().__init__()
        self.group = group if group is not None else mesh.tp_group()
        self.tp = _ws(self.group) if self.group is not None else 1
        if in_features % self.tp:
            raise ValueError(f"in_features {in_features} not divisible by tp {self.tp}")
        self.in_features, self.out_features = in_features, out_features
        self.in_per_rank = in_features // self.tp
        self.input_is_parallel, self.sequence_parallel = input_is_parallel, sequence_parallel
        self.init, self.init_std = init, init_std
        self.weight = nn.Parameter(torch.empty(out_features, self.in_per_rank))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None
        self.reset_parameters()

    def reset_parameters(self) -> None:
        from .init import init_full

        key = getattr(self, "_st_init_key", None)
        if key is None:
            _init_shard_(self.weight, self.init, self.init_std, self.in_features)
        else:
            full = init_full((self.out_features, self.in_features), self.init, self.init_std, self.in_features,
                             key, self.weight.device)
            r = C.get_rank(self.group) if self.tp > 1 else 0
            with torch.no_grad():
                self.weight.copy_(full.chunk(self.tp, dim=1)[r])
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, x: torch.Tensor, act: str | None = None) -> torch.Tensor:
        """``act="swiglu"``: x is a fused gate|up output and the SwiGLU is applied here,
        on one rank with the activation recomputed in backward (ops.mlp.swiglu_linear)."""
        from .. import ops
        from ..ops.mlp import linear, swiglu_linear

        if act == "swiglu":
            if self.tp == 1 and self.bias is None:
                y = swiglu_linear(x, self.weight)
                if y is not None:
                    return y
            x = ops.swiglu(x)
        if not self.input_is_parallel and self.tp > 1:
            x = ScatterToTensorParallelRegion.apply(x, self.group)
        if self.tp > 1 and not self.sequence_parallel:
            y = _RowParallelFn.apply(x, self.weight, self.group)  # GEMM / all-reduce pipelined
        elif (self.tp > 1 and x.dim() == 3 and x.shape[1] % self.tp == 0 and torch.is_grad_enabled()
              and getattr(self.weight, "main_grad", None) is not None and _sp_overlap(x)):
            y = _SPRowParallelFn.apply(x, self.weight, self.group)  # GEMM / reduce-scatter pipelined
        else:
            y = linear(x, self.weight, None)
            if self.tp > 1:
                y = ReduceScatterToSequenceParallelRegion.apply(y, self.group)
        if self.bias is not None:
            y = y + self.bias
        return y


class FusedColumnParallelLinear(ColumnParallelLinear):
    """Several column-parallel projections of the same input as ONE GEMM.

    ``splits`` are the GLOBAL output sizes of the fused pieces (e.g. q, k, v);
    each rank holds ``[piece_0/tp; piece_1/tp; ...]``.  ``names`` gives the
    reference module names for state-dict conversion (``q_proj`` ...).
    """

    def __init__(self, in_features: int, splits: list[int], names: list[str], **kw):
        self.splits, self.names = list(splits), list(names)
        super().__init__(in_features, sum(splits), **kw)
        for s in splits:
            if s % self.tp:
                raise ValueError(f"fused piece {s} not divisible by tp {self.tp}")
        self.local_splits = [s // self.tp for s in splits]

    def _row_pieces(self) -> list[int]:
        return self.splits

    def split_output(self, y: torch.Tensor) -> list[torch.Tensor]:
        return list(y.split(self.local_splits, dim=-1))

    def reference_pieces(self, tensor: torch.Tensor) -> list[torch.Tensor]:
        """Split a fused weight/bias into the per-projection shards (reference names)."""
        return list(tensor.split(self.local_splits, dim=0))


class VocabParallelEmbedding(nn.Module):
    """Embedding rows split over TP (reference tensor_parallel.py:375-517).

    Out-of-shard ids read a zero row; the partial embeddings are all-reduced
    (or reduce-scattered along seq under SP).
    """

    def __init__(self, num_embeddings: int, embedding_dim: int, sequence_parallel: bool = False,
                 init_std: float | None = None, group=None):
        super().__init__()
        self.group = group if group is not None else mesh.tp_group()
        self.tp = _ws(self.group) if self.group is not None else 1
        self.rank = C.get_rank(self.group) if self.tp > 1 else 0
        if num_embeddings % self.tp:
            raise ValueError(f"vocab {num_embeddings} not divisible by tp {self.tp}")
        self.num_embeddings, self.embedding_dim = num_embeddings, embedding_dim
        self.per_rank = num_embeddings // self.tp
        self.vocab_start = self.rank * self.per_rank
        self.sequence_parallel = sequence_parallel
        self.init_std = init_std
        self.weight = nn.Parameter(torch.empty(self.per_rank, embedding_dim))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        from .init import init_full

        std = self.init_std if self.init_std is not None else 1.0 / math.sqrt(self.embedding_dim)
        key = getattr(self, "_st_init_key", None)
        with torch.no_grad():
            if key is None:
                self.weight.normal_(0.0, std)
            else:
                full = init_full((self.num_embeddings, self.embedding_dim), "normal", std, self.embedding_dim, key,
                                 self.weight.device)
                self.weight.copy_(full.chunk(self.tp, dim=0)[self.rank])

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        from .embedding import embedding

        if self.tp == 1:
            return embedding(ids, self.weight)
        local = ids - self.vocab_start
        mask = (local < 0) | (local >= self.per_rank)
        # forward reads row 0 for out-of-shard ids (zeroed below); the backward scatters
        # only in-shard ids (-1 = skip), so 1-1/tp of the tokens do not pile onto row 0
        out = embedding(local.masked_fill(mask, 0), self.weight, local.masked_fill(mask, -1))
        out = out.masked_fill(mask[..., None], 0.0)
        if self.sequence_parallel:
            return ReduceScatterToSequenceParallelRegion.apply(out, self.group)
        return ReduceFromTensorParallelRegion.apply(out, self.group)


def apply_tensor_parallel(model: nn.Module) -> nn.Module:
    """Compatibility entry point (reference tensor_parallel.py:22-144).

    Models in this package are constructed TP-sharded from the mesh, so this is
    a validation pass: it checks every TP layer agrees with the active mesh.
    """
    tp = mesh.tp_size()
    for name, m in model.named_modules():
        if isinstance(m, (ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding)) and m.tp != tp:
            raise RuntimeError(f"{name} built for tp={m.tp} but the mesh has tp={tp}; build the model after "
                               "setup_process_group_manager()")
    return model

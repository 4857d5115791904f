"""Mixture-of-Experts MLP (Qwen3-MoE / Mixtral) with autograd-aware expert parallelism.

Reference: MoERouter / MoEExperts / MoELayer in scaletorch/models/model_qwen3_moe.py:30-292
and dispatch/gather in scaletorch/parallel/expert_parallel/ep_comms.py.  Fixes
and MI355X-first changes:

* dispatch/combine all-to-alls are autograd Functions (backward = the reverse
  all-to-all), so router and experts receive gradients under EP > 1 (the
  reference detached them);
* ONE hidden-state all-to-all each way per layer (expert ids / weights never
  travel: the permutation is recomputed locally), plus one tiny count exchange;
* tokens are sorted by expert once (device-side ``argsort``/``bincount``), so
  every expert runs one contiguous GEMM over its rows (no per-expert
  ``nonzero`` host syncs, reference model_qwen3_moe.py:143-171);
* local experts are stored STACKED ([E_local, 2I, h] gate|up and
  [E_local, h, I] down) for grouped GEMMs; checkpoints expand them to the
  reference's ``moe.experts.experts.{e}.{gate,up,down}_proj.weight`` keys;
* the Switch-style load-balancing aux loss is returned to the trainer and added
  to the LM loss (the reference computed and dropped it).
"""
from __future__ import annotations

import math
import os
from typing import NamedTuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..dist import collectives as C
from ..dist import trace
from ..parallel import mesh
from ..parallel.tensor_parallel import (AllGatherFromSequenceParallelRegion, ReduceFromTensorParallelRegion,
                                        ReduceScatterToSequenceParallelRegion)
from .config import ModelConfig


class _AllToAll(torch.autograd.Function):
    """Variable-split all-to-all of rows; backward is the reverse exchange."""

    @staticmethod
    def forward(ctx, x, out_splits, in_splits, group):
        trace.record("ep.all_to_all", x, group_size=C.get_world_size(group), send=list(in_splits), recv=list(out_splits))
        ctx.splits = (out_splits, in_splits)
        ctx.group = group
        return C.all_to_all(x.contiguous(), group=group, output_split_sizes=out_splits, input_split_sizes=in_splits)

    @staticmethod
    def backward(ctx, g):
        out_splits, in_splits = ctx.splits
        trace.record("ep.all_to_all_bwd", g, group_size=C.get_world_size(ctx.group))
        return (C.all_to_all(g.contiguous(), group=ctx.group, output_split_sizes=in_splits,
                             input_split_sizes=out_splits), None, None, None)


def all_to_all_rows(x, out_splits, in_splits, group):
    if C.get_world_size(group) == 1:
        return x
    return _AllToAll.apply(x, out_splits, in_splits, group)


# ---------------------------------------------------------------- capacity-bounded dispatch
# EP dispatch options (trainer: --moe_capacity_factor / --moe_ep_chunks)
_DISPATCH = {"capacity_factor": 0.0, "chunks": 1, "comm": "rccl"}
_EP_XGMI: dict = {}      # id(ep group) -> dist/xgmi.XgmiAllReduce
_EP_STREAMS: dict = {}   # device -> side stream of the xGMI all-to-alls


def set_moe_dispatch(capacity_factor: float = 0.0, chunks: int = 1, comm: str = "rccl") -> None:
    if comm not in ("rccl", "xgmi"):
        raise ValueError(f"ep_comm must be rccl or xgmi, got {comm!r}")
    _DISPATCH.update(capacity_factor=float(capacity_factor), chunks=max(1, int(chunks)), comm=comm)


def ep_area_bytes(tokens: int, ep: int, top_k: int, num_experts: int, hidden: int,
                  capacity_factor: float = 0.0) -> int:
    """IPC data area the EP exchange of a run needs: the dropless landing rows at the host
    bound R_max = ep * T * min(k, E/ep) (or the capacity dispatch's cf * T * k rows) of
    ``hidden`` bf16, rounded up to 8 MiB, at least 16 MiB (Mixtral EP 8 at 4,096 tokens:
    268 MiB)."""
    El = max(1, num_experts // max(1, ep))
    rows = ep * tokens * min(top_k, El)
    if capacity_factor > 0:
        rows = max(rows, int(math.ceil(capacity_factor * tokens * top_k)))
    need = rows * hidden * 2
    return max(16 << 20, -(-need // (8 << 20)) * (8 << 20))


def setup_ep_xgmi(group, area_bytes: int | None = None) -> None:
    """Create the EP group's xGMI communicator (collective over the group, at start-up):
    the capacity dispatch's equal-split all-to-alls then PUSH rows straight into the
    peers' buffers over all 7 links (csrc/xgmi_allreduce.hip mode 4).  ``area_bytes``: the
    run's need (``ep_area_bytes``); ST_XGMI_EP_MAX_MB overrides, 512 MiB without either."""
    from ..dist.xgmi import XgmiAllReduce, _max_bytes_default

    if group is not None and C.get_world_size(group) > 1:
        size = area_bytes if (area_bytes and not os.environ.get("ST_XGMI_EP_MAX_MB")) else _max_bytes_default("ep")
        _EP_XGMI[id(group)] = XgmiAllReduce(group, max_bytes=size)


def check_ep_xgmi() -> None:
    """Raise if an EP exchange of this process timed out: a kernel that gave up waiting for
    a peer leaves its output rows unwritten (one host sync per communicator)."""
    for comm in list(_EP_XGMI.values()):
        comm.check()


def _ep_a2a(x: torch.Tensor, group, async_op: bool):
    """Equal-split all-to-all: the xGMI push kernel when set up and the message fits
    (on a side stream when ``async_op``), else RCCL.  Returns out or (out, work)."""
    comm = _EP_XGMI.get(id(group)) if (_DISPATCH["comm"] == "xgmi" and x.is_cuda) else None
    if comm is None or not comm.supports(x) or x.shape[0] % comm.world:
        return C.all_to_all(x, group=group, async_op=async_op)
    if not async_op:
        return comm.all_to_all(x)
    from ..parallel.tensor_parallel import _StreamWork

    st = _EP_STREAMS.get(x.device.index)
    if st is None:
        st = _EP_STREAMS[x.device.index] = torch.cuda.Stream(device=x.device)
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        out = comm.all_to_all(x)
    x.record_stream(st)
    out.record_stream(torch.cuda.current_stream())
    return out, _StreamWork(st)


class _A2AStart(torch.autograd.Function):
    """Equal-split all-to-all of rows issued asynchronously: RCCL runs it on its own
    stream and the host continues; ``_A2AWait`` makes the consumer's stream wait for it
    (no host block on RCCL).  Backward: the reverse equal-split exchange."""

    @staticmethod
    def forward(ctx, x, holder, group):
        trace.record("ep.all_to_all", x, group_size=C.get_world_size(group))
        ctx.group = group
        out, work = _ep_a2a(x.contiguous(), group, async_op=True)
        holder.append(work)
        return out

    @staticmethod
    def backward(ctx, g):
        trace.record("ep.all_to_all_bwd", g, group_size=C.get_world_size(ctx.group))
        return _ep_a2a(g.contiguous(), ctx.group, async_op=False), None, None


class _A2AWait(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, holder):
        for w in holder:
            if w is not None:
                w.wait()
        holder.clear()
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g, None


class CapacityPlan(NamedTuple):
    send_idx: torch.Tensor    # [ep*cap] expert-sorted row feeding each send slot
    send_valid: torch.Tensor  # [ep*cap] slot holds a row (else zero padding)
    kept: torch.Tensor        # [ep, El] rows per (destination, local expert) after truncation
    back_idx: torch.Tensor    # [rows] slot each expert-sorted row returns from
    keep_row: torch.Tensor    # [rows] row was sent (not dropped)
    cap: int


def capacity_plan(counts: torch.Tensor, ep: int, cap: int, rows: int) -> CapacityPlan:
    """Sender side of the static-capacity dispatch, all on the device.  ``counts`` [E]:
    rows per global expert of the expert-sorted buffer (``rows`` = T*k, host-known).
    Destination d (experts [d*El, (d+1)*El)) gets its first ``cap`` rows in expert
    order; the rest are dropped (the truncation takes the last local experts' rows)."""
    dev = counts.device
    El = counts.numel() // ep
    mat = counts.view(ep, El).long()
    cum = torch.cumsum(mat, 1) - mat
    kept = torch.clamp(torch.minimum(mat, cap - cum), min=0)
    dcount = mat.sum(1)
    dend = torch.cumsum(dcount, 0)
    dstart = dend - dcount
    dkept = kept.sum(1)
    j = torch.arange(cap, device=dev)
    send_valid = (j[None, :] < dkept[:, None]).reshape(-1)
    send_idx = torch.where(send_valid, (dstart[:, None] + j[None, :]).reshape(-1), 0)
    p = torch.arange(rows, device=dev)
    d = torch.searchsorted(dend, p, right=True).clamp(max=ep - 1)
    jp = p - dstart[d]
    keep_row = jp < dkept[d]
    back_idx = torch.where(keep_row, d * cap + jp, 0)
    return CapacityPlan(send_idx, send_valid, kept, back_idx, keep_row, cap)


def capacity_receive_order(recv_kept: torch.Tensor, cap: int):
    """Receiver side: the static [ep*cap] received rows (block s = source s: its rows for
    local expert 0, 1, ..., then padding) -> expert-major order.  Returns ``order`` (a
    permutation: row i of the expert input = received row order[i]; the valid rows of
    every expert first, then every padding row) and the per-expert inclusive ``offs``
    (int32) of the grouped GEMMs.  Device only: no host read of the counts."""
    ep, El = recv_kept.shape
    dev = recv_kept.device
    total = ep * cap
    rk = recv_kept.long()
    within = torch.cumsum(rk, 1) - rk
    src_start = torch.arange(ep, device=dev)[:, None] * cap + within
    counts_es = rk.t().reshape(-1)
    src_start_es = src_start.t().reshape(-1)
    ends = torch.cumsum(counts_es, 0)
    starts = ends - counts_es
    V = ends[-1]
    i = torch.arange(total, device=dev)
    blk = torch.searchsorted(ends, i, right=True).clamp(max=ep * El - 1)
    order_valid = src_start_es[blk] + (i - starts[blk])
    ktot = rk.sum(1)
    padc = cap - ktot
    pend = torch.cumsum(padc, 0)
    pstart = pend - padc
    ip = (i - V).clamp(min=0)
    ps = torch.searchsorted(pend, ip, right=True).clamp(max=ep - 1)
    order_pad = ps * cap + ktot[ps] + (ip - pstart[ps])
    order = torch.where(i < V, order_valid, order_pad)
    offs = torch.cumsum(rk.sum(0), 0).to(torch.int32)
    return order, offs


# ---------------------------------------------------------------- dropless exchange, device counts
# Every EP rank all-gathers its per-expert row counts into M [ep, E] (device, int32).
# From M alone each rank knows where every row goes: source s holds its rows sorted
# by global expert (P[s][g] = first row of expert g), owner d = g // El receives its
# experts' rows EXPERT-MAJOR (expert g = [rows from source 0 | source 1 | ...]), row
# (s, i) of expert g landing at q = EO[g] + SO[s][g] + (i - P[s][g]).  The exchange
# buffers are sized by the host bound R_max = ep * T_max * min(k, El) rows (every
# token routes at most min(k, El) rows to one owner), so nothing is ever dropped and
# no count is read by the host: on one node the push kernel
# (csrc/xgmi_allreduce.hip ``ep_exchange_kernel``) places the rows straight at q in
# the owner's buffer; elsewhere RCCL moves them with exact splits after one host read
# of M per layer.  The grouped GEMMs run on the R_max-row buffer with device offsets,
# so only the real rows cost FLOPs.  Reference: dispatch_tokens / gather_tokens,
# scaletorch/parallel/expert_parallel/ep_comms.py:41-171 (host-synced splits, three
# all-to-alls, no autograd).
_TOKEN_BOUND: dict = {"n": None}


def set_ep_token_bound(n: int | None) -> None:
    """Declare the token count of every MoE call on every EP rank (the trainer: micro-batch x
    sequence / cp -- identical on all ranks by construction, its loaders drop ragged tail
    batches).  With it the exchange buffers are sized on the host with NO collective; without
    it (library use, tests) every call agrees on the bound with one small all-reduce."""
    _TOKEN_BOUND["n"] = None if n is None else int(n)


def ep_rows_range(T: int, group, agree: bool = False) -> tuple[int, int]:
    """(smallest, largest) local token count over the EP group.

    Every rank takes the same branch on every call, so the collectives on the EP group stay
    in step even when the token counts change between calls: with a declared bound
    (``set_ep_token_bound``) no collective runs and the range is (T, bound) -- a local T above
    the bound raises; otherwise ONE all-reduce per call (no cache keyed on the local T: a rank
    whose T repeats would skip the collective its peers enter -- ADVICE r04).  ``agree``
    forces the all-reduce even with a declared bound: the capacity dispatch needs the TRUE
    range, so a rank below the bound makes every rank raise together instead of leaving its
    peers in the all-to-all."""
    n = _TOKEN_BOUND["n"]
    if n is not None and not agree:
        if int(T) > n:
            raise ValueError(f"MoE call with {T} tokens exceeds the declared EP token bound {n}")
        return int(T), n
    t = torch.tensor([int(T), -int(T)], dtype=torch.int64,
                     device="cuda" if (torch.cuda.is_available() and _group_on_gpu(group)) else "cpu")
    if C.get_world_size(group) > 1:
        C.all_reduce(t, op="max", group=group)
    return -int(t[1].item()), int(t[0].item())


def ep_rows_bound(T: int, group) -> int:
    """Largest local token count over the EP group (sizes the dropless exchange buffers)."""
    return ep_rows_range(T, group)[1]


def _group_on_gpu(group) -> bool:
    import torch.distributed as dist

    try:
        return dist.get_backend(group) == "nccl"
    except (RuntimeError, ValueError, AttributeError):
        return False


def ep_owner_positions(M: torch.Tensor, El: int, owner: int, rows: int) -> torch.Tensor:
    """Expert-major position q of every row ``owner`` receives, in ARRIVAL order (source
    0's rows of the owner's experts in expert order, then source 1's, ...); ``rows`` =
    their number (host).  Device only."""
    Ml = M.long()
    ep, E = Ml.shape
    blk = Ml[:, owner * El:(owner + 1) * El]                        # [s, e] block sizes
    SO = torch.cumsum(Ml, 0) - Ml                                   # rows of g from sources < s
    tot = blk.sum(0)                                                # [e]
    EO = torch.cumsum(tot, 0) - tot                                 # owner's expert offsets
    base = (EO[None, :] + SO[:, owner * El:(owner + 1) * El]).reshape(-1)
    sizes = blk.reshape(-1)
    start = torch.cumsum(sizes, 0) - sizes
    rep = torch.repeat_interleave(torch.arange(ep * El, device=M.device), sizes, output_size=rows)
    return base[rep] + (torch.arange(rows, device=M.device) - start[rep])


def ep_exchange_reference(xs: list, M: torch.Tensor, El: int, direction: int, out_rows: int) -> list:
    """All ranks' exchange in ONE process (tests): ``xs[r]`` = rank r's input.  Direction
    0: rank r's sorted rows -> every owner's expert-major rows (``out_rows`` per owner,
    the tail past the received rows zero); 1: the reverse (each source gets its own
    sum(M[s]) rows; ``out_rows`` unused).  Built from explicit per-row loops over M, independent of the position
    formula it checks."""
    Mh = M.to("cpu", torch.int64)
    ep, E = Mh.shape
    rows = [out_rows] * ep if direction == 0 else [int(Mh[s].sum()) for s in range(ep)]
    outs = [xs[0].new_zeros(rows[r], xs[0].shape[1]) for r in range(ep)]
    # expert-major slot lists per owner: for each local expert, sources in order
    for d in range(ep):
        slot = 0
        for e in range(El):
            g = d * El + e
            for s in range(ep):
                first = int(Mh[s, :g].sum())
                for j in range(int(Mh[s, g])):
                    if direction == 0:
                        outs[d][slot] = xs[s][first + j]
                    else:
                        outs[s][first + j] = xs[d][slot]
                    slot += 1
    return outs


def _ep_exchange_rccl(x: torch.Tensor, M: torch.Tensor, El: int, direction: int, out_rows: int, group,
                      Mh: torch.Tensor | None = None):
    """The exchange over RCCL / gloo with exact splits, same layouts as the push kernel.
    ``Mh``: M already read to the host -- the MoE layer reads it ONCE per forward and hands
    it to the dispatch, the combine and both backward exchanges (``_EPExchange``)."""
    ep = M.shape[0]
    me = C.get_rank(group)
    if Mh is None:
        Mh = M.detach().to("cpu", torch.int64)
    rows_to = Mh.view(ep, ep, El).sum(2)  # [source, owner]
    R = int(rows_to[:, me].sum())
    q = ep_owner_positions(M.to(x.device), El, me, R)
    if direction == 0:
        r = C.all_to_all(x.contiguous(), group=group, output_split_sizes=rows_to[:, me].tolist(),
                         input_split_sizes=rows_to[me].tolist())
        out = x.new_zeros(out_rows, x.shape[1]) if _ZERO_PAD[0] else x.new_empty(out_rows, x.shape[1])
        out.index_copy_(0, q, r)
        return out
    out = C.all_to_all(x.index_select(0, q), group=group, output_split_sizes=rows_to[me].tolist(),
                       input_split_sizes=rows_to[:, me].tolist())
    if out.shape[0] != out_rows:
        raise RuntimeError(f"EP combine returned {out.shape[0]} rows, expected {out_rows}")
    return out


_ZERO_PAD = [os.environ.get("ST_MOE_ZERO_PAD", "0") == "1"]  # zero the unused tail of R_max buffers (debug)
_DEBUG_ROUTING = [os.environ.get("ST_MOE_DEBUG", "0") == "1"]  # router input / index checks (debug runs)
_DEBUG_CALLS = [0]  # router calls checked so far


def _ep_exchange(x, M, El, direction, out_rows, area_rows, group, comm, Mh=None):
    # bytes counted = the rows that really travel per rank (dispatch: this rank's T*k sorted
    # rows; combine: the T*k rows it gets back), not the R_max-row padded expert buffer
    trace.record("ep.exchange" if direction == 0 else "ep.exchange_back", x if direction == 0 else x[:out_rows],
                 group_size=C.get_world_size(group), transport="xgmi" if comm is not None else "rccl")
    if comm is not None:
        out = comm.ep_exchange(x, M, El, direction, out_rows, area_rows)
        if _ZERO_PAD[0] and direction == 0:  # rows past the received ones hold stale data
            valid = M[:, C.get_rank(group) * El:(C.get_rank(group) + 1) * El].sum()
            out.masked_fill_((torch.arange(out_rows, device=out.device) >= valid)[:, None], 0)
        return out
    return _ep_exchange_rccl(x, M, El, direction, out_rows, group)


class _EPExchange(torch.autograd.Function):
    """Dispatch (direction 0: sorted rows -> owners' expert-major rows) or combine
    (direction 1); backward is the other direction with the same counts."""

    @staticmethod
    def forward(ctx, x, M, El, direction, out_rows, bounds, group, comm, Mh=None):
        ctx.save_for_backward(M)
        ctx.meta = (El, direction, x.shape[0], bounds, group, comm, Mh)
        area = bounds[0] if direction == 0 else bounds[1]
        return _ep_exchange(x, M, El, direction, out_rows, area, group, comm, Mh)

    @staticmethod
    def backward(ctx, g):
        (M,) = ctx.saved_tensors
        El, direction, in_rows, bounds, group, comm, Mh = ctx.meta
        rev = 1 - direction
        area = bounds[0] if rev == 0 else bounds[1]
        return (_ep_exchange(g.contiguous(), M, El, rev, in_rows, area, group, comm, Mh),
                None, None, None, None, None, None, None, None)


def ep_counts_matrix(counts: torch.Tensor, group, comm=None) -> torch.Tensor:
    """[ep, E] int32 routing counts of every EP rank (device all-gather, no host sync)."""
    c = counts.to(torch.int32).contiguous()
    if comm is not None:
        return comm.ep_counts(c)
    return C.all_gather(c, group=group).view(C.get_world_size(group), -1)


def ep_comm_for(group):
    """The EP group's xGMI communicator when the push exchange is enabled, else None."""
    return _EP_XGMI.get(id(group)) if _DISPATCH["comm"] == "xgmi" else None


def select_ep_transport(group, requested: str = "auto", area_bytes: int | None = None) -> str:
    """Collective over the EP group at start-up.  "auto": set up the xGMI communicator
    (one node, one GPU per rank) and self-test the push exchange against the RCCL
    exchange on random routing (bitwise equal both ways); the MIN-reduced verdict picks
    xgmi or rccl for every rank.  Sets the dispatch transport and returns it."""
    if requested == "rccl" or C.get_world_size(group) <= 1:
        _DISPATCH["comm"] = "rccl"
        return "rccl"
    ok = 0
    info: dict = {}
    try:
        setup_ep_xgmi(group, area_bytes)
        comm = _EP_XGMI.get(id(group))
        if comm is not None:
            ok, info = _ep_selftest(comm, group)
    except Exception as e:  # noqa: BLE001 -- every rank still joins the vote
        ok, info = 0, {"error": repr(e)[:200]}
        if requested == "xgmi":
            raise
    flag = torch.tensor([ok], dtype=torch.int32, device="cuda" if _group_on_gpu(group) else "cpu")
    C.all_reduce(flag, op="min", group=group)
    choice = "xgmi" if int(flag.item()) == 1 else "rccl"
    if requested == "xgmi" and choice != "xgmi":
        raise RuntimeError(f"ep_comm xgmi requested but the push exchange self-test failed: {info}")
    if choice == "rccl":
        # free the losing communicator's IPC area (kHeader + 4 x 512 MiB by default) once no
        # peer can still be reading it
        comm = _EP_XGMI.pop(id(group), None)
        if comm is not None:
            torch.cuda.synchronize()
            C.barrier(group=group)
            comm.close()
    _DISPATCH["comm"] = choice
    EP_TRANSPORT.update(ep=choice, selftest=info)
    return choice


EP_TRANSPORT: dict = {"ep": "rccl", "selftest": None}


def _ep_selftest(comm, group):
    ep = C.get_world_size(group)
    El, T, k, h = 2, 96, 2, 64
    E = El * ep
    g = torch.Generator(device="cuda").manual_seed(77 + C.get_rank(group))
    topi = torch.stack([torch.randperm(E, generator=g, device="cuda")[:k] for _ in range(T)])
    counts = torch.bincount(topi.reshape(-1), minlength=E).to(torch.int32)
    x = torch.randn(T * k, h, device="cuda", dtype=torch.bfloat16, generator=g)
    M = ep_counts_matrix(counts, group, comm)
    M_ref = ep_counts_matrix(counts, group, None)
    R_max, Tk = ep * T * min(k, El), T * k
    a = comm.ep_exchange(x, M, El, 0, R_max, R_max)
    b = _ep_exchange_rccl(x, M, El, 0, R_max, group)
    valid = int(M[:, C.get_rank(group) * El:(C.get_rank(group) + 1) * El].sum())
    back_a = comm.ep_exchange(a, M, El, 1, Tk, Tk)
    back_b = _ep_exchange_rccl(b, M, El, 1, Tk, group)
    comm.check()
    ok = bool(torch.equal(M, M_ref) and torch.equal(a[:valid], b[:valid]) and torch.equal(back_a, back_b)
              and torch.equal(back_a, x))
    return (1 if ok else 0), {"rows": valid, "bitwise": ok}


_GMM_OK: bool | None = None


def _grouped_mm_available() -> bool:
    """torch._grouped_mm (device offsets, autograd) exists and runs on this device;
    ST_MOE_GROUPED_GEMM=0 forces the per-expert loop."""
    global _GMM_OK
    import os

    if os.environ.get("ST_MOE_GROUPED_GEMM", "1") == "0":
        return False
    if _GMM_OK is None:
        _GMM_OK = False
        if hasattr(torch, "_grouped_mm") and torch.cuda.is_available():
            try:
                a = torch.randn(32, 64, device="cuda", dtype=torch.bfloat16)
                b = torch.randn(2, 64, 32, device="cuda", dtype=torch.bfloat16)
                torch._grouped_mm(a, b, offs=torch.tensor([16, 32], device="cuda", dtype=torch.int32))
                _GMM_OK = True
            except (RuntimeError, NotImplementedError, TypeError):
                _GMM_OK = False
    return _GMM_OK


def expert_major_order(recv_mat: torch.Tensor, total: int) -> torch.Tensor:
    """Row permutation taking received rows from [src rank][local expert] order to
    [local expert][src rank] order (each expert's rows contiguous for the grouped
    GEMM), derived on the device from the received count matrix ``recv_mat``
    [ep, E_local] -- no host loop, no sync (``total`` = rows received, known on the
    host from the all-to-all splits).  ``order[i]`` = received row placed at i."""
    ep, el = recv_mat.shape
    dev = recv_mat.device
    counts_se = recv_mat.reshape(-1).long()                  # blocks in arrival order (s, e)
    start_se = torch.cumsum(counts_se, 0) - counts_se        # arrival offset of block (s, e)
    counts_es = recv_mat.t().reshape(-1).long()              # blocks in expert-major order (e, s)
    block_es = torch.arange(ep * el, device=dev).view(ep, el).t().reshape(-1)  # (e, s) -> flat (s, e) id
    start_es = torch.cumsum(counts_es, 0) - counts_es
    blk = torch.repeat_interleave(torch.arange(ep * el, device=dev), counts_es, output_size=total)
    within = torch.arange(total, device=dev) - start_es[blk]
    return start_se[block_es[blk]] + within


class MoERouter(nn.Module):
    """Top-k softmax router (reference model_qwen3_moe.py:30-92)."""

    def __init__(self, hidden: int, num_experts: int, top_k: int, norm_topk_prob: bool, aux_coef: float,
                 init_std: float = 0.02):
        super().__init__()
        self.num_experts, self.top_k = num_experts, top_k
        self.norm_topk_prob, self.aux_coef = norm_topk_prob, aux_coef
        self.init_std = init_std
        self.gate = nn.Linear(hidden, num_experts, bias=False)
        self._st_reads = (self.gate,)  # forward reads gate.weight directly (DataParallel bucket waits)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        from ..parallel.init import keyed_generator

        g = keyed_generator(getattr(self, "_st_init_key", None), self.gate.weight.device)
        with torch.no_grad():
            full = torch.empty(self.gate.weight.shape, dtype=torch.float32, device=self.gate.weight.device)
            full.normal_(0.0, self.init_std, generator=g)
            self.gate.weight.copy_(full)

    def forward(self, x2d: torch.Tensor):
        logits = ops.linear(x2d, self.gate.weight).float()
        # fused softmax + top-k + renorm (one wave per token, csrc/moe.hip)
        probs, topw, topi = ops.moe.router_topk(logits, self.top_k, self.norm_topk_prob)
        # Switch aux loss: coef * E * sum_e f_e * P_e
        T = x2d.shape[0]
        if _DEBUG_ROUTING[0]:  # ST_MOE_DEBUG=1: host checks (one sync per router call) before the scatter
            _DEBUG_CALLS[0] += 1
            bad_in = int((~torch.isfinite(x2d)).sum())
            lo, hi = int(topi.min()), int(topi.max())
            if bad_in or lo < 0 or hi >= self.num_experts:
                raise RuntimeError(f"router call {_DEBUG_CALLS[0]}: {bad_in} non-finite inputs, top-k "
                                   f"indices in [{lo}, {hi}] of {self.num_experts} experts (T {T})")
        counts = torch.zeros(self.num_experts, device=x2d.device, dtype=torch.float32)
        counts.scatter_add_(0, topi.reshape(-1).long(), torch.ones(topi.numel(), device=x2d.device))
        f = counts / max(1, T * self.top_k)
        P = probs.mean(0)
        aux = self.aux_coef * self.num_experts * (f * P).sum()
        return topw, topi, aux


def _gmm_fallback(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor, wn: bool) -> torch.Tensor:
    """``torch._grouped_mm`` when it runs here, else one GEMM per expert (one host read
    of the offsets).  Rows past ``offs[-1]`` come back zero."""
    wt = w if wn else w.transpose(-2, -1)
    if _grouped_mm_available():
        return torch._grouped_mm(x, wt, offs=offs)
    ends = offs.tolist()
    y = x.new_zeros(x.shape[0], wt.shape[2])
    start = 0
    for g, end in enumerate(ends):
        if end > start:
            y[start:end] = x[start:end] @ wt[g]
        start = end
    return y


def _gemm4w_ok(x: torch.Tensor, w: torch.Tensor, N: int) -> bool:
    """The one-wave-per-SIMD kernel (csrc/gemm4w.hip) takes this [G, N, K] expert GEMM and wins
    on it: long K (>= 4,096: Mixtral's experts, +8-12 % over the 8-phase grouped kernel; at
    Qwen3-MoE's K 768 / 2,048 the grouped kernel is ahead -- tools/bench_grouped_gemm.py,
    profiles/r05/gemm4w/grouped_vs_gemm4w.log).  ``ST_MOE_GEMM4W=0``: off (A/B)."""
    from ..ops import _lib

    K = x.shape[1]
    return (os.environ.get("ST_MOE_GEMM4W", "1") == "1" and _lib.use_native(x) and x.dtype == torch.bfloat16
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.is_contiguous() and K % 64 == 0 and K >= 4096
            and N % 256 == 0 and x.shape[0] > 0)


def _gmm(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor, wn: bool) -> torch.Tensor:
    """Per-expert ``x[rows of g] @ (w[g] if wn else w[g]^T)`` with device offsets: ONE launch
    of csrc/grouped_gemm.hip.  ``ST_MOE_HIP_GMM=0``, or a shape the kernel does not tile
    (K not a whole number of 64-wide K tiles, N not of 128-wide N tiles, operands past
    the kernel's 32-bit buffer offsets -- the binding then returns None), falls back to
    ``_gmm_fallback``."""
    from ..ops import _lib

    K = x.shape[1]
    N = w.shape[2] if wn else w.shape[1]
    if not wn and _gemm4w_ok(x, w, N):
        y = _lib.ops().gemm4w(x, w, offs)
        if y is not None:
            return y
    if (os.environ.get("ST_MOE_HIP_GMM", "1") == "1" and _lib.use_native(x) and x.dtype == torch.bfloat16
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.is_contiguous() and K % 64 == 0 and N % 128 == 0
            and x.shape[0] > 0):
        y = _lib.ops().grouped_gemm(x, w, offs, wn)
        if y is not None:
            return y
    return _gmm_fallback(x, w, offs, wn)


def _gmm_tail_split(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor, wn: bool, padded: bool) -> torch.Tensor:
    """One local expert (G = 1) whose rows are exactly ``x``'s (the RCCL exchange sizes the
    buffer): a narrow GEMM (N = 4,096: 16 column tiles of 256) fills the 256 CUs only in
    whole bands of 4,096 rows, so a few hundred rows past a band cost a third, mostly idle,
    wave (tools/bench_ep8_expert.py: gate|up dgrad 1.46 ms at 8,192 rows, 1.98 ms at 8,544).
    The whole bands run on the grouped kernel and a tail of at most half a band as ONE
    batched hipBLASLt product over K slices (fp32 partials summed once): as one plain GEMM
    the tail's 16-32 tiles took 0.33 ms of a 1.75 ms call.  ``ST_MOE_TAIL_SPLIT=0``: off (A/B)."""
    N = w.shape[2] if wn else w.shape[1]
    M = x.shape[0]
    band = (256 * 256 * 256) // N if N else 0  # rows per full wave of 256 x 256 tiles on 256 CUs
    tail = M % band if band else 0
    if (padded or w.shape[0] != 1 or not x.is_cuda or band == 0 or M < band or tail == 0 or tail > band // 2
            or os.environ.get("ST_MOE_TAIL_SPLIT", "1") != "1"):
        return _gmm(x, w, offs, wn)
    M1 = M - tail
    head = _gmm(x[:M1], w, offs.new_full((1,), M1), wn)
    # the tail's few row tiles alone would leave most CUs idle: split its K over ks batched
    # products (fp32 partials, summed once) so ~a wave of tiles covers the chip
    K = x.shape[1]
    tiles = -(-tail // 256) * (N // 256)
    ks = 1
    while ks < 8 and tiles * ks * 2 <= 256 and K % (ks * 2 * 64) == 0:
        ks *= 2
    wk = (w[0] if wn else w[0].t()).unflatten(0, (ks, K // ks))          # [ks, K/ks, N]
    xk = x[M1:].unflatten(1, (ks, K // ks)).transpose(0, 1)               # [ks, tail, K/ks]
    rest = torch.ops.aten.bmm.dtype(xk, wk, torch.float32).sum(0).to(x.dtype)
    return torch.cat([head, rest], 0)


def _gmm_swiglu(x: torch.Tensor, w_gu: torch.Tensor, offs: torch.Tensor):
    """(gu, a = silu(gate) * up) of the grouped gate|up GEMM: ONE launch with the SwiGLU
    in the epilogue (csrc/grouped_gemm.hip EPI 1) when the kernel takes the shape
    (I % 128 == 0), else the GEMM and a separate SwiGLU pass (valid rows only)."""
    from ..ops import _lib

    K, N = x.shape[1], w_gu.shape[1]
    if os.environ.get("ST_MOE_FUSED_SWIGLU", "1") == "1" and (N // 2) % 128 == 0 and _gemm4w_ok(x, w_gu, N):
        out = _lib.ops().gemm4w_swiglu_grouped(x, w_gu, offs)
        if out:
            return out[0], out[1]
    if (os.environ.get("ST_MOE_FUSED_SWIGLU", "1") == "1" and _lib.use_native(x) and x.dtype == torch.bfloat16
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w_gu.is_contiguous() and K % 64 == 0
            and N % 256 == 0 and x.shape[0] > 0):
        out = _lib.ops().grouped_gemm_swiglu(x, w_gu, offs)
        if out:
            return out[0], out[1]
    gu = _gmm(x, w_gu, offs, wn=False)
    if gu.is_cuda and _lib.use_native(gu):
        return gu, _lib.ops().swiglu_fwd(gu, offs[-1:])
    return gu, ops.swiglu(gu)


def _gmm_dswiglu(dy: torch.Tensor, w_dn: torch.Tensor, offs: torch.Tensor, gu: torch.Tensor) -> torch.Tensor:
    """dgu = SwiGLU-backward(dy @ w_dn[g], gu): the down projection's data-gradient GEMM with
    the SwiGLU backward in its epilogue (EPI 2), else GEMM + swiglu_bwd (valid rows)."""
    from ..ops import _lib

    K, I = dy.shape[1], w_dn.shape[2]
    if (os.environ.get("ST_MOE_FUSED_SWIGLU", "1") == "1" and _lib.use_native(dy) and dy.dtype == torch.bfloat16
            and dy.stride(1) == 1 and dy.stride(0) % 8 == 0 and w_dn.is_contiguous() and K % 64 == 0
            and I % 128 == 0 and dy.shape[0] > 0 and gu.is_contiguous()):
        dgu = _lib.ops().grouped_gemm_dswiglu(dy, w_dn, offs, gu)
        if dgu is not None:
            return dgu
    da = _gmm(dy, w_dn, offs, wn=True)
    return _lib.ops().swiglu_bwd(da.contiguous(), gu, offs[-1:])


def _vendor_expert_gemms() -> str:
    """``ST_MOE_VENDOR_GEMM``: ``0`` (default) -- the HIP grouped kernels (gate|up with the
    SwiGLU in its epilogue, the down dgrad with the SwiGLU backward in its epilogue) on
    every transport; ``1`` -- one hipBLASLt GEMM per local expert (one host read of the
    counts per layer when the transport has not already made one); ``auto`` -- hipBLASLt
    when the RCCL exchange already holds the counts on the host and the rank has few
    experts with many rows each.  In the step the grouped kernels win even there: the
    Mixtral EP8 slice (one expert x ~8,192 rows per micro-batch) runs 760.7 ms/step on them
    against 806.9 ms with per-expert hipBLASLt + separate SwiGLU passes
    (profiles/r06/slices/mixtral_variants.md), although the isolated FFN microbench had
    hipBLASLt 7 % ahead (tools/bench_expert_ffn.py, profiles/r05/expert_ffn_ab.log)."""
    return os.environ.get("ST_MOE_VENDOR_GEMM", "0")


def _gemm_per_expert(x: torch.Tensor, w: torch.Tensor, counts: list, wn: bool, rows: int) -> torch.Tensor:
    """``y[rows of e] = x[rows of e] @ (w[e] if wn else w[e]^T)`` as one library GEMM per
    non-empty expert (host-known row counts); rows past the last expert are left undefined,
    as on the grouped kernel."""
    N = w.shape[2] if wn else w.shape[1]
    y = x.new_empty(rows, N)
    s = 0
    for e, n in enumerate(counts):
        if n:
            torch.matmul(x[s:s + n], w[e] if wn else w[e].t(), out=y[s:s + n])
        s += n
    return y


def _expert_wgrad(w: torch.Tensor, dout: torch.Tensor, inp: torch.Tensor, offs: torch.Tensor, counts):
    """``w.main_grad[e] (+)= dout[rows of e]^T inp[rows of e]`` for every local expert: ONE
    grouped launch (csrc/wgrad_gemm.hip ``st_wgrad_grouped``), else per-expert GEMMs after one
    host read of the counts (returned, so the second weight reuses it)."""
    from ..ops import _lib
    from ..ops.grad import take_fresh, wgrad_into

    fresh = take_fresh(w)
    grouped = os.environ.get("ST_MOE_GROUPED_WGRAD", "1") == "1"  # 0: per-expert launches (A/B)
    if grouped and _lib.ops().wgrad_grouped_(w.main_grad, dout, inp, offs, 0 if fresh else 1):
        return counts
    if counts is None:
        counts = torch.diff(offs, prepend=offs.new_zeros(1)).tolist()
    off = 0
    for e, n in enumerate(counts):
        if n:
            wgrad_into(w.main_grad[e], dout[off:off + n], inp[off:off + n], 0 if fresh else 1, variant=1)
        elif fresh:
            w.main_grad[e].zero_()
        off += n
    return counts


class _ExpertFFNFn(torch.autograd.Function):
    """Grouped expert SwiGLU FFN: forward and data-gradient GEMMs are one launch each over
    all local experts (``_gmm``, csrc/grouped_gemm.hip), and the weight gradients are
    fp32 GEMMs straight into ``main_grad``.  (``torch._grouped_mm``'s own backward only
    emits bf16: its weight gradient went bf16 -> fp32 copy -> add into the arena.)

    The weight gradient of every local expert is ONE launch per weight
    (csrc/wgrad_gemm.hip ``st_wgrad_grouped``): the expert row ranges come from the
    device offsets, so the backward neither reads the routing counts on the host nor
    loops over experts (the reference does the expert backward as one grouped op too,
    scaletorch/models/npu_patch.py:94-127).  Shapes the kernel does not tile fall back
    to per-expert GEMMs after one host read of the counts.

    ``counts_host`` (a list, when the routing counts are on the host): the forward and
    data-gradient GEMMs run as one hipBLASLt GEMM per expert instead (``_vendor_expert_gemms``);
    the SwiGLU passes and the grouped weight-gradient kernel are shared."""

    @staticmethod
    def forward(ctx, x, offs, w_gu, w_dn, counts_host=None):
        from ..ops import _lib

        ctx.counts_host = counts_host
        if counts_host is not None:
            R = x.shape[0]
            gu = _gemm_per_expert(x, w_gu, counts_host, False, R)
            a = _lib.ops().swiglu_fwd(gu, offs[-1:])  # valid rows only
            y = _gemm_per_expert(a, w_dn, counts_host, False, R)
        else:
            gu, a = _gmm_swiglu(x, w_gu, offs)
            y = _gmm_tail_split(a, w_dn, offs, False, getattr(x, "_st_padded", False))
        # padded buffers (dropless EP: R_max rows, the real ones counted on the device):
        # keep only gu and recompute a over the valid rows in backward
        ctx.keep_a = os.environ.get("ST_MOE_SAVE_ACT", "auto") == "1" or (
            os.environ.get("ST_MOE_SAVE_ACT", "auto") == "auto" and not getattr(x, "_st_padded", False))
        ctx.padded = getattr(x, "_st_padded", False)
        ctx.save_for_backward(x, gu, a if ctx.keep_a else None, offs)
        ctx.w_gu, ctx.w_dn = w_gu, w_dn
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops import _lib
        from ..ops.grad import _grad_ready

        x, gu, a, offs = ctx.saved_tensors
        w_gu, w_dn = ctx.w_gu, ctx.w_dn
        dy = dy.contiguous()
        if a is None:
            a = _lib.ops().swiglu_fwd(gu, offs[-1:])  # valid rows only
        ch = ctx.counts_host
        if ch is not None:
            da = _gemm_per_expert(dy, w_dn, ch, True, dy.shape[0])
            dgu = _lib.ops().swiglu_bwd(da, gu, offs[-1:])
            dx = _gemm_per_expert(dgu, w_gu, ch, True, dy.shape[0])
        else:
            dgu = _gmm_dswiglu(dy, w_dn, offs, gu)
            dx = _gmm_tail_split(dgu, w_gu, offs, True, ctx.padded)
        counts = ch
        for w, dout, inp in ((w_dn, dy, a), (w_gu, dgu, x)):
            counts = _expert_wgrad(w, dout, inp, offs, counts)
            _grad_ready(w)
        return dx, None, None, None, None


class MoEExperts(nn.Module):
    """Stacked local experts: ``w_gate_up`` [E, 2I/tp, h], ``w_down`` [E, h, I/tp]."""

    def __init__(self, num_local: int, hidden: int, inter: int, init_std: float = 0.02, num_global: int | None = None,
                 ep_rank: int = 0):
        super().__init__()
        tp = mesh.tp_size()
        self.tp, self.tp_rank = tp, mesh.tp_rank()
        self.num_global, self.ep_rank = num_global or num_local, ep_rank
        self.inter_global = inter
        if inter % tp:
            raise ValueError(f"moe_intermediate_size {inter} not divisible by tp {tp}")
        self.num_local, self.hidden, self.inter = num_local, hidden, inter // tp
        self.init_std = init_std
        self.w_gate_up = nn.Parameter(torch.empty(num_local, 2 * self.inter, hidden))
        self.w_down = nn.Parameter(torch.empty(num_local, hidden, self.inter))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        """Generate the FULL [E, 2I, h] / [E, h, I] tensors, keep this rank's experts and TP slice."""
        from ..parallel.init import keyed_generator

        key = getattr(self, "_st_init_key", None)
        dev = self.w_gate_up.device
        E, I, h = self.num_global, self.inter_global, self.hidden
        e0 = self.ep_rank * self.num_local
        with torch.no_grad():
            gu = torch.empty(E, 2 * I, h, dtype=torch.float32, device=dev)
            gu.normal_(0.0, self.init_std, generator=keyed_generator(key and key + ".gate_up", dev))
            gu = gu[e0:e0 + self.num_local]
            g, u = gu[:, :I].chunk(self.tp, 1)[self.tp_rank], gu[:, I:].chunk(self.tp, 1)[self.tp_rank]
            self.w_gate_up.copy_(torch.cat([g, u], dim=1))
            dn = torch.empty(E, h, I, dtype=torch.float32, device=dev)
            dn.normal_(0.0, self.init_std, generator=keyed_generator(key and key + ".down", dev))
            self.w_down.copy_(dn[e0:e0 + self.num_local].chunk(self.tp, 2)[self.tp_rank])

    def forward(self, x: torch.Tensor, counts=None, offs: torch.Tensor | None = None,
                counts_host: list | None = None) -> torch.Tensor:
        """x: rows grouped by local expert (``counts[e]`` rows each -- list or device
        tensor -- or the inclusive device prefix ``offs``); rows past the last expert's
        (capacity / R_max padding) are not computed: their output is undefined on the
        grouped-GEMM path and zero (still connected) on the per-expert path.

        GPU: two grouped GEMMs over all local experts (csrc/grouped_gemm.hip, device
        offsets): no per-expert launches and no host read of the routing counts; with
        ``counts_host`` (or ``ST_MOE_VENDOR_GEMM=1``) one hipBLASLt GEMM per expert instead.
        CPU / fallback: one GEMM pair per expert."""
        if x.is_cuda and _grouped_mm_available() and x.dtype == torch.bfloat16:
            if offs is None:
                if not isinstance(counts, torch.Tensor):
                    counts = torch.tensor(counts, dtype=torch.int32)
                offs = torch.cumsum(counts.to(device=x.device, dtype=torch.int32), 0, dtype=torch.int32)
            if x.shape[0] == 0:
                return self._empty(x)
            mg_gu, mg_dn = (getattr(w, "main_grad", None) for w in (self.w_gate_up, self.w_down))
            if (torch.is_grad_enabled() and mg_gu is not None and mg_dn is not None
                    and mg_gu.dtype == torch.float32 and mg_dn.dtype == torch.float32 and self.inter % 8 == 0
                    and os.environ.get("ST_MOE_FP32_WGRAD", "1") == "1"):
                mode = _vendor_expert_gemms()
                if mode == "0":
                    counts_host = None
                elif mode == "1" and counts_host is None:
                    counts_host = torch.diff(offs, prepend=offs.new_zeros(1)).tolist()  # one host read
                return _ExpertFFNFn.apply(x.contiguous(), offs, self.w_gate_up, self.w_down, counts_host)
            gu = torch._grouped_mm(x.contiguous(), self.w_gate_up.transpose(-2, -1), offs=offs)
            return torch._grouped_mm(ops.swiglu(gu), self.w_down.transpose(-2, -1), offs=offs)
        if counts is None:
            counts = torch.diff(offs.long(), prepend=offs.new_zeros(1, dtype=torch.long))
        if isinstance(counts, torch.Tensor):
            counts = counts.tolist()
        outs = []
        off = 0
        for e, n in enumerate(counts):
            if n == 0:
                continue
            xe = x[off: off + n]
            gu = torch.matmul(xe, self.w_gate_up[e].t())
            outs.append(torch.matmul(ops.swiglu(gu), self.w_down[e].t()))
            off += n
        if off < x.shape[0]:  # padding rows past the last expert: zero output, connected
            outs.append(x[off:] * 0)
        if not outs:
            return self._empty(x)
        return torch.cat(outs, 0)

    def _empty(self, x: torch.Tensor) -> torch.Tensor:
        """No rows routed here: an empty result that stays CONNECTED to the graph
        (x and the expert weights), so backward still reaches the dispatch
        all-to-all on this rank -- every EP peer must issue the same collectives."""
        z = (x.sum() + self.w_gate_up.sum() + self.w_down.sum()) * 0
        return z.to(x.dtype).expand(0, self.hidden)


class MoELayer(nn.Module):
    def __init__(self, cfg: ModelConfig, sequence_parallel: bool = False):
        super().__init__()
        ep = mesh.ep_size()
        if cfg.num_experts % ep:
            raise ValueError(f"num_experts {cfg.num_experts} not divisible by ep {ep}")
        self.num_experts, self.top_k = cfg.num_experts, cfg.num_experts_per_tok
        self.ep, self.ep_rank = ep, mesh.ep_rank()
        self.num_local = cfg.num_experts // ep
        self.hidden = cfg.hidden_size
        self.sequence_parallel = sequence_parallel and mesh.tp_size() > 1
        self.router = MoERouter(cfg.hidden_size, cfg.num_experts, cfg.num_experts_per_tok, cfg.norm_topk_prob,
                                cfg.router_aux_loss_coef, cfg.initializer_range)
        self.experts = MoEExperts(self.num_local, cfg.hidden_size, cfg.moe_intermediate_size, cfg.initializer_range,
                                  num_global=cfg.num_experts, ep_rank=self.ep_rank)
        for p in self.experts.parameters():
            p._st_expert = True  # reduced over the expert-DP group, not dense-DP
        self.last_aux_loss: torch.Tensor | None = None
        self.dropped_rows: torch.Tensor | None = None  # capacity dispatch: rows dropped in the last forward

    def reset_parameters(self) -> None:
        self.router.reset_parameters()
        self.experts.reset_parameters()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        tp_group = mesh.tp_group()
        tp = mesh.tp_size()
        if self.sequence_parallel:
            # route on the local sequence shard, then gather tokens + routing
            # results: gradients of both come back summed over TP by the
            # reduce-scatter, which is exactly the sum of the TP partials.
            B = x.shape[0]
            topw, topi, aux = self.router(x.reshape(-1, x.shape[-1]))
            k = self.top_k
            topw = AllGatherFromSequenceParallelRegion.apply(topw.view(B, -1, k), tp_group).reshape(-1, k)
            topi = C.all_gather(topi.view(B, -1, k).transpose(0, 1).contiguous(),
                                group=tp_group).transpose(0, 1).reshape(-1, k)
            x = AllGatherFromSequenceParallelRegion.apply(x, tp_group)
            x2 = x.reshape(-1, x.shape[-1])
        else:
            x2 = x.reshape(-1, x.shape[-1])
            topw, topi, aux = self.router(x2)
            if tp > 1:
                # experts see TP-partial intermediate shards: sum their input /
                # combine-weight gradients over TP in backward
                from ..parallel.tensor_parallel import CopyToTensorParallelRegion

                x2 = CopyToTensorParallelRegion.apply(x2, tp_group)
                topw = CopyToTensorParallelRegion.apply(topw, tp_group)
        shape = x.shape
        self.last_aux_loss = aux if self.training else None
        if self.ep > 1 and _DISPATCH["capacity_factor"] > 0:
            out = self._forward_ep_capacity(x2, topw, topi).view(shape)
            return self._tp_reduce(out, tp_group)
        # stable sort of the T*k (token, slot) entries by global expert + row gather
        perm = ops.moe.permutation(topi, self.num_experts)
        xs = ops.moe.gather_rows(x2, perm)  # rows sorted by global expert
        if self.ep == 1:
            y = self.experts(xs, perm.counts)  # device counts: no host sync on the grouped-GEMM path
        else:
            y = self._forward_ep_dropless(xs, perm.counts)
        out = ops.moe.combine(y, topw, perm).view(shape)
        return self._tp_reduce(out, tp_group)

    def _forward_ep_dropless(self, xs: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
        """Dropless expert parallelism with device-side counts (see ``ep_owner_positions``):
        one count all-gather, one dispatch exchange, the grouped expert GEMMs over the
        R_max-row buffer (device offsets), one combine exchange.  No host read of the
        routing on the xGMI transport; one per layer (the splits) on RCCL."""
        group = mesh.pgm.ep_group
        ep, El, k = self.ep, self.num_local, self.top_k
        comm = ep_comm_for(group)
        Tk = xs.shape[0]
        T_max = ep_rows_bound(Tk // k, group)
        R_max, Tk_max = ep * T_max * min(k, El), T_max * k
        if comm is not None and not (comm.ep_fits(R_max, xs) and comm.ep_fits(Tk_max, xs)):
            comm = None  # buffers too small for this shape: RCCL exchange
        M = ep_counts_matrix(counts, group, comm)
        # RCCL transport: ONE host read of the counts per layer forward, shared by the dispatch,
        # the combine and both backward exchanges (the xGMI push exchange reads none)
        Mh = M.detach().to("cpu", torch.int64) if comm is None else None
        mine = M[:, self.ep_rank * El:(self.ep_rank + 1) * El]
        offs = torch.cumsum(mine.sum(0), 0, dtype=torch.int32)  # grouped-GEMM offsets (device)
        # RCCL transport: the host counts size the expert buffers EXACTLY (the rows this rank
        # receives); the xGMI push exchange writes into R_max-row buffers (device counts), of
        # which the first offs[-1] rows are real -- the FFN then recomputes a over those
        # instead of keeping an R_max x I activation.  At Mixtral EP 8, R_max = 32,768 rows
        # against ~8,192 received: the exact buffers hold ~4x less per MoE layer.
        rows = int(Mh[:, self.ep_rank * El:(self.ep_rank + 1) * El].sum()) if Mh is not None else R_max
        xe = _EPExchange.apply(xs, M, El, 0, rows, (R_max, Tk_max), group, comm, Mh)
        xe._st_padded = Mh is None
        # host counts (RCCL exchange) hand the per-expert hipBLASLt path its row counts when
        # ST_MOE_VENDOR_GEMM asks for it (``_vendor_expert_gemms``: the grouped kernels win in
        # the step by default)
        mode = _vendor_expert_gemms()
        ch = Mh[:, self.ep_rank * El:(self.ep_rank + 1) * El].sum(0).tolist() if Mh is not None else None
        if ch is not None and (mode == "0" or (mode == "auto" and not (El <= 4 and sum(ch) >= 4096 * El))):
            ch = None
        ye = self.experts(xe, offs=offs, counts_host=ch)
        self.dropped_rows = xs.new_zeros((), dtype=torch.int64)  # dropless by construction
        self.ep_rows_sent = Tk - mine[self.ep_rank].sum()  # rows that left this rank (device)
        return _EPExchange.apply(ye, M, El, 1, Tk, (R_max, Tk_max), group, comm, Mh)

    def _tp_reduce(self, out: torch.Tensor, tp_group) -> torch.Tensor:
        # expert down-projections are TP partial sums: reduce once, after the combine
        if self.sequence_parallel:
            return ReduceScatterToSequenceParallelRegion.apply(out, tp_group)
        if mesh.tp_size() > 1:
            return ReduceFromTensorParallelRegion.apply(out, tp_group)
        return out

    def _forward_ep_capacity(self, x2: torch.Tensor, topw: torch.Tensor, topi: torch.Tensor) -> torch.Tensor:
        """Expert-parallel MoE with static per-(source, destination) capacity: every
        buffer size is known on the host, so no routing count is ever read back (the
        dropless path reads one [2, ep] count matrix per layer).  The tokens go in
        ``moe_ep_chunks`` chunks: all dispatch all-to-alls are issued first (async,
        RCCL's stream), then chunk c's expert GEMMs run while chunk c+1's rows are in
        flight, and each chunk's combine all-to-all overlaps the next chunk's experts.
        Rows past a destination's capacity are dropped (their combine weight has
        nothing to add: the token keeps its residual), counted in ``dropped_rows``
        (a device scalar).  Reference: dispatch_tokens / gather_tokens,
        scaletorch/parallel/expert_parallel/ep_comms.py:41-171 (host-synced splits)."""
        group = mesh.pgm.ep_group
        ep, k = self.ep, self.top_k
        T = x2.shape[0]
        lo, hi = ep_rows_range(T, group, agree=True)  # one [2] all-reduce: every rank sees the same range
        if lo != hi:  # the static buffers assume one token count on every EP rank (raised on every rank)
            raise ValueError(f"capacity EP dispatch needs the same token count on every EP rank (got {lo}..{hi}); "
                             "use the dropless dispatch (--moe_capacity_factor 0)")
        nch = max(1, min(_DISPATCH["chunks"], T))
        cf = _DISPATCH["capacity_factor"]
        bounds = [T * c // nch for c in range(nch + 1)]
        dropped = torch.zeros((), dtype=torch.int64, device=x2.device)
        stage = []
        for c in range(nch):
            a, b = bounds[c], bounds[c + 1]
            perm = ops.moe.permutation(topi[a:b], self.num_experts)
            xs = ops.moe.gather_rows(x2[a:b], perm)
            rows = (b - a) * k
            cap = max(1, math.ceil(cf * rows / ep))
            plan = capacity_plan(perm.counts, ep, cap, rows)
            send = torch.where(plan.send_valid[:, None], xs.index_select(0, plan.send_idx), xs.new_zeros(()))
            recv_kept = C.all_to_all(plan.kept.to(torch.int32).contiguous(), group=group)  # [src, local expert]
            holder: list = []
            r = _A2AStart.apply(send, holder, group)
            stage.append((perm, topw[a:b], plan, recv_kept, r, holder))
            dropped = dropped + (rows - plan.keep_row.sum())
        back = []
        for perm, tw, plan, recv_kept, r, holder in stage:
            r = _A2AWait.apply(r, holder)
            order, _ = capacity_receive_order(recv_kept, plan.cap)
            ye = self.experts(r.index_select(0, order), recv_kept.sum(0))
            inv = torch.empty_like(order).scatter_(0, order, torch.arange(order.numel(), device=order.device))
            h2: list = []
            yb = _A2AStart.apply(ye.index_select(0, inv), h2, group)
            back.append((perm, tw, plan, yb, h2))
        outs = []
        for perm, tw, plan, yb, h2 in back:
            yb = _A2AWait.apply(yb, h2)
            ys = torch.where(plan.keep_row[:, None], yb.index_select(0, plan.back_idx), yb.new_zeros(()))
            outs.append(ops.moe.combine(ys, tw, perm))
        self.dropped_rows = dropped
        return torch.cat(outs, 0) if len(outs) > 1 else outs[0]

    # reference checkpoint names: experts.experts.{e}.{gate,up,down}_proj.weight
    def reference_items(self) -> dict[str, torch.Tensor]:
        out = {}
        I = self.experts.inter
        for e in range(self.num_local):
            gu = self.experts.w_gate_up[e].detach()
            out[f"experts.experts.{e}.gate_proj.weight"] = gu[:I]
            out[f"experts.experts.{e}.up_proj.weight"] = gu[I:]
            out[f"experts.experts.{e}.down_proj.weight"] = self.experts.w_down[e].detach()
        return out

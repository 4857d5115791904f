"""Context parallelism for long sequences (ring-attention semantics, KV all-gather transport).

Reference: RingAttentionFunc (scaletorch/parallel/context_parallel/context_parallel.py:83-473)
-- materialised S^2 scores per ring step on K/V expanded to all query heads,
contiguous chunks, and (in practice) never enabled by the trainer.

Here:
* sequences are split ZIG-ZAG (data/loader.py): with 2*cp chunks rank r owns
  chunks r and 2cp-1-r, so every rank does the same causal work;
* K/V travel at GQA size (Hkv heads, never expanded): per layer ONE RCCL
  all-gather of the packed local [K|V] block (xGMI all-gather uses every
  link), re-ordered into global sequence order, then each local query chunk
  runs the HIP flash kernel against the keys it can see ([0, chunk_end)) with
  its GLOBAL position offset -- no S^2 tensor, no per-step host sync;
* backward: the flash backward of each chunk yields dQ locally and dK/dV for
  the full prefix; dK|dV are summed and ONE reduce-scatter returns every rank
  its own slice;
* RoPE uses the loader's explicit global ``position_ids`` (the reference
  sliced a cp-partitioned table, wrong unless seq == max_pos).
A P2P ring transport (``ring_attention`` in this module) implements the
reference's rotation schedule with the same kernels, for configurations where
the gathered K/V would not fit; both produce identical results.
"""
from __future__ import annotations

import torch

from .. import ops
from ..dist import collectives as C
from ..dist import trace
from ..ops import _lib
from . import mesh


def _cp():
    pg = mesh.pgm
    return pg.cp_group, pg.cp_world_size, pg.cp_rank


def zigzag_chunk_starts(seq_len: int, cp: int, rank: int) -> tuple[int, int, int]:
    """(start of first local chunk, start of second, chunk length) in global positions."""
    c = seq_len // (2 * cp)
    return rank * c, (2 * cp - 1 - rank) * c, c


def _global_order_index(S: int, cp: int, device) -> torch.Tensor:
    """Index mapping rank-ordered gathered rows -> global sequence order (zig-zag)."""
    c = S // (2 * cp)
    src = torch.empty(S, dtype=torch.long)
    for r in range(cp):
        a, b, _ = zigzag_chunk_starts(S, cp, r)
        base = r * 2 * c
        src[a: a + c] = torch.arange(base, base + c)
        src[b: b + c] = torch.arange(base + c, base + 2 * c)
    return src.to(device)


def _gather_seq_dim1(x: torch.Tensor, group) -> torch.Tensor:
    """[B, s, ...] on every rank -> [B, cp*s, ...] in rank order."""
    xt = x.transpose(0, 1).contiguous()
    out = C.all_gather(xt, group=group)
    return out.transpose(0, 1)


def _reduce_scatter_seq_dim1(x: torch.Tensor, group) -> torch.Tensor:
    xt = x.transpose(0, 1).contiguous()
    trace.record("cp.dkv_reduce_scatter", xt, group_size=C.get_world_size(group))
    out = C.reduce_scatter(xt, group=group)
    return out.transpose(0, 1)


class _CPAttnFn(torch.autograd.Function):
    """K/V all-gather transport with the gather OVERLAPPED: the packed local [K|V]
    all-gather is issued async, and while it is in flight every local query chunk
    attends to its OWN chunk (the causal diagonal block, all local data); after
    the gather lands, each chunk attends to the keys before it ([0, g0), no mask)
    and the two partial results are combined by the LSE-merge kernel.  Backward:
    one flash backward per chunk over its visible prefix, writing dQ and dK/dV
    straight into their output buffers (the widest prefix first, the next one
    added in place), then ONE reduce-scatter.  Rounding: each chunk's partial is
    rounded to bf16 once by the kernel, and the in-place bf16 add evaluates the
    sum in fp32 and rounds once -- for the two zig-zag chunks that is bitwise the
    result of summing the two bf16 partials in an fp32 accumulator and casting
    once (tests/test_units.py::test_cp_dkv_inplace_add_equals_fp32_accumulation),
    without a full-S fp32 buffer."""

    @staticmethod
    def forward(ctx, q, kv, H, Hkv, D, scale, zigzag):
        """q [B, s, H, D] (roped), kv [B, s, 2*Hkv, D] (k roped | v) local shards."""
        group, cp, rank = _cp()
        B, s = q.shape[0], q.shape[1]
        S = s * cp
        xt = kv.transpose(0, 1).contiguous()
        trace.record("cp.kv_all_gather", xt, group_size=cp)
        gathered, work = C.all_gather(xt, group=group, async_op=True)
        chunks = _chunks_of(rank, S, cp, s, zigzag)
        parts = []
        for off, n, g0 in chunks:  # diagonal blocks: local keys only, under the gather
            o, l = ops.flash_attn_fwd(q[:, off: off + n], kv[:, off: off + n, :Hkv], kv[:, off: off + n, Hkv:],
                                      scale, True, g0, g0)
            parts.append((o, l))
        if work is not None:
            work.wait()
        kv_g = gathered.transpose(0, 1)  # [B, S, 2Hkv, D] rank order
        kv_g = kv_g.index_select(1, _global_order_index(S, cp, q.device)) if zigzag else kv_g.contiguous()
        k_full, v_full = kv_g[:, :, :Hkv], kv_g[:, :, Hkv:]
        outs, lses = [], []
        for (off, n, g0), (o, l) in zip(chunks, parts):
            if g0 > 0:  # every key of [0, g0) precedes every query of the chunk
                bo, bl = ops.flash_attn_fwd(q[:, off: off + n], k_full[:, :g0], v_full[:, :g0], scale, True, g0, 0)
                acc = o.float()
                _merge(acc, l, bo, bl)
                o = acc.to(q.dtype)
            outs.append(o)
            lses.append(l)
        out = torch.cat(outs, dim=1) if len(outs) > 1 else outs[0]
        ctx.save_for_backward(q, kv_g, out, *lses)
        ctx.meta = (H, Hkv, D, scale, zigzag, chunks, S)
        return out

    @staticmethod
    def backward(ctx, dout):
        """Two phases per chunk (csrc/flash_attn.hip's dS-materialising backward): first
        every chunk's dK/dV pass (dS tiles stored), then the dK/dV reduce-scatter is issued
        ASYNC and the chunks' dQ passes (dQ = dS K, HBM-bound) run while it is in flight;
        it is joined only at the very end.  (Shapes the dS path does not take run the
        one-shot backward in phase 1.)"""
        q, kv_g, out = ctx.saved_tensors[:3]
        lses = ctx.saved_tensors[3:]
        H, Hkv, D, scale, zigzag, chunks, S = ctx.meta
        group, cp, rank = _cp()
        k_full, v_full = kv_g[:, :, :Hkv], kv_g[:, :, Hkv:]
        dq = torch.empty_like(q)
        dkv = torch.empty(kv_g.shape, dtype=q.dtype, device=q.device)
        dout = dout.contiguous()
        order = sorted(range(len(chunks)), key=lambda i: -(chunks[i][2] + chunks[i][1]))  # widest prefix first
        covered = 0
        pending_dq = []  # (chunk, workspace) whose dQ pass runs under the reduce-scatter
        pending_bytes, budget = 0, _ds_budget_bytes()
        native = _lib.use_native(q)
        for i in order:
            off, n, g0 = chunks[i]
            kend = g0 + n
            args = (dout[:, off: off + n], q[:, off: off + n], k_full[:, :kend], v_full[:, :kend],
                    out[:, off: off + n].contiguous(), lses[i], scale, True, g0, 0)
            first = covered == 0
            if first:
                dkv[:, kend:].zero_()
                covered = kend
            ws = None
            # the widest-prefix chunk (first in `order`) takes the dS path, so its HBM-bound dQ
            # pass runs under the dK/dV reduce-scatter; the others take the one-shot backward,
            # 2-20 % faster per chunk in isolation at the cp8 @ 32K shapes and no workspace
            # (profiles/r05/cp_flash_bwd_ab.log)
            if native and (first or not _CP_ONE_SHOT_REST[0]):
                dk_c, dv_c, ws = _lib.ops().flash_bwd_kv(*args, dkv[:, :kend, :Hkv] if first else None,
                                                         dkv[:, :kend, Hkv:] if first else None)
                if ws.numel() and pending_bytes + ws.numel() * ws.element_size() > budget and pending_dq:
                    # the kept workspaces would pass the budget: this chunk's dQ runs now and
                    # its workspace is freed before the next chunk (peak = budget
                    # + one chunk, not the sum over chunks)
                    _lib.ops().flash_bwd_q_ds(q[:, off: off + n], k_full[:, :kend], ws, scale, True, g0, 0,
                                              dq[:, off: off + n])
                    ws = False
                elif ws.numel():
                    pending_dq.append((i, ws))
                    pending_bytes += ws.numel() * ws.element_size()
                else:
                    ws = None
            if ws is None:  # one-shot backward (dQ now); ws False: dS path, dQ already done
                if first:
                    ops.flash_attn_bwd(*args, dq=dq[:, off: off + n], dk=dkv[:, :kend, :Hkv],
                                       dv=dkv[:, :kend, Hkv:], one_shot=True)
                    continue
                _, dk_c, dv_c = ops.flash_attn_bwd(*args, dq=dq[:, off: off + n], one_shot=True)
            if not first:
                dkv[:, :kend, :Hkv] += dk_c
                dkv[:, :kend, Hkv:] += dv_c
        if zigzag:
            dkv = dkv.index_select(1, _inverse(_global_order_index(S, cp, q.device)))  # back to rank order
        xt = dkv.transpose(0, 1).contiguous()
        trace.record("cp.dkv_reduce_scatter", xt, group_size=cp, overlapped=bool(pending_dq))
        rs, work = C.reduce_scatter(xt, group=group, async_op=True)
        for i, ws in pending_dq:  # dQ passes under the reduce-scatter
            off, n, g0 = chunks[i]
            _lib.ops().flash_bwd_q_ds(q[:, off: off + n], k_full[:, :g0 + n], ws, scale, True, g0, 0,
                                      dq[:, off: off + n])
        if work is not None:
            work.wait()
        return dq, rs.transpose(0, 1).contiguous(), None, None, None, None, None


_CP_ONE_SHOT_REST = [__import__("os").environ.get("ST_CP_ONE_SHOT_REST", "1") == "1"]


def _ds_budget_bytes() -> int:
    """Bytes of dS workspace the CP backward may keep alive for its deferred dQ passes
    (ST_CP_DS_BUDGET_GB, default 6 GB): the first chunk's workspace is always deferred, a
    later one only while the total stays within the budget."""
    import os

    return int(float(os.environ.get("ST_CP_DS_BUDGET_GB", "6")) * 1e9)


def _chunks_of(rank: int, S: int, cp: int, s: int, zigzag: bool):
    """[(local offset, length, global start)] of one rank's sequence shard."""
    if zigzag:
        a, b, c = zigzag_chunk_starts(S, cp, rank)
        return [(0, c, a), (c, c, b)]
    return [(0, s, rank * s)]


def _ring_exchange(tensors: list[torch.Tensor], group, cp: int, rank: int):
    """Async send of ``tensors`` to the next CP rank / receive from the previous one."""
    recv = [torch.empty_like(t) for t in tensors]
    return recv, _ring_p2p(tensors, recv, group, cp, rank)


def _ring_p2p(sends: list[torch.Tensor], recvs: list[torch.Tensor], group, cp: int, rank: int):
    """Post ``sends`` to the next CP rank and ``recvs`` from the previous one (async, one
    batch).  Messages between a pair of ranks match in issue order, so every rank must
    post its receives in the order its predecessor sends."""
    import torch.distributed as dist

    nxt = C.global_rank_of(group, (rank + 1) % cp)
    prv = C.global_rank_of(group, (rank - 1) % cp)
    ops = []
    for t in sends:
        trace.record("cp.ring_send_recv", t, peer=f"{nxt}<-{prv}", group_size=cp)
        ops.append(dist.P2POp(dist.isend, t, nxt, group))
    for r in recvs:
        ops.append(dist.P2POp(dist.irecv, r, prv, group))
    return dist.batch_isend_irecv(ops) if ops else []


class _RingAttnFn(torch.autograd.Function):
    """Ring transport: K/V (GQA-sized, packed) rotate around the CP ring; each
    step's block attention runs the flash kernel with global offsets while the
    next block is in flight (async RCCL p2p); partial results are combined by
    the LSE-merge kernel.  Backward rotates K/V again together with an fp32
    dK/dV accumulator that arrives back at its owner after cp hops."""

    @staticmethod
    def forward(ctx, q, kv, H, Hkv, D, scale, zigzag):
        group, cp, rank = _cp()
        B, s = q.shape[0], q.shape[1]
        S = s * cp
        qch = _chunks_of(rank, S, cp, s, zigzag)
        acc = [torch.zeros(B, n, H, D, dtype=torch.float32, device=q.device) for _, n, _ in qch]
        lse = [torch.full((B, H, n), float("-inf"), dtype=torch.float32, device=q.device) for _, n, _ in qch]
        cur = kv.contiguous()
        for j in range(cp):
            src = (rank - j) % cp
            pending = None
            if j < cp - 1:
                nxt_kv, pending = _ring_exchange([cur], group, cp, rank)
            for (ko, kn, kg) in _chunks_of(src, S, cp, s, zigzag):
                kc, vc = cur[:, ko: ko + kn, :Hkv], cur[:, ko: ko + kn, Hkv:]
                for i, (qo, qn, qg) in enumerate(qch):
                    if kg > qg + qn - 1:
                        continue  # block entirely in the future
                    bo, bl = ops.flash_attn_fwd(q[:, qo: qo + qn], kc, vc, scale, True, qg, kg)
                    _merge(acc[i], lse[i], bo, bl)
            if pending is not None:
                for w in pending:
                    w.wait()
                cur = nxt_kv[0]
        out = torch.cat([a.to(q.dtype) for a in acc], dim=1) if len(acc) > 1 else acc[0].to(q.dtype)
        ctx.save_for_backward(q, kv, out, *lse)
        ctx.meta = (H, Hkv, D, scale, zigzag)
        return out

    @staticmethod
    def backward(ctx, dout):
        """K/V rotate as in the forward.  The fp32 dK/dV accumulator of a block follows
        it one step BEHIND: at step j a rank computes its partial for the block in hand
        into a fresh buffer, and only then adds the accumulator that the previous rank
        finished at the end of ITS step j-1 -- exchanged in the same async batch as this
        step's K/V, so it travels during this step's flash backward -- and forwards the
        sum with the next step's batch.  After cp steps every accumulator is home; only
        the last hop is exposed.  Within each batch the accumulator precedes the K/V
        block on both ends (messages between a pair match in issue order)."""
        q, kv, out = ctx.saved_tensors[:3]
        lses = ctx.saved_tensors[3:]
        H, Hkv, D, scale, zigzag = ctx.meta
        group, cp, rank = _cp()
        B, s = q.shape[0], q.shape[1]
        S = s * cp
        qch = _chunks_of(rank, S, cp, s, zigzag)
        dout = dout.contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        cur = kv.contiguous()
        a_out = None  # accumulator finished last step, forwarded in this step's exchange
        for j in range(cp):
            src = (rank - j) % cp
            sends, recvs = [], []
            a_in = kv_next = None
            if a_out is not None:
                sends.append(a_out)
            if j < cp - 1:
                sends.append(cur)
            if j >= 1:  # accumulator of this block from the previous rank (its step j-1)
                a_in = torch.empty(kv.shape, dtype=torch.float32, device=q.device)
                recvs.append(a_in)
            if j < cp - 1:
                kv_next = torch.empty_like(cur)
                recvs.append(kv_next)
            # one batch: the accumulator and K/V travel in the same group in both directions
            # (at cp = 2 next == prev: separate send-only groups would meet head-on)
            works = _ring_p2p(sends, recvs, group, cp, rank)  # joined below, after this step's compute
            part = torch.zeros(kv.shape, dtype=torch.float32, device=q.device)
            for (ko, kn, kg) in _chunks_of(src, S, cp, s, zigzag):
                kc, vc = cur[:, ko: ko + kn, :Hkv], cur[:, ko: ko + kn, Hkv:]
                for i, (qo, qn, qg) in enumerate(qch):
                    if kg > qg + qn - 1:
                        continue
                    g_q, g_k, g_v = ops.flash_attn_bwd(dout[:, qo: qo + qn], q[:, qo: qo + qn], kc, vc,
                                                       out[:, qo: qo + qn].contiguous(), lses[i], scale, True,
                                                       qg, kg)
                    dq[:, qo: qo + qn].add_(g_q)  # fp32 += bf16: one pass, no upcast copy
                    part[:, ko: ko + kn, :Hkv].add_(g_k)
                    part[:, ko: ko + kn, Hkv:].add_(g_v)
            for w in works:
                w.wait()
            if a_in is not None:
                part.add_(a_in)
            a_out = part
            if kv_next is not None:
                cur = kv_next
        home = torch.empty(kv.shape, dtype=torch.float32, device=q.device)
        works = _ring_p2p([a_out], [home], group, cp, rank)  # own block's accumulator: the last hop
        for w in works:
            w.wait()
        return dq.to(q.dtype), home.to(kv.dtype), None, None, None, None, None


def _merge(acc: torch.Tensor, lse: torch.Tensor, bo: torch.Tensor, bl: torch.Tensor) -> None:
    """acc/lse <- online-softmax combination with a block result (HIP kernel on GPU)."""
    if _lib.use_native(acc):
        _lib.ops().lse_merge_(acc, lse, bo, bl)
        return
    L = torch.logaddexp(lse, bl)
    wa = torch.exp(lse - L).nan_to_num(0.0).transpose(1, 2)[..., None]
    wb = torch.exp(bl - L).nan_to_num(0.0).transpose(1, 2)[..., None]
    acc.copy_(acc * wa + bo.float() * wb)
    lse.copy_(L)


# ---------------------------------------------------------------- Ulysses (all-to-all) transport
def _a2a(x: torch.Tensor, group) -> torch.Tensor:
    """all_to_all_single over dim 0 (= destination rank on input, source rank on output)."""
    trace.record("cp.ulysses_all_to_all", x, group_size=C.get_world_size(group))
    return C.all_to_all(x.contiguous(), group=group)


def _kv_heads_for(Hkv: int, P: int) -> int:
    """kv heads per rank after the head scatter (GQA groups stay whole)."""
    if Hkv % P == 0:
        return Hkv // P
    if P % Hkv == 0:
        return 1  # kv heads replicated P/Hkv times, one per rank
    raise ValueError(f"ulysses needs Hkv % cp == 0 or cp % Hkv == 0 (Hkv={Hkv}, cp={P})")


def _scatter_heads(x: torch.Tensor, P: int, group) -> torch.Tensor:
    """[B, s, P*h, D] sequence shard -> [B, P*s, h, D] head shard (rank order of sequence)."""
    B, s, HH, D = x.shape
    h = HH // P
    t = x.view(B, s, P, h, D).permute(2, 0, 1, 3, 4)  # [P(dst), B, s, h, D]
    r = _a2a(t, group)  # [P(src), B, s, h, D]
    return r.permute(1, 0, 2, 3, 4).reshape(B, P * s, h, D)


def _gather_heads(x: torch.Tensor, P: int, group) -> torch.Tensor:
    """Inverse of _scatter_heads: [B, P*s, h, D] -> [B, s, P*h, D]."""
    B, S, h, D = x.shape
    s = S // P
    t = x.view(B, P, s, h, D).permute(1, 0, 2, 3, 4)  # [P(dst: seq owner), B, s, h, D]
    r = _a2a(t, group)  # [P(src: head owner), B, s, h, D]
    return r.permute(1, 2, 0, 3, 4).reshape(B, s, P * h, D)


class _UlyssesAttnFn(torch.autograd.Function):
    """DeepSpeed-Ulysses sequence parallelism (absent in the reference):
    one all-to-all turns the sequence-sharded q/k/v into head-sharded full
    sequences, the HIP flash kernel runs plain causal attention on H/cp heads,
    and one all-to-all returns the output to sequence shards.  4 all-to-alls
    per layer (fwd 2, bwd 2) of activation size / cp each -- per-link traffic
    independent of cp, versus the K/V all-gather's (cp-1)/cp of the sequence;
    best when heads >= cp and the sequence is long."""

    @staticmethod
    def forward(ctx, q, kv, H, Hkv, D, scale, zigzag):
        group, P, rank = _cp()
        if H % P:
            raise ValueError(f"ulysses needs num_attention_heads % cp == 0 (H={H}, cp={P})")
        B, s = q.shape[0], q.shape[1]
        S = s * P
        hk = _kv_heads_for(Hkv, P)
        k, v = kv[:, :, :Hkv], kv[:, :, Hkv:]
        rep = (P * hk) // Hkv
        if rep > 1:  # every rank needs the kv head of its query-head block
            k, v = k.repeat_interleave(rep, dim=2), v.repeat_interleave(rep, dim=2)
        qf = _scatter_heads(q, P, group)  # [B, S, H/P, D]
        kvf = _scatter_heads(torch.cat([k.reshape(B, s, P, hk, D), v.reshape(B, s, P, hk, D)], dim=3)
                             .reshape(B, s, P * 2 * hk, D), P, group)  # [B, S, 2hk, D]
        if zigzag:
            idx = _global_order_index(S, P, q.device)
            qf, kvf = qf.index_select(1, idx), kvf.index_select(1, idx)
        kf, vf = kvf[:, :, :hk], kvf[:, :, hk:]
        o, lse = ops.flash_attn_fwd(qf, kf, vf, scale, True, 0, 0)
        ctx.save_for_backward(qf, kvf, o, lse)
        ctx.meta = (H, Hkv, hk, rep, D, scale, zigzag, S)
        if zigzag:
            o = o.index_select(1, _inverse(idx))
        return _gather_heads(o, P, group)  # [B, s, H, D]

    @staticmethod
    def backward(ctx, dout):
        qf, kvf, o, lse = ctx.saved_tensors
        H, Hkv, hk, rep, D, scale, zigzag, S = ctx.meta
        group, P, rank = _cp()
        B, s = dout.shape[0], dout.shape[1]
        dof = _scatter_heads(dout.contiguous(), P, group)
        if zigzag:
            idx = _global_order_index(S, P, dout.device)
            dof = dof.index_select(1, idx)
        kf, vf = kvf[:, :, :hk], kvf[:, :, hk:]
        dq, dk, dv = ops.flash_attn_bwd(dof.contiguous(), qf, kf, vf, o, lse, scale, True, 0, 0)
        dkv = torch.cat([dk, dv], dim=2)
        if zigzag:
            inv = _inverse(idx)
            dq, dkv = dq.index_select(1, inv), dkv.index_select(1, inv)
        dq = _gather_heads(dq, P, group)  # [B, s, H, D]
        dkv = _gather_heads(dkv, P, group).view(B, s, P, 2, hk, D)  # per rank block [k heads | v heads]
        dk = dkv[:, :, :, 0].reshape(B, s, P * hk, D)
        dv = dkv[:, :, :, 1].reshape(B, s, P * hk, D)
        if rep > 1:  # sum the replicas of each kv head
            dk = dk.float().view(B, s, Hkv, rep, D).sum(3).to(dout.dtype)
            dv = dv.float().view(B, s, Hkv, rep, D).sum(3).to(dout.dtype)
        return dq, torch.cat([dk, dv], dim=2), None, None, None, None, None


def _inverse(idx: torch.Tensor) -> torch.Tensor:
    inv = torch.empty_like(idx)
    inv[idx] = torch.arange(idx.numel(), device=idx.device)
    return inv


_CP_COMM = "auto"
_CP_FNS = {"allgather": "_CPAttnFn", "ring": "_RingAttnFn", "ulysses": "_UlyssesAttnFn"}


def set_cp_comm(mode: str) -> None:
    global _CP_COMM
    if mode not in _CP_FNS and mode != "auto":
        raise ValueError(f"cp_comm must be auto or one of {sorted(_CP_FNS)}, got {mode!r}")
    _CP_COMM = mode


def resolve_cp_comm(cp: int) -> str:
    """``auto`` = the overlapped K/V all-gather at every cp.  On a fully connected
    xGMI node RCCL's all-gather / reduce-scatter drive all 7 links of a GPU at once,
    while the ring's point-to-point hops each use the ONE link to the next rank: at
    cp = 8 and 32K tokens a layer's K/V all-gather is 7 x 16 MiB over 7 links versus 7
    sequential 16 MiB hops (plus 7 fp32 dK/dV hops of 32 MiB) over one.  The gathered
    K/V costs 128 MiB per layer of HBM (4 GiB over 32 layers), nothing at 288 GB.
    ``ring`` stays selectable (--cp_comm ring) for multi-node CP where the ring's
    neighbour traffic is what the network favours."""
    if _CP_COMM != "auto":
        return _CP_COMM
    return "allgather"


def context_parallel_attention(qkv: torch.Tensor, cos, sin, position_ids, H: int, Hkv: int, D: int,
                               scale: float, zigzag: bool | None = None) -> torch.Tensor:
    """qkv [B, s, (H+2Hkv)*D] local CP shard -> attention output [B, s, H*D]."""
    B, s = qkv.shape[0], qkv.shape[1]
    if zigzag is None:
        zigzag = _ZIGZAG
    qkv4 = qkv.view(B, s, H + 2 * Hkv, D)
    q = ops.apply_rope(qkv4[:, :, :H], cos, sin, position_ids)
    k = ops.apply_rope(qkv4[:, :, H: H + Hkv], cos, sin, position_ids)
    kv = torch.cat([k, qkv4[:, :, H + Hkv:]], dim=2)
    fn = globals()[_CP_FNS[resolve_cp_comm(mesh.cp_size())]]
    out = fn.apply(q.contiguous(), kv.contiguous(), H, Hkv, D, scale, zigzag)
    return out.reshape(B, s, H * D)


def update_rope_for_context_parallel(cos: torch.Tensor, sin: torch.Tensor, seq_len: int, zigzag: bool = True):
    """Per-rank cos/sin rows (reference API, context_parallel.py:427-473); prefer position_ids."""
    from ..data.loader import cp_slice_indices

    pg = mesh.pgm
    idx = cp_slice_indices(seq_len, pg.cp_world_size, pg.cp_rank, zigzag).to(cos.device)
    return cos[idx], sin[idx]


_ZIGZAG = True


def set_cp_zigzag(flag: bool) -> None:
    global _ZIGZAG
    _ZIGZAG = bool(flag)


def apply_context_parallel(model, zigzag: bool = True):
    """Reference-compatible entry point: models here read the CP size from the
    mesh at forward time, so this only records the chunking mode (which must
    match the data loader's)."""
    set_cp_zigzag(zigzag)
    return model

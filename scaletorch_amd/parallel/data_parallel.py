"""Data parallelism: flat parameter / fp32 gradient arenas + bucketed, overlapped
RCCL all-reduce.

Reference: DataParallelBucket / BucketManager in
scaletorch/parallel/data_parallel/{data_parallel.py,bucket.py}.  MI355X-first
design and fixes:

* ``GradArena`` flattens every trainable parameter of one reduction group into
  ONE contiguous bf16 buffer (``param.data`` becomes a view) and gives each a
  ``main_grad`` view into ONE contiguous fp32 buffer.  Fused ops accumulate
  weight gradients straight into ``main_grad`` (GEMM epilogue, ops/grad.py);
  the optimizer step is then a single kernel over the arena (optim.py).
* Buckets are contiguous ranges of the arena in REVERSE registration order
  (= backward order), so a bucket fills while backward is still running and
  its all-reduce is issued immediately (async on RCCL's stream, overlapped
  with the remaining backward GEMMs); the reference packed buckets by size
  (best-fit), which fires them in no useful order.
* Gradient accumulation: ``no_sync()`` covers only the first GA-1
  micro-batches (``require_backward_grad_sync``); the reference wrapped ALL
  micro-batches and never reduced.
* Bucket size defaults to 64 Mi elements (``--bucket_size_mb 256`` of fp32): on 8x
  MI355X (7 xGMI links/GPU, ring per-link bound) large messages amortise RCCL launch
  latency; a bucket closes at the first parameter that takes it past the size, so a
  Llama-3-8B step issues ~66 buckets (~2 per decoder layer of 218 M parameters),
  the first right after the LM head's backward.  128 / 512 MiB measured equal on
  one GPU (profiles/r02/bucket_size_mbs6_ab.log).
* Reduction dtype: fp32 (exact) or bf16 (half the xGMI bytes; the arena keeps
  accumulating in fp32 and only the cross-rank sum is bf16).
* Dense parameters reduce over DP x CP x EP, expert parameters over DP x CP
  (mesh.py); the reference skipped CP grads when DP == 1.
"""
from __future__ import annotations

import contextlib
import math
import os
from collections import defaultdict

import torch
import torch.distributed as dist
import torch.nn as nn

from ..dist import collectives as C
from ..dist import trace
from . import mesh

ALIGN = 64  # elements: keeps every param view 128-B aligned for 16-B vector loads


def _is_expert(p) -> bool:
    return bool(getattr(p, "_st_expert", False))


def _is_tp_sharded(p) -> bool:
    return bool(getattr(p, "_st_tp_sharded", False))


class Bucket:
    __slots__ = ("start", "end", "params", "pending", "handle", "comm_buf", "comm_out", "launched",
                 "shard_lo", "shard_hi", "state_lo", "ag_handle", "opt_event")

    def __init__(self, start: int, end: int, params: list):
        self.start, self.end, self.params = start, end, params
        self.pending = 0
        self.handle = None
        self.comm_buf = None
        self.comm_out = None
        self.launched = False
        self.shard_lo, self.shard_hi, self.state_lo = start, end, start
        self.ag_handle = None
        self.opt_event = None  # side-stream optimizer update of this bucket (optim.py overlap)


def _is_rccl(group) -> bool:
    """RCCL (backend "nccl") process group: AVG reductions and in-place
    reduce-scatter (recv = send + rank * count) are used; gloo gets SUM + divide."""
    return dist.get_backend(group) == "nccl"


def _aligned(n: int) -> int:
    return math.ceil(n / ALIGN) * ALIGN


def _wait_wgrad_stream(stream, device) -> None:
    """Order ``stream`` after every weight gradient issued so far on the side wgrad
    stream (ops/grad.py ``ST_WGRAD_STREAM=side``); no-op otherwise."""
    from ..ops.grad import wgrad_side_stream

    ws = wgrad_side_stream(device)
    if ws is not None:
        stream.wait_stream(ws)


class GradArena:
    """Flat parameter + fp32 gradient storage for one reduction group.

    ``zero1``: ZeRO stage-1 / distributed optimizer.  Every bucket is padded to
    a multiple of ``world * ALIGN`` and split evenly over the group; backward
    REDUCE-SCATTERS each bucket (half the bytes of an all-reduce land on this
    rank: only its shard is reduced), the optimizer updates only this rank's
    shards (fp32 master / m / v are 1/world of the arena), and the updated bf16
    shards are ALL-GATHERED back bucket by bucket in forward order, each
    forward layer waiting only for the bucket that holds its weights.
    Reference: the FSDP/ZeRO examples (examples/FSDP2/*);
    design is Megatron's distributed optimizer on our arenas.
    """

    def __init__(self, params: list[nn.Parameter], group, name: str, bucket_size: int = 64 * 1024 * 1024,
                 reduce_dtype: torch.dtype = torch.float32, grad_dtype: torch.dtype = torch.float32,
                 use_counts: dict | None = None, zero1: bool = False):
        self.name, self.group = name, group
        self.world = C.get_world_size(group)
        self.rank = C.get_rank(group) if self.world > 1 else 0
        self.zero1 = bool(zero1) and self.world > 1
        # expert grads already SUM the contributions of the ep data replicas that routed tokens
        # to them (all-to-all); dividing by ep turns that into the data-parallel mean
        self.post_scale = 1.0 / mesh.ep_size() if name == "expert" else 1.0
        self.reduce_dtype = reduce_dtype
        self.params = params
        if not params:
            raise ValueError("empty arena")
        dtype = params[0].dtype
        device = params[0].device
        if any(p.dtype != dtype for p in params):
            raise ValueError(f"arena {name}: mixed parameter dtypes")
        # bucket membership first (contiguous runs in registration = backward order, params
        # never split), then the layout: TP-sharded / expert params first, TP-replicated last
        # (grad-norm dedup segments); under ZeRO-1 each bucket is padded to world * ALIGN
        runs, cur, size = [], [], 0
        for p in params:
            cur.append(p)
            size += _aligned(p.numel())
            if size >= bucket_size:
                runs.append(cur)
                cur, size = [], 0
        if cur:
            runs.append(cur)
        quantum = ALIGN * (self.world if self.zero1 else 1)
        offs, off, spans = [], 0, []
        for run in runs:
            start = off
            for p in run:
                offs.append(off)
                off += _aligned(p.numel())
            off = start + math.ceil((off - start) / quantum) * quantum
            spans.append((start, off, run))
        self.numel = off
        self.offsets = offs
        self.param_flat = torch.zeros(self.numel, dtype=dtype, device=device)
        self.grad_flat = torch.zeros(self.numel, dtype=grad_dtype, device=device)
        for p, o in zip(params, offs):
            n = p.numel()
            view = self.param_flat[o: o + n].view_as(p)
            view.copy_(p.data)
            p.data = view
            p.main_grad = self.grad_flat[o: o + n].view_as(p)
        # segment boundary: [0, repl_start) sharded, [repl_start, numel) TP-replicated
        self.repl_start = self.numel
        for p, o in zip(params, offs):
            if not (_is_tp_sharded(p) or _is_expert(p)):
                self.repl_start = o
                break
        self.buckets: list[Bucket] = [Bucket(s, e, run) for s, e, run in spans]
        # optimizer segments: (arena_lo, arena_hi, state_lo); the whole arena, or this
        # rank's shard of every bucket under ZeRO-1
        state = 0
        for b in self.buckets:
            if self.zero1:
                n = (b.end - b.start) // self.world
                b.shard_lo = b.start + self.rank * n
                b.shard_hi = b.shard_lo + n
            b.state_lo = state
            state += b.shard_hi - b.shard_lo
        self.state_numel = state
        self.expected = {}
        self.bucket_of = {}
        for i, b in enumerate(self.buckets):
            for p in b.params:
                self.bucket_of[id(p)] = i
                self.expected[id(p)] = (use_counts or {}).get(id(p), 1)
        self.remaining = {}
        # optimizer side stream (set by DataParallel on GPU): per-bucket grad sum-of-squares
        # during backward (world == 1) and the overlapped optimizer update (optim.py)
        self.side_stream = None
        self.sq_acc = None
        self.sq_count = 0
        self.reset_counts()

    def reset_counts(self) -> None:
        self.remaining = dict(self.expected)
        for b in self.buckets:
            b.pending = len(b.params)
            b.handle = None
            b.launched = False

    def zero_grad(self) -> None:
        self.grad_flat.zero_()
        for p in self.params:
            p._st_fresh = False

    def mark_fresh(self) -> None:
        """Lazy zeroing: the first gradient write of the next step overwrites
        (ops/grad.py ``take_fresh``), so no fill pass over the fp32 arena."""
        for p in self.params:
            p._st_fresh = True

    def zero_fresh(self, params=None) -> None:
        """Zero the gradients nobody wrote this step (before they are reduced / read)."""
        for p in (self.params if params is None else params):
            if getattr(p, "_st_fresh", False):
                p.main_grad.zero_()
                p._st_fresh = False

    # ---------------------------------------------------------------- comm
    def launch(self, b: Bucket) -> None:
        if b.launched:
            return
        b.launched = True
        self.zero_fresh(b.params)
        if self.world == 1:
            if not dist.is_initialized() or dist.get_world_size() == 1:
                self._bucket_sumsq(b)  # only consumed when no TP/PP/EP peer shares the norm
            return
        g = self.grad_flat[b.start: b.end]
        st = self.side_stream if g.is_cuda else None
        if st is not None and self.reduce_dtype != g.dtype and os.environ.get("ST_CAST_SIDE", "1") == "1":
            # the fp32 -> bf16 cast of the bucket (6 B per gradient element: ~10 ms per step
            # for Llama-3-8B) runs on the side stream, off the backward's critical path; the
            # collective is issued from the same stream so RCCL's stream waits for the cast
            # (finish() joins the handle on the compute stream)
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(st):
                st.wait_event(ev)
                _wait_wgrad_stream(st, g.device)
                self._launch_comm(b, g)
            return
        if g.is_cuda:
            _wait_wgrad_stream(torch.cuda.current_stream(), g.device)
        self._launch_comm(b, g)

    def _launch_comm(self, b: Bucket, g: torch.Tensor) -> None:
        nccl = _is_rccl(self.group)
        if self.reduce_dtype != g.dtype:
            if b.comm_buf is None or b.comm_buf.numel() != g.numel():
                b.comm_buf = torch.empty(g.numel(), dtype=self.reduce_dtype, device=g.device)
            b.comm_buf.copy_(g)
            buf = b.comm_buf
        else:
            buf = g
        if not nccl:
            buf.div_(self.world)
        op = dist.ReduceOp.AVG if nccl else dist.ReduceOp.SUM
        if self.zero1:
            n = b.shard_hi - b.shard_lo
            if buf is g and nccl:  # in place: this rank's chunk of the bucket is the output
                out = self.grad_flat[b.shard_lo: b.shard_hi]
            else:
                if b.comm_out is None or b.comm_out.numel() != n:
                    b.comm_out = torch.empty(n, dtype=buf.dtype, device=buf.device)
                out = b.comm_out
            trace.record("dp.reduce_scatter", buf, group_size=self.world, arena=self.name)
            b.handle = dist.reduce_scatter_tensor(out, buf, op=op, group=self.group, async_op=True)
        else:
            trace.record("dp.all_reduce", buf, group_size=self.world, arena=self.name)
            b.handle = dist.all_reduce(buf, op=op, group=self.group, async_op=True)

    def _bucket_sumsq(self, b: Bucket) -> None:
        """world == 1: this bucket's gradients are final -> add their squared norm
        into ``sq_acc`` on the side stream while the rest of backward runs (the
        global-norm pass after backward then reads one scalar per arena)."""
        st = self.side_stream
        if st is None or os.environ.get("ST_BUCKET_NORM", "1") != "1":  # 0: one pass after backward (A/B)
            return
        from ..ops import _lib

        if _lib.probe_env("ST_NORM_PROBE_SKIP"):  # timing probe (optim.grad_norm), diagnostic library only
            return

        g = self.grad_flat[b.start: b.end]
        if not _lib.use_native(g) or g.numel() % 4:
            return
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(st):
            st.wait_event(ev)
            _wait_wgrad_stream(st, g.device)
            if self.sq_count == 0:
                if self.sq_acc is None:
                    self.sq_acc = torch.zeros(1, dtype=torch.float32, device=g.device)
                else:
                    self.sq_acc.zero_()
            _lib.ops().sumsq_(g, self.sq_acc)
        self.sq_count += 1

    def take_sumsq(self):
        """The backward-accumulated sum of squares (device scalar) if every bucket
        contributed this step, else None; joins the side stream."""
        if self.side_stream is None or self.world != 1 or self.sq_count != len(self.buckets):
            self.sq_count = 0
            return None
        self.sq_count = 0
        torch.cuda.current_stream().wait_stream(self.side_stream)
        return self.sq_acc

    def finish(self) -> None:
        """Launch whatever did not fire (unused params) and join every bucket."""
        for b in self.buckets:
            if not b.launched:
                self.launch(b)
        for b in self.buckets:
            if b.handle is not None:
                b.handle.wait()  # stream-ordered join (no host block on RCCL)
                b.handle = None
            if self.world == 1:
                continue
            if self.zero1:
                if b.comm_out is not None:
                    self.grad_flat[b.shard_lo: b.shard_hi].copy_(b.comm_out)
            elif b.comm_buf is not None:
                self.grad_flat[b.start: b.end].copy_(b.comm_buf)
        if self.post_scale != 1.0:
            for lo, hi, _ in self.segments():
                self.grad_flat[lo:hi].mul_(self.post_scale)

    # ---------------------------------------------------------------- ZeRO-1
    def segments(self) -> list[tuple[int, int, int]]:
        """(arena_lo, arena_hi, state_lo) ranges the optimizer owns on this rank."""
        if not self.zero1:
            return [(0, self.numel, 0)]
        return [(b.shard_lo, b.shard_hi, b.state_lo) for b in self.buckets]

    def gather_params(self) -> None:
        """All-gather the updated bf16 shards, first-used (last registered) bucket first."""
        if not self.zero1:
            return
        for b in reversed(self.buckets):
            trace.record("dp.all_gather", self.param_flat[b.start: b.end], group_size=self.world, arena=self.name)
            b.ag_handle = dist.all_gather_into_tensor(self.param_flat[b.start: b.end],
                                                      self.param_flat[b.shard_lo: b.shard_hi],
                                                      group=self.group, async_op=True)

    def wait_bucket(self, i: int) -> None:
        b = self.buckets[i]
        if b.ag_handle is not None:
            b.ag_handle.wait()
            b.ag_handle = None
        if b.opt_event is not None:
            torch.cuda.current_stream().wait_event(b.opt_event)
            b.opt_event = None

    def wait_params(self) -> None:
        for i in range(len(self.buckets)):
            self.wait_bucket(i)

    def mark_ready(self, p) -> bool:
        """Returns True when this call completed the bucket (and launched it)."""
        k = id(p)
        r = self.remaining.get(k)
        if r is None:
            return False
        r -= 1
        self.remaining[k] = r
        if r != 0:
            return False
        b = self.buckets[self.bucket_of[k]]
        b.pending -= 1
        if b.pending == 0:
            self.launch(b)
            return True
        return False


def _use_counts(model: nn.Module) -> dict:
    counts = defaultdict(int)
    for _, p in model.named_parameters(remove_duplicate=False):
        counts[id(p)] += 1
    return counts


class DataParallel(nn.Module):
    """Bucketed, backward-overlapped data parallelism over flat gradient arenas.

    Also used with DP world size 1: it still provides the arenas (main_grad,
    flat params) the fused optimizer and gradient accumulation rely on.
    """

    def __init__(self, module: nn.Module, bucket_size: int = 64 * 1024 * 1024,
                 reduce_dtype: torch.dtype | str = torch.float32, dense_group=None, expert_group=None,
                 expose_grads: bool = False, zero1: bool = False):
        super().__init__()
        self.module = module
        if zero1 and expose_grads:
            raise ValueError("zero1 keeps only a gradient shard per rank; expose_grads needs full grads")
        # expose_grads: after the sync, point ``p.grad`` at the reduced main_grad so stock
        # torch.optim optimizers can be used (examples); the arena optimizers read main_grad
        self.expose_grads = expose_grads
        if isinstance(reduce_dtype, str):
            reduce_dtype = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16,
                            "bfloat16": torch.bfloat16}[reduce_dtype]
        # no 5-D mesh configured: plain data parallelism over every rank of the job
        # (examples wrap a model without building a ProcessGroupManager)
        world_default = None if C.is_distributed() and C.get_world_size() > 1 else C.SINGLE
        if dense_group is None:
            dense_group = mesh.pgm.dense_dp_group if mesh.pgm else world_default
        if expert_group is None:
            expert_group = mesh.pgm.expert_dp_group if mesh.pgm else world_default
        self.require_backward_grad_sync = True
        self._callback_queued = False
        uses = _use_counts(module)
        params = [p for p in module.parameters() if p.requires_grad]
        params = list(reversed(params))  # backward order
        groups = {"dense": [p for p in params if not _is_expert(p)],
                  "expert": [p for p in params if _is_expert(p)]}
        # TP-replicated dense params go last (norm weights etc.; grad-norm dedup segment)
        groups["dense"] = ([p for p in groups["dense"] if _is_tp_sharded(p)]
                           + [p for p in groups["dense"] if not _is_tp_sharded(p)])
        self.arenas: list[GradArena] = []
        for name, ps in groups.items():
            if not ps:
                continue
            g = dense_group if name == "dense" else expert_group
            self.arenas.append(GradArena(ps, g, name, bucket_size, reduce_dtype, use_counts=uses, zero1=zero1))
        self.zero1 = any(a.zero1 for a in self.arenas)
        # one side stream per model on GPU: per-bucket gradient norms during backward and the
        # optimizer update overlapped with the NEXT forward (optim.py); each module's forward
        # pre-hook waits only for the buckets holding its own parameters
        dev = params[0].device if params else torch.device("cpu")
        self.side_stream = None
        if dev.type == "cuda" and os.environ.get("ST_OVERLAP_OPT", "1") == "1":
            # ST_SIDE_STREAM_PRIORITY: HIP stream priority of the side stream (0 = default,
            # -1 = high: its AdamW buckets are dispatched ahead of the forward's kernels)
            prio = int(os.environ.get("ST_SIDE_STREAM_PRIORITY", "0"))
            self.side_stream = torch.cuda.Stream(device=dev, priority=prio)
            for a in self.arenas:
                a.side_stream = self.side_stream
        if self.zero1 or self.side_stream is not None:
            self._install_param_waits()
        # TP-replicated params whose grads are TP-partial (per-head QK-norm weights; every
        # norm / router weight under sequence parallelism): summed over TP after backward
        self.tp_group = mesh.tp_group() if mesh.pgm else C.SINGLE
        self.tp_partial = [p for p in params if getattr(p, "_st_tp_partial_grad", False)]
        self._arena_of = {}
        for a in self.arenas:
            for p in a.params:
                self._arena_of[id(p)] = a
                p._st_grad_ready = self._grad_ready
                if not getattr(p, "_st_hooked", False):
                    p.register_post_accumulate_grad_hook(self._post_accumulate)
                    p._st_hooked = True

    # ---------------------------------------------------------------- hooks
    def _install_param_waits(self) -> None:
        """Each module waits (stream-ordered) for the buckets holding its own
        parameters right before its forward: the ZeRO-1 parameter all-gather and/or
        the side-stream optimizer update of the previous step overlap the next
        forward instead of preceding it."""
        where = {}
        for a in self.arenas:
            for i, b in enumerate(a.buckets):
                for p in b.params:
                    where[id(p)] = (a, i)

        def make_hook(needs):
            def hook(_mod, _inp):
                for a, i in needs:
                    a.wait_bucket(i)
            return hook

        self.wait_cover = {}
        for m in self.module.modules():
            params = list(m.parameters(recurse=False))
            # weights a module's forward reads without calling their owner (fused kernels)
            for sub in getattr(m, "_st_reads", ()):
                params += list(sub.parameters())
            needs = sorted({where[id(p)] for p in params if id(p) in where},
                           key=lambda t: (id(t[0]), t[1]))
            if needs:
                m.register_forward_pre_hook(make_hook(needs))
                self.wait_cover[m] = {id(p) for p in params}

    def gather_params(self) -> None:
        for a in self.arenas:
            a.gather_params()

    def uncovered_params(self, run_forward) -> list[str]:
        """Debug check: names of trainable parameters NOT covered by the bucket wait of
        any module whose forward actually ran in ``run_forward()`` -- such a weight
        could be read before its (side-stream / ZeRO-1) update lands."""
        if not hasattr(self, "wait_cover"):
            self._install_param_waits()
        called = []
        hook = nn.modules.module.register_module_forward_pre_hook(lambda m, _i: called.append(m))
        try:
            run_forward()
        finally:
            hook.remove()
        covered = set()
        for m in called:
            covered |= self.wait_cover.get(m, set())
        return [n for n, p in self.module.named_parameters() if p.requires_grad and id(p) not in covered]

    def wait_params(self) -> None:
        for a in self.arenas:
            a.wait_params()

    def _post_accumulate(self, p) -> None:
        """Params whose grads come through plain autograd (no fused op)."""
        if p.grad is None:
            return
        if self.expose_grads and p.grad.data_ptr() == p.main_grad.data_ptr():
            p.grad = None  # stale exposed view from the previous step: autograd accumulated into main_grad
            self._grad_ready(p)
            return
        if getattr(p, "_st_fresh", False):
            p._st_fresh = False
            p.main_grad.copy_(p.grad.view_as(p.main_grad))
        else:
            p.main_grad.add_(p.grad.view_as(p.main_grad))
        p.grad = None
        self._grad_ready(p)

    def _grad_ready(self, p) -> None:
        if not self._callback_queued:
            self._queue_callback()
        if self.require_backward_grad_sync:
            self._arena_of[id(p)].mark_ready(p)

    def _queue_callback(self) -> None:
        if self._callback_queued:
            return
        self._callback_queued = True
        try:
            torch.autograd.Variable._execution_engine.queue_callback(self._post_backward)
        except RuntimeError:  # not inside a backward pass (direct call)
            self._callback_queued = False

    def _post_backward(self) -> None:
        self._callback_queued = False
        if torch.cuda.is_available():  # side-stream weight gradients land before anyone reads them
            _wait_wgrad_stream(torch.cuda.current_stream(), torch.device("cuda", torch.cuda.current_device()))
        # final_backward False (interleaved pipeline: a chunk's last micro-batch, other
        # chunks still to come): buckets fire as their params become ready, but the
        # join and the TP-partial reduction wait for the step's last backward
        if self.require_backward_grad_sync and getattr(self, "final_backward", True):
            for a in self.arenas:
                a.finish()
                a.reset_counts()
            self._reduce_tp_partial()
            self._expose()

    def _expose(self) -> None:
        if not self.expose_grads:
            return
        for a in self.arenas:
            for p in a.params:
                p.grad = p.main_grad if p.main_grad.dtype == p.dtype else p.main_grad.to(p.dtype)

    def _reduce_tp_partial(self) -> None:
        if not self.tp_partial or C.get_world_size(self.tp_group) == 1:
            return
        flat = torch.cat([p.main_grad.reshape(-1) for p in self.tp_partial])
        C.all_reduce(flat, group=self.tp_group)
        off = 0
        for p in self.tp_partial:
            n = p.numel()
            p.main_grad.copy_(flat[off: off + n].view_as(p.main_grad))
            off += n

    # ---------------------------------------------------------------- API
    def forward(self, *args, **kwargs):
        out = self.module(*args, **kwargs)
        # parameters no forward hook covered (unused this step) must not be written by
        # backward while the previous optimizer update may still read their gradients
        self.wait_params()
        return out

    @contextlib.contextmanager
    def no_sync(self):
        prev = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = prev

    def zero_grad(self, set_to_none: bool = False) -> None:  # noqa: ARG002 - arenas are persistent
        from ..ops.grad import bump_weight_epoch

        bump_weight_epoch()  # a new step: the weights' W^T copies (dgrad layout) are stale
        for a in self.arenas:
            a.mark_fresh()
            a.reset_counts()
        for p in self.module.parameters():
            p.grad = None

    def sync_grads_manually(self) -> None:
        """Reduce every bucket now (pipeline schedules call this after the last backward)."""
        for a in self.arenas:
            for b in a.buckets:
                a.launch(b)
            a.finish()
            a.reset_counts()
        self._reduce_tp_partial()

    reset = zero_grad

    def grad_sumsq_segments(self):
        """(tensor, weight) pairs whose weighted squared norms sum to this rank's
        de-duplicated share of the global gradient norm.

        Without ZeRO-1 the shares are summed over the model-parallel group (dense
        grads are replicated over EP); with ZeRO-1 every rank holds a distinct
        shard of its reduction group and the shares are summed over ALL ranks
        (``norm_over_world``): sharded dense / expert weight 1, TP-replicated 1/tp."""
        tp = mesh.tp_size()
        ep = mesh.ep_size()
        out = []
        if self.zero1:
            for a in self.arenas:
                for lo, hi, _ in a.segments():
                    if a.name == "expert":
                        out.append((a.grad_flat[lo:hi], 1.0))
                        continue
                    r = a.repl_start
                    if lo < min(hi, r):
                        out.append((a.grad_flat[lo: min(hi, r)], 1.0))
                    if max(lo, r) < hi:
                        out.append((a.grad_flat[max(lo, r): hi], 1.0 / tp))
            return out
        for a in self.arenas:
            if a.name == "expert":
                out.append((a.grad_flat, 1.0))
            else:
                if a.repl_start > 0:
                    out.append((a.grad_flat[: a.repl_start], 1.0 / ep))
                if a.repl_start < a.numel:
                    out.append((a.grad_flat[a.repl_start:], 1.0 / (ep * tp)))
        return out

    def state_dict(self, *args, **kwargs):
        self.wait_params()
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        return self.module.load_state_dict(*args, **kwargs)


class BasicDataParallel(DataParallel):
    """Per-parameter all-reduce (bucket size 1 element) -- the reference's naive
    DataParallelBase/BasicDataParallel mode, kept for tests and teaching."""

    def __init__(self, module: nn.Module, **kw):
        super().__init__(module, bucket_size=1, **kw)


def mark_tp_sharded(module: nn.Module) -> None:
    """Tag parameters that are sharded across TP (not replicated)."""
    from .tensor_parallel import ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding

    for m in module.modules():
        if isinstance(m, (ColumnParallelLinear, VocabParallelEmbedding)):
            for p in m.parameters(recurse=False):
                p._st_tp_sharded = True
        elif isinstance(m, RowParallelLinear):
            m.weight._st_tp_sharded = True

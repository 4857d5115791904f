"""Pipeline parallelism: stage partitioning + AFAB and 1F1B schedules over RCCL p2p.

Reference: scaletorch/parallel/pipeline_parallel/{pipeline_parallel.py,pp_comms.py}.
Differences:
* stages are built stage-local (models/transformer.py ``stage_layer_range``:
  same even split with the remainder on the first stages, or an explicit
  ``layer_distribution``); embedding lives on the first stage, final
  norm + LM head on the last;
* every exchange is non-blocking (``batch_isend_irecv``); the paired
  send-forward/recv-backward of the 1F1B steady state is ONE grouped RCCL call;
  a received tensor is waited for right before its first use, and a pure send
  is never waited on the compute path: its work handle (and the tensor) is kept
  until the end of the step, so the next micro-batch's compute does not stall
  until the peer has posted its receive (the reference blocked on every
  send/recv, pp_comms.py:181-186).  The RCCL issue order is unchanged, so this
  cannot introduce a p2p deadlock;
* the schedule owns the loss (the reference stored it on the DP wrapper and
  crashed with PP+DP), losses stay on device (one host sync
  per step, at logging), and the DP gradient sync is enabled only for the last
  backward of the stage so its buckets overlap that backward;
* p2p shapes are known statically ([mbs, S/cp(/tp under SP), h]), no handshake.
"""
from __future__ import annotations

from collections import deque

import torch
import torch.distributed as dist

from ..dist import collectives as C
from ..dist import trace
from . import mesh

_STATS = {"send_forward": 0, "recv_forward": 0, "send_backward": 0, "recv_backward": 0}


def get_communication_stats() -> dict:
    return dict(_STATS)


def reset_communication_stats() -> None:
    for k in _STATS:
        _STATS[k] = 0


# sends in flight: (work handles, tensors kept alive) -- joined by ``wait_sends`` at step end
_INFLIGHT: list = []


def wait_sends() -> None:
    """Join every un-waited send (stream-ordered on RCCL, host wait on gloo)."""
    while _INFLIGHT:
        works, _keep = _INFLIGHT.pop()
        for w in works:
            w.wait()


def _p2p(send_fwd=None, send_bwd=None, recv_fwd_shape=None, recv_bwd_shape=None, dtype=torch.bfloat16,
         device=None):
    """One grouped exchange with the neighbouring stages; returns (recv_fwd, recv_bwd).

    Groups with a receive are joined before returning (the caller consumes the data
    next); send-only groups are left in flight (``wait_sends``)."""
    pg = mesh.pgm
    group = pg.pp_group
    ops, rf, rb = [], None, None
    if send_fwd is not None and pg.pp_next_rank is not None:
        ops.append(dist.P2POp(dist.isend, send_fwd.contiguous(), pg.pp_next_rank, group))
        _STATS["send_forward"] += 1
        trace.record("pp.send_forward", send_fwd, peer=pg.pp_next_rank)
    if send_bwd is not None and pg.pp_prev_rank is not None:
        ops.append(dist.P2POp(dist.isend, send_bwd.contiguous(), pg.pp_prev_rank, group))
        _STATS["send_backward"] += 1
        trace.record("pp.send_backward", send_bwd, peer=pg.pp_prev_rank)
    if recv_fwd_shape is not None and pg.pp_prev_rank is not None:
        rf = torch.empty(recv_fwd_shape, dtype=dtype, device=device)
        ops.append(dist.P2POp(dist.irecv, rf, pg.pp_prev_rank, group))
        _STATS["recv_forward"] += 1
        trace.record("pp.recv_forward", rf, peer=pg.pp_prev_rank)
    if recv_bwd_shape is not None and pg.pp_next_rank is not None:
        rb = torch.empty(recv_bwd_shape, dtype=dtype, device=device)
        ops.append(dist.P2POp(dist.irecv, rb, pg.pp_next_rank, group))
        _STATS["recv_backward"] += 1
        trace.record("pp.recv_backward", rb, peer=pg.pp_next_rank)
    if ops:
        works = dist.batch_isend_irecv(ops)
        if rf is None and rb is None:
            _INFLIGHT.append((works, [op.tensor for op in ops]))
        else:
            for w in works:
                w.wait()
    if rf is not None:
        rf.requires_grad_(True)
    return rf, rb


def pipeline_communicate(operation: str, tensor=None, shapes=None, dtype=torch.bfloat16, device=None):
    """Reference-compatible single-direction API (pp_comms.py:86-190)."""
    if operation == "recv_forward":
        return _p2p(recv_fwd_shape=shapes, dtype=dtype, device=device)[0]
    if operation == "send_forward":
        _p2p(send_fwd=tensor)
        return None
    if operation == "recv_backward":
        return _p2p(recv_bwd_shape=shapes, dtype=dtype, device=device)[1]
    if operation == "send_backward":
        _p2p(send_bwd=tensor)
        return None
    raise ValueError(operation)


def bidirectional_pipeline_communicate(operation: str, send_tensor, recv_shapes, dtype=torch.bfloat16, device=None):
    if operation == "send_fwd_recv_bwd":
        return _p2p(send_fwd=send_tensor, recv_bwd_shape=recv_shapes, dtype=dtype, device=device)[1]
    if operation == "send_bwd_recv_fwd":
        return _p2p(send_bwd=send_tensor, recv_fwd_shape=recv_shapes, dtype=dtype, device=device)[0]
    raise ValueError(operation)


class PipelineEngine:
    """Runs one optimizer step's worth of micro-batches through this stage."""

    def __init__(self, model, loss_fn, tensor_shape, dtype=torch.bfloat16, device=None,
                 gradient_checkpointing: bool = False, aux_loss_fn=None, head_kwargs_fn=None,
                 virtual_stages: int = 1):
        self.model = model  # DataParallel-wrapped stage
        self.loss_fn = loss_fn  # (logits or the fused head's loss, batch) -> scalar loss
        self.head_kwargs_fn = head_kwargs_fn  # batch -> extra model kwargs on the last stage (fused LM head)
        self.tensor_shape = tuple(tensor_shape)
        self.dtype, self.device = dtype, device
        self.gc = gradient_checkpointing
        self.aux_loss_fn = aux_loss_fn
        self.virtual_stages = virtual_stages

    @property
    def _first(self):
        return mesh.pgm.pp_is_first_stage

    @property
    def _last(self):
        return mesh.pgm.pp_is_last_stage

    def _forward(self, batch, x, num_micro):
        extra = self.head_kwargs_fn(batch) if (self._last and self.head_kwargs_fn is not None) else {}
        out = self.model(input_ids=batch["input_ids"] if self._first else None,
                         position_ids=batch["position_ids"], hidden_states=x, gradient_checkpointing=self.gc,
                         **extra)
        if self._last:
            loss = self.loss_fn(out, batch) / num_micro
            if self.aux_loss_fn is not None:
                aux = self.aux_loss_fn()
                if aux is not None:
                    loss = loss + aux / num_micro
            return loss
        if self.aux_loss_fn is not None:
            aux = self.aux_loss_fn()
            if aux is not None:  # MoE aux loss on non-last stages: fold into the output's graph
                out = _AttachAux.apply(out, aux / num_micro)
        return out

    def _backward(self, x, y, dy, last_backward: bool):
        self.model.require_backward_grad_sync = last_backward
        if self._last:
            y.backward()
        else:
            torch.autograd.backward(y, dy)
        self.model.require_backward_grad_sync = True
        return x.grad if x is not None else None

    def train_step_afab(self, data_iter, num_micro: int) -> torch.Tensor:
        ins, outs = deque(), deque()
        loss_sum = torch.zeros((), dtype=torch.float32, device=self.device)
        for _ in range(num_micro):
            x = _p2p(recv_fwd_shape=self.tensor_shape, dtype=self.dtype, device=self.device)[0]
            batch = next(data_iter)
            y = self._forward(batch, x, num_micro)
            if not self._last:
                _p2p(send_fwd=y.detach())
            else:
                loss_sum += y.detach().float()
            ins.append(x)
            outs.append(y)
        for i in range(num_micro):
            dy = _p2p(recv_bwd_shape=self.tensor_shape, dtype=self.dtype, device=self.device)[1]
            x, y = ins.popleft(), outs.popleft()
            dx = self._backward(x, y, dy, last_backward=(i == num_micro - 1))
            _p2p(send_bwd=dx)
        wait_sends()
        return loss_sum

    def train_step_1f1b(self, data_iter, num_micro: int) -> torch.Tensor:
        pg = mesh.pgm
        warmup = min(pg.pp_world_size - pg.pp_rank - 1, num_micro)
        steady = num_micro - warmup
        ins, outs = deque(), deque()
        loss_sum = torch.zeros((), dtype=torch.float32, device=self.device)
        n_bwd = 0

        def fwd(x):
            batch = next(data_iter)
            y = self._forward(batch, x, num_micro)
            if self._last:
                loss_sum.add_(y.detach().float())
            return y

        for _ in range(warmup):
            x = _p2p(recv_fwd_shape=self.tensor_shape, dtype=self.dtype, device=self.device)[0]
            y = fwd(x)
            _p2p(send_fwd=None if self._last else y.detach())
            ins.append(x)
            outs.append(y)
        x = _p2p(recv_fwd_shape=self.tensor_shape, dtype=self.dtype, device=self.device)[0] if steady > 0 else None
        for i in range(steady):
            y = fwd(x)
            dy = _p2p(send_fwd=None if self._last else y.detach(), recv_bwd_shape=self.tensor_shape,
                      dtype=self.dtype, device=self.device)[1]
            ins.append(x)
            outs.append(y)
            xo, yo = ins.popleft(), outs.popleft()
            n_bwd += 1
            dx = self._backward(xo, yo, dy, last_backward=(n_bwd == num_micro))
            if i == steady - 1:
                x = None
                _p2p(send_bwd=dx)
            else:
                x = _p2p(send_bwd=dx, recv_fwd_shape=self.tensor_shape, dtype=self.dtype, device=self.device)[0]
        for _ in range(warmup):
            xo, yo = ins.popleft(), outs.popleft()
            dy = _p2p(recv_bwd_shape=self.tensor_shape, dtype=self.dtype, device=self.device)[1]
            n_bwd += 1
            dx = self._backward(xo, yo, dy, last_backward=(n_bwd == num_micro))
            _p2p(send_bwd=dx)
        wait_sends()
        return loss_sum


    # ------------------------------------------------------------------ interleaved 1F1B
    def train_step_interleaved(self, data_iter, num_micro: int) -> torch.Tensor:
        """Interleaved 1F1B over this rank's ``virtual_stages`` model chunks
        (parallel/interleaved.py has the schedule and its deadlock-free proof by
        simulation).  Exchanges are batched p2p on the pipeline ring; a batch with
        a receive is joined before the data is used, send-only batches stay in
        flight until the end of the step.  The DP gradient sync is enabled for the
        last micro-batch of each chunk, so every bucket fires during backward."""
        from .interleaved import Exchange, build_schedule, bwd_chunk, fwd_chunk, micro_batch

        pg = mesh.pgm
        P, r, V, M = pg.pp_world_size, pg.pp_rank, self.virtual_stages, num_micro
        ring = pg.pp_group_ids
        nxt, prv = ring[(r + 1) % P], ring[(r - 1) % P]
        group = pg.pp_group
        batches: list = []

        def batch(m):
            while len(batches) <= m:
                batches.append(next(data_iter))
            return batches[m]

        inputs, grads = {}, {}        # fwd step -> received input; bwd step -> received output grad
        acts = {}                     # (chunk, micro) -> (x, y)
        outs, dxs = {}, {}            # fwd step -> output to send; bwd step -> input grad to send
        loss_sum = torch.zeros((), dtype=torch.float32, device=self.device)
        for a in build_schedule(P, V, M, r):
            if isinstance(a, Exchange):
                ops, rbufs = [], []
                for kind, k in a.send:
                    t = outs.pop(k) if kind == "fwd" else dxs.pop(k)
                    peer = nxt if kind == "fwd" else prv
                    ops.append(dist.P2POp(dist.isend, t.contiguous(), peer, group))
                    _STATS["send_forward" if kind == "fwd" else "send_backward"] += 1
                    trace.record("pp.send_" + ("forward" if kind == "fwd" else "backward"), t, peer=peer)
                for kind, k in a.recv:
                    buf = torch.empty(self.tensor_shape, dtype=self.dtype, device=self.device)
                    peer = prv if kind == "fwd" else nxt
                    ops.append(dist.P2POp(dist.irecv, buf, peer, group))
                    rbufs.append((kind, k, buf))
                    _STATS["recv_forward" if kind == "fwd" else "recv_backward"] += 1
                    trace.record("pp.recv_" + ("forward" if kind == "fwd" else "backward"), buf, peer=peer)
                works = dist.batch_isend_irecv(ops)
                if rbufs:
                    for w in works:
                        w.wait()
                    for kind, k, buf in rbufs:
                        if kind == "fwd":
                            inputs[k] = buf.requires_grad_(True)
                        else:
                            grads[k] = buf
                else:
                    _INFLIGHT.append((works, [op.tensor for op in ops]))
                continue
            kind, k = a
            if kind == "F":
                v, m = fwd_chunk(k, P, V), micro_batch(k, P, V)
                first, last = r == 0 and v == 0, r == P - 1 and v == V - 1
                x = None if first else inputs.pop(k)
                b = batch(m)
                extra = self.head_kwargs_fn(b) if (last and self.head_kwargs_fn is not None) else {}
                y = self.model(input_ids=b["input_ids"] if first else None, position_ids=b["position_ids"],
                               hidden_states=x, gradient_checkpointing=self.gc, chunk=v, **extra)
                aux = self.aux_loss_fn(v) if self.aux_loss_fn is not None else None
                if last:
                    y = self.loss_fn(y, b) / M
                    if aux is not None:
                        y = y + aux / M
                    loss_sum += y.detach().float()
                else:
                    if aux is not None:
                        y = _AttachAux.apply(y, aux / M)
                    outs[k] = y.detach()
                acts[(v, m)] = (x, y)
            else:
                v, m = bwd_chunk(k, P, V), micro_batch(k, P, V)
                x, y = acts.pop((v, m))
                self.model.require_backward_grad_sync = m == M - 1
                self.model.final_backward = k == M * V - 1
                if r == P - 1 and v == V - 1:
                    y.backward()
                else:
                    torch.autograd.backward(y, grads.pop(k))
                self.model.require_backward_grad_sync = True
                self.model.final_backward = True
                if x is not None:
                    dxs[k] = x.grad
        wait_sends()
        return loss_sum


class _AttachAux(torch.autograd.Function):
    """Identity on ``x`` whose backward also back-propagates d(aux)=1 into the aux loss."""

    @staticmethod
    def forward(ctx, x, aux):
        ctx.aux_shape = aux.shape
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g, torch.ones(ctx.aux_shape, device=g.device, dtype=torch.float32)


def train_step_pipeline_1f1b(engine: PipelineEngine, data_iter, num_micro: int):
    return engine.train_step_1f1b(data_iter, num_micro)


def train_step_pipeline_afab(engine: PipelineEngine, data_iter, num_micro: int):
    return engine.train_step_afab(data_iter, num_micro)

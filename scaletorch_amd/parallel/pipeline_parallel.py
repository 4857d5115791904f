"""Pipeline parallelism: stage partitioning + AFAB and 1F1B schedules over RCCL p2p.

Reference: scaletorch/parallel/pipeline_parallel/{pipeline_parallel.py,pp_comms.py}.
Differences:
* stages are built stage-local (models/transformer.py ``stage_layer_range``:
  same even split with the remainder on the first stages, or an explicit
  ``layer_distribution``); embedding lives on the first stage, final
  norm + LM head on the last;
* every exchange is non-blocking, and receives are POSTED AHEAD: activations
  travel on the pipeline communicator and gradients on a second one
  (every directed stage pair has its own 2-rank communicator, ``mesh.pp_channel``),
  so each direction between two stages is its own RCCL stream and a receive
  posted early can never block a send the peer is waiting for.
  The engine keeps the next micro-batch's receive in flight in each direction
  (``_Mailbox``, depth 2) and waits (a stream wait on RCCL) right before the
  data is used, so the transfer runs under the current micro-batch's forward /
  backward; a send is never waited on the compute path (its handle and tensor
  are kept until the end of the step).  The reference blocked on every
  send/recv (pp_comms.py:181-186);
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
    """One exchange with the neighbouring stages; returns (recv_fwd, recv_bwd).

    Each op runs on its directed channel's communicator (``mesh.pp_channel``).
    Receives are joined before returning (the caller consumes the data next);
    sends are left in flight (``wait_sends``)."""
    pg = mesh.pgm
    r = pg.pp_rank
    rf = rb = None
    if send_fwd is not None and pg.pp_next_rank is not None:
        _send(send_fwd, pg.pp_next_rank, pg.pp_channel("fwd", r), "forward")
    if send_bwd is not None and pg.pp_prev_rank is not None:
        _send(send_bwd, pg.pp_prev_rank, pg.pp_channel("bwd", r - 1), "backward")
    if recv_fwd_shape is not None and pg.pp_prev_rank is not None:
        rf = _Recv(recv_fwd_shape, dtype, device, pg.pp_prev_rank, pg.pp_channel("fwd", r - 1), "forward").get()
        rf.requires_grad_(True)
    if recv_bwd_shape is not None and pg.pp_next_rank is not None:
        rb = _Recv(recv_bwd_shape, dtype, device, pg.pp_next_rank, pg.pp_channel("bwd", r), "backward").get()
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


class _Recv:
    """One posted receive; ``get()`` waits for it (stream-ordered on RCCL)."""

    __slots__ = ("buf", "works")

    def __init__(self, shape, dtype, device, peer, group, kind):
        self.buf = torch.empty(shape, dtype=dtype, device=device)
        _STATS["recv_" + kind] += 1
        trace.record("pp.recv_" + kind, self.buf, peer=peer)
        self.works = dist.batch_isend_irecv([dist.P2POp(dist.irecv, self.buf, peer, group)])

    def get(self) -> torch.Tensor:
        for w in self.works:
            w.wait()
        self.works = ()
        return self.buf


class _Mailbox:
    """Receives of ONE direction from one peer, posted ``depth`` ahead in the order the
    peer sends them (a FIFO on that direction's own communicator), at most ``total``."""

    def __init__(self, total: int, shape, dtype, device, peer, group, kind: str, depth: int = 2):
        self.total, self.posted = total, 0
        self.args = (shape, dtype, device, peer, group, kind)
        self.q: deque = deque()
        self.depth = depth
        self.fill()

    def fill(self) -> None:
        while len(self.q) < self.depth and self.posted < self.total:
            self.q.append(_Recv(*self.args))
            self.posted += 1

    def take(self) -> _Recv:
        """Next receive (still in flight); the one after it is posted right away."""
        r = self.q.popleft()
        self.fill()
        return r


def _send(t: torch.Tensor, peer: int, group, kind: str) -> None:
    """Async send kept in flight until ``wait_sends`` (end of step)."""
    t = t.contiguous()
    _STATS["send_" + kind] += 1
    trace.record("pp.send_" + kind, t, peer=peer)
    works = dist.batch_isend_irecv([dist.P2POp(dist.isend, t, peer, group)])
    _INFLIGHT.append((works, [t]))


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

    def _mailboxes(self, num_micro: int):
        """(activation mailbox or None, gradient mailbox or None, forward-send channel,
        gradient-send channel) of this stage; every channel is its own 2-rank
        communicator (mesh.ProcessGroupManager._pp_channels)."""
        pg = mesh.pgm
        r = pg.pp_rank
        rf = None if self._first else _Mailbox(num_micro, self.tensor_shape, self.dtype, self.device,
                                               pg.pp_prev_rank, pg.pp_channel("fwd", r - 1), "forward")
        rb = None if self._last else _Mailbox(num_micro, self.tensor_shape, self.dtype, self.device,
                                              pg.pp_next_rank, pg.pp_channel("bwd", r), "backward")
        return rf, rb, pg.pp_channel("fwd", r), pg.pp_channel("bwd", r - 1)

    def train_step_afab(self, data_iter, num_micro: int) -> torch.Tensor:
        pg = mesh.pgm
        rf, rb, fwd_out, bwd_out = self._mailboxes(num_micro)
        ins, outs = deque(), deque()
        loss_sum = torch.zeros((), dtype=torch.float32, device=self.device)
        for _ in range(num_micro):
            x = rf.take().get().requires_grad_(True) if rf is not None else None
            batch = next(data_iter)
            y = self._forward(batch, x, num_micro)
            if not self._last:
                _send(y.detach(), pg.pp_next_rank, fwd_out, "forward")
            else:
                loss_sum += y.detach().float()
            ins.append(x)
            outs.append(y)
        for i in range(num_micro):
            dy = rb.take().get() if rb is not None else None
            x, y = ins.popleft(), outs.popleft()
            dx = self._backward(x, y, dy, last_backward=(i == num_micro - 1))
            if not self._first:
                _send(dx, pg.pp_prev_rank, bwd_out, "backward")
        wait_sends()
        return loss_sum

    def train_step_1f1b(self, data_iter, num_micro: int) -> torch.Tensor:
        """1F1B: warm-up forwards, steady one-forward-one-backward, cool-down backwards.
        The next micro-batch's activation and gradient receives are always in flight
        (``_Mailbox``), so each transfer overlaps the compute before its use."""
        pg = mesh.pgm
        warmup = min(pg.pp_world_size - pg.pp_rank - 1, num_micro)
        steady = num_micro - warmup
        rf, rb, fwd_out, bwd_out = self._mailboxes(num_micro)
        ins, outs = deque(), deque()
        loss_sum = torch.zeros((), dtype=torch.float32, device=self.device)
        n_bwd = 0

        def fwd():
            x = rf.take().get().requires_grad_(True) if rf is not None else None
            y = self._forward(next(data_iter), x, num_micro)
            if self._last:
                loss_sum.add_(y.detach().float())
            else:
                _send(y.detach(), pg.pp_next_rank, fwd_out, "forward")
            ins.append(x)
            outs.append(y)

        def bwd():
            nonlocal n_bwd
            dy = rb.take().get() if rb is not None else None
            xo, yo = ins.popleft(), outs.popleft()
            n_bwd += 1
            dx = self._backward(xo, yo, dy, last_backward=(n_bwd == num_micro))
            if not self._first:
                _send(dx, pg.pp_prev_rank, bwd_out, "backward")

        for _ in range(warmup):
            fwd()
        for _ in range(steady):
            fwd()
            bwd()
        for _ in range(warmup):
            bwd()
        wait_sends()
        return loss_sum

    # ------------------------------------------------------------------ interleaved 1F1B
    def train_step_interleaved(self, data_iter, num_micro: int) -> torch.Tensor:
        """Interleaved 1F1B over this rank's ``virtual_stages`` model chunks
        (parallel/interleaved.py has the schedule and its deadlock-free proof by
        simulation).  Activations and gradients travel on their own communicators
        (one FIFO per direction), receives are posted two ahead and waited right
        before use, sends stay in flight until the end of the step.  The DP gradient sync is enabled for the
        last micro-batch of each chunk, so every bucket fires during backward."""
        from .interleaved import Exchange, build_schedule, bwd_chunk, fwd_chunk, micro_batch

        pg = mesh.pgm
        P, r, V, M = pg.pp_world_size, pg.pp_rank, self.virtual_stages, num_micro
        ring = pg.pp_group_ids
        nxt, prv = ring[(r + 1) % P], ring[(r - 1) % P]
        # one 2-rank communicator per directed channel (mesh._pp_channels): every RCCL
        # stream carries ONE direction between ONE pair of ranks, so a receive posted
        # ahead only ever waits for its own sender (interleaved.simulate_streams)
        fwd_out, fwd_in = pg.pp_channel("fwd", r), pg.pp_channel("fwd", r - 1)
        bwd_out, bwd_in = pg.pp_channel("bwd", r - 1), pg.pp_channel("bwd", r)
        batches: list = []

        def batch(m):
            while len(batches) <= m:
                batches.append(next(data_iter))
            return batches[m]

        sched = build_schedule(P, V, M, r)
        # receives per direction, in schedule order (= the sender's order on that
        # direction's communicator): posted 2 ahead by the mailboxes, waited at use
        n_recv = {"fwd": 0, "bwd": 0}
        for a in sched:
            if isinstance(a, Exchange):
                for kind, _ in a.recv:
                    n_recv[kind] += 1
        box = {"fwd": _Mailbox(n_recv["fwd"], self.tensor_shape, self.dtype, self.device, prv, fwd_in, "forward"),
               "bwd": _Mailbox(n_recv["bwd"], self.tensor_shape, self.dtype, self.device, nxt, bwd_in,
                               "backward")}
        inputs, grads = {}, {}        # fwd step -> posted receive of its input; bwd step -> of its output grad
        acts = {}                     # (chunk, micro) -> (x, y)
        outs, dxs = {}, {}            # fwd step -> output to send; bwd step -> input grad to send
        loss_sum = torch.zeros((), dtype=torch.float32, device=self.device)
        for a in sched:
            if isinstance(a, Exchange):
                for kind, k in a.send:
                    if kind == "fwd":
                        _send(outs.pop(k), nxt, fwd_out, "forward")
                    else:
                        _send(dxs.pop(k), prv, bwd_out, "backward")
                for kind, k in a.recv:
                    (inputs if kind == "fwd" else grads)[k] = box[kind].take()
                continue
            kind, k = a
            if kind == "F":
                v, m = fwd_chunk(k, P, V), micro_batch(k, P, V)
                first, last = r == 0 and v == 0, r == P - 1 and v == V - 1
                x = None if first else inputs.pop(k).get().requires_grad_(True)
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
                    torch.autograd.backward(y, grads.pop(k).get())
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

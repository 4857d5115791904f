"""Loopback process group: ONE rank of a multi-GPU layout on one GPU ("per-rank compute slice").

``init_loopback(world, rank)`` starts torch.distributed with the in-process ``fake`` backend
(every collective returns at once, no peer exists) and gives every collective whose fake
form would leave its output unwritten a same-shape LOCAL COPY instead, so the rank runs its
real program -- the same kernels on the same per-rank shapes, at full model depth -- with the
communication replaced by device copies of the same size:

==========================  ===========================================================
collective                  loopback result on this rank
==========================  ===========================================================
all_reduce / broadcast      unchanged (the local contribution is the "sum")
all_gather(_into_tensor)    every slot = this rank's input (fake backend's own copy)
reduce_scatter(_tensor)     this rank's chunk of its own input
all_to_all(_single)         the output filled cyclically from this rank's input, so a
                            receive buffer of any split holds realistic values (EP: every
                            source sends what this rank sends, i.e. uniform routing)
isend / irecv (PP, CP ring) a receive takes the newest tensor this rank sent with the same
                            shape and dtype, or N(0, 0.02) data before the first send
==========================  ===========================================================

Nothing here is a measurement of communication: a slice prices the per-rank COMPUTE and
memory of a layout that cannot be run here (bench.py ``--slice``).
Reference layouts: scripts/benchmark_comprehensive.py:54-173.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

_STATE = {"on": False, "sent": {}}


class _Done:
    """Work handle of a loopback collective (already complete)."""

    def wait(self, timeout=None):
        return True

    def is_completed(self):
        return True

    def is_success(self):
        return True

    def get_future(self):
        fut = torch.futures.Future()
        fut.set_result(None)
        return fut


def active() -> bool:
    return _STATE["on"]


def _group_rank(group) -> int:
    return dist.get_rank(group) if group is not None else dist.get_rank()


def _fill_cyclic(out: torch.Tensor, src: torch.Tensor) -> None:
    o = out.view(-1)
    s = src.reshape(-1).to(out.dtype)
    if o.numel() == 0:
        return
    if s.numel() == 0:
        o.zero_()
        return
    if s.numel() >= o.numel():
        o.copy_(s[: o.numel()])
    else:
        o.copy_(s.repeat(math.ceil(o.numel() / s.numel()))[: o.numel()])


def _reduce_scatter_tensor(output, input, op=None, group=None, async_op=False):
    w = input.numel() // max(1, output.numel())
    r = _group_rank(group) % max(1, w)
    output.copy_(input.reshape(w, -1)[r].view_as(output))
    return _Done() if async_op else None


def _reduce_scatter(output, input_list, op=None, group=None, async_op=False):
    output.copy_(input_list[_group_rank(group) % len(input_list)])
    return _Done() if async_op else None


def _all_to_all_single(output, input, output_split_sizes=None, input_split_sizes=None, group=None, async_op=False):
    _fill_cyclic(output, input)
    return _Done() if async_op else None


def _all_to_all(output_tensor_list, input_tensor_list, group=None, async_op=False):
    n = len(input_tensor_list)
    for i, o in enumerate(output_tensor_list):
        _fill_cyclic(o, input_tensor_list[i % n])
    return _Done() if async_op else None


def _remember(t: torch.Tensor) -> None:
    _STATE["sent"][(tuple(t.shape), t.dtype, t.device)] = t.detach()


def _deliver(t: torch.Tensor) -> None:
    prev = _STATE["sent"].get((tuple(t.shape), t.dtype, t.device))
    if prev is not None:
        t.copy_(prev)
    elif t.is_floating_point():
        t.normal_(0.0, 0.02)
    else:
        t.zero_()


def _batch_isend_irecv(p2p_op_list):
    # P2POp accepts only torch's own isend / irecv, so those stay unpatched: point-to-point
    # traffic (PP stages, the CP ring) goes through batch_isend_irecv, handled here
    sends = [op for op in p2p_op_list if op.op is _REAL["isend"]]
    for op in sends:  # sends first: a batch that exchanges with itself sees its own data
        _remember(op.tensor)
    for op in p2p_op_list:
        if op.op is not _REAL["isend"]:
            _deliver(op.tensor)
    return [_Done()]


_REAL: dict = {}


def _broadcast_object_list(object_list, src=None, group=None, device=None, group_src=None):
    return None  # this process already holds every rank's objects


def _all_gather_object(object_list, obj, group=None):
    for i in range(len(object_list)):
        object_list[i] = obj


def init_loopback(world: int, rank: int) -> None:
    """Start the loopback default process group of ``world`` ranks as rank ``rank``."""
    from torch.testing._internal.distributed.fake_pg import FakeStore

    if not dist.is_initialized():
        dist.init_process_group("fake", rank=rank, world_size=world, store=FakeStore())
    if _STATE["on"]:
        return
    _STATE["on"] = True
    dist.reduce_scatter_tensor = _reduce_scatter_tensor
    dist.reduce_scatter = _reduce_scatter
    dist.all_to_all_single = _all_to_all_single
    dist.all_to_all = _all_to_all
    _REAL["isend"] = dist.isend
    dist.batch_isend_irecv = _batch_isend_irecv
    dist.broadcast_object_list = _broadcast_object_list
    dist.all_gather_object = _all_gather_object
    if hasattr(dist, "_reduce_scatter_base"):
        dist._reduce_scatter_base = _reduce_scatter_tensor

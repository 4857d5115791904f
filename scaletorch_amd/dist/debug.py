"""Collective-order race detection: cross-rank fingerprints of every collective.

A rank that issues collectives in a different order, on a different group, or
with a different shape / dtype than its peers does not fail on RCCL -- it
hangs (or silently reduces mismatched buffers).  With ``enable()`` every
``torch.distributed`` collective first publishes a fingerprint
``(op, shape, dtype)`` of its k-th call on its group to the c10d store and
compares it with the k-th fingerprint of every peer; a mismatch raises
``CollectiveMismatch`` naming both call sites instead of hanging.

SURVEY.md §5.2 (the reference has no race detection beyond bucket state-machine
asserts).  Store-based, so it needs no extra communicator and works for RCCL
and gloo groups alike; debug-only (two store round trips per collective).

    from scaletorch_amd.dist import debug
    debug.enable()          # or --debug_collectives
"""
from __future__ import annotations

import hashlib
import threading
import traceback
from collections import defaultdict

import torch
import torch.distributed as dist

_PATCHED: dict[str, object] = {}
_STATE = threading.local()  # re-entrancy flag (per thread)
_CHECKER = None  # process-wide: backward hooks run on autograd's device threads


class CollectiveMismatch(RuntimeError):
    pass


class _Checker:
    def __init__(self, timeout_s: float = 120.0):
        import datetime

        self.store = dist.distributed_c10d._get_default_store()
        self.store.set_timeout(datetime.timedelta(seconds=timeout_s))
        self.counters: dict[str, int] = defaultdict(int)
        self.rank = dist.get_rank()
        self.calls = 0

    def check(self, op: str, group, tensors, shape_sensitive: bool = True) -> None:
        if group is None or group is dist.GroupMember.WORLD:
            ranks = tuple(range(dist.get_world_size()))
        else:
            ranks = tuple(dist.get_process_group_ranks(group))
        if len(ranks) <= 1:
            return
        gid = hashlib.md5(repr(ranks).encode()).hexdigest()[:10]
        k = self.counters[gid]
        self.counters[gid] += 1
        self.calls += 1
        desc = []
        for t in tensors:
            if isinstance(t, torch.Tensor):
                desc.append(f"{tuple(t.shape) if shape_sensitive else '*'}:{str(t.dtype).replace('torch.', '')}")
        fp = f"{op}[{','.join(desc)}]"
        site = "".join(traceback.format_stack(limit=6)[:-3]).strip().splitlines()
        where = site[-2].strip() if len(site) >= 2 else "?"
        self.store.set(f"stcc/{gid}/{k}/{self.rank}", f"{fp}@@{where}")
        for r in ranks:
            if r == self.rank:
                continue
            other = self.store.get(f"stcc/{gid}/{k}/{r}").decode()
            ofp, _, owhere = other.partition("@@")
            if ofp != fp:
                raise CollectiveMismatch(
                    f"collective #{k} on group {ranks}: rank {self.rank} issued {fp} at {where}; "
                    f"rank {r} issued {ofp} at {owhere}")


def _wrap(name: str, tensor_args, shape_sensitive: bool, group_pos: int):
    orig = getattr(dist, name)

    def wrapper(*args, **kwargs):
        chk = _CHECKER
        if chk is not None and not getattr(_STATE, "inside", False):
            group = kwargs.get("group", args[group_pos] if group_pos < len(args) else None)
            tensors = [args[i] if i < len(args) else kwargs.get(n) for i, n in tensor_args]
            _STATE.inside = True  # collectives that call other collectives internally
            try:
                chk.check(name, group, tensors, shape_sensitive)
            finally:
                _STATE.inside = False
        return orig(*args, **kwargs)

    wrapper.__wrapped__ = orig
    return wrapper


# name -> ([(positional index, keyword)] of the tensors whose shape must agree,
#          shapes compared?, positional index of ``group``)
_COLLECTIVES = {
    "all_reduce": ([(0, "tensor")], True, 2),
    "all_gather_into_tensor": ([(0, "output_tensor"), (1, "input_tensor")], True, 2),
    "reduce_scatter_tensor": ([(0, "output"), (1, "input")], True, 3),
    "broadcast": ([(0, "tensor")], True, 2),
    "reduce": ([(0, "tensor")], True, 3),
    "all_to_all_single": ([(0, "output"), (1, "input")], False, 4),  # uneven splits are legal
    "all_gather": ([(1, "tensor")], True, 2),
    "barrier": ([], True, 0),
}


def enable(timeout_s: float = 120.0) -> None:
    """Install the checker on this rank (call on every rank, after init_process_group)."""
    global _CHECKER
    if not (dist.is_available() and dist.is_initialized()):
        return
    _CHECKER = _Checker(timeout_s)
    for name, (targs, sens, gpos) in _COLLECTIVES.items():
        if name not in _PATCHED and hasattr(dist, name):
            _PATCHED[name] = getattr(dist, name)
            setattr(dist, name, _wrap(name, targs, sens, gpos))


def disable() -> None:
    global _CHECKER
    for name, orig in _PATCHED.items():
        setattr(dist, name, orig)
    _PATCHED.clear()
    _CHECKER = None


def checked_calls() -> int:
    return _CHECKER.calls if _CHECKER else 0

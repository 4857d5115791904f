"""Per-call communication tracing (``VERBOSE=1`` or ``set_verbose(True)``).

Reference: under ``VERBOSE`` the reference logs every context-parallel and
pipeline send/recv (scaletorch/parallel/context_parallel/cp_comms.py:60-70,
scaletorch/parallel/pipeline_parallel/pp_comms.py:18-26) and counts PP ops
(pp_comms.py:273-285).  Here one hook covers every hot-path exchange -- PP p2p,
CP ring / all-gather / reduce-scatter, EP all-to-all, TP all-reduce -- with the
op, peer(s), shape, dtype and bytes; ``stats()`` keeps per-op call and byte
counters whether or not lines are printed (always on: a dict increment).
"""
from __future__ import annotations

import logging
import os
from collections import defaultdict

import torch

_log = logging.getLogger("scaletorch_amd.comm")
_VERBOSE = [os.environ.get("VERBOSE", "0") not in ("", "0", "false", "False")]
_STATS: dict = defaultdict(lambda: [0, 0])


def set_verbose(flag: bool) -> None:
    _VERBOSE[0] = bool(flag)


def verbose() -> bool:
    return _VERBOSE[0]


def record(op: str, tensor: torch.Tensor | None = None, peer=None, group_size: int | None = None, **extra) -> None:
    """Count one communication call (and log it when verbose)."""
    nbytes = tensor.numel() * tensor.element_size() if tensor is not None else 0
    s = _STATS[op]
    s[0] += 1
    s[1] += nbytes
    if extra.get("transport") == "xgmi":  # which transport really carried it (per call)
        x = _STATS[op + "@xgmi"]
        x[0] += 1
        x[1] += nbytes
    if _VERBOSE[0]:
        rank = os.environ.get("RANK", "0")
        shape = tuple(tensor.shape) if tensor is not None else ()
        dtype = str(tensor.dtype).replace("torch.", "") if tensor is not None else "-"
        parts = [f"[rank {rank}] {op}", f"shape={shape}", f"dtype={dtype}", f"bytes={nbytes}"]
        if peer is not None:
            parts.append(f"peer={peer}")
        if group_size is not None:
            parts.append(f"group={group_size}")
        parts += [f"{k}={v}" for k, v in extra.items()]
        _log.warning(" ".join(parts))


def stats() -> dict:
    """{op: {"calls": n, "bytes": b}} since the last ``reset()``."""
    return {k: {"calls": v[0], "bytes": v[1]} for k, v in _STATS.items()}


def reset() -> None:
    _STATS.clear()

"""roctx ranges + torch.profiler wiring (the reference has no
profiler/roctx integration at all).

``range(name)`` pushes a roctx range (``torch.cuda.nvtx`` is roctx on ROCm, so
the ranges show up in ``rocprofv3 --marker-trace`` / ``--kernel-trace``
timelines and in torch.profiler traces) only when profiling is enabled
(``set_enabled(True)``, ``--profile``, or ``ST_ROCTX=1``); otherwise it is a
zero-cost no-op so it can stay in the step code.
"""
from __future__ import annotations

import contextlib
import os

import torch

_ENABLED = os.environ.get("ST_ROCTX", "0") == "1"


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def enabled() -> bool:
    return _ENABLED


def _nvtx():
    if not torch.cuda.is_available():
        return None
    try:
        return torch.cuda.nvtx
    except Exception:  # pragma: no cover
        return None


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range
    nv = _nvtx() if _ENABLED else None
    if nv is None:
        yield
        return
    nv.range_push(name)
    try:
        yield
    finally:
        nv.range_pop()


def make_profiler(out_dir: str, wait: int = 1, warmup: int = 1, active: int = 3, rank: int = 0):
    """torch.profiler (ROCm: roctracer/rocprofiler backend) writing a chrome trace per rank."""
    from torch.profiler import ProfilerActivity, profile, schedule

    os.makedirs(out_dir, exist_ok=True)

    def _handler(p):
        p.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}_step{p.step_num}.json"))

    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    return profile(activities=acts, schedule=schedule(wait=wait, warmup=warmup, active=active),
                   on_trace_ready=_handler, record_shapes=False, with_stack=False)

"""LR schedulers with warm-up + a registry (reference: scaletorch/trainer/lr_scheduler.py:27-211).

``eta_min`` for cosine is a FACTOR of the base LR, as in the reference.
"""
from __future__ import annotations

import math
from typing import Callable

from torch.optim.lr_scheduler import LambdaLR

_REGISTRY: dict[str, Callable] = {}


def register_scheduler(name: str):
    def deco(fn):
        _REGISTRY[name] = fn
        return fn
    return deco


def available_schedulers() -> list[str]:
    return sorted(_REGISTRY)


def _warm(step: int, warmup: int) -> float | None:
    if warmup > 0 and step < warmup:
        return (step + 1) / warmup
    return None


@register_scheduler("constant")
def _constant(total: int, warmup: int, **_):
    return lambda s: _warm(s, warmup) or 1.0


@register_scheduler("linear")
def _linear(total: int, warmup: int, **_):
    def f(s):
        w = _warm(s, warmup)
        if w is not None:
            return w
        return max(0.0, (total - s) / max(1, total - warmup))
    return f


@register_scheduler("cosine")
def _cosine(total: int, warmup: int, T_max: int | None = None, eta_min: float = 0.0, **_):
    tmax = T_max or max(1, total - warmup)

    def f(s):
        w = _warm(s, warmup)
        if w is not None:
            return w
        p = min(1.0, (s - warmup) / tmax)
        return eta_min + (1 - eta_min) * 0.5 * (1 + math.cos(math.pi * p))
    return f


@register_scheduler("polynomial")
def _poly(total: int, warmup: int, power: float = 1.0, **_):
    def f(s):
        w = _warm(s, warmup)
        if w is not None:
            return w
        return max(0.0, 1 - (s - warmup) / max(1, total - warmup)) ** power
    return f


@register_scheduler("step")
def _step(total: int, warmup: int, step_size: int = 1, gamma: float = 0.1, **_):
    def f(s):
        w = _warm(s, warmup)
        if w is not None:
            return w
        return gamma ** ((s - warmup) // step_size)
    return f


@register_scheduler("onecycle")
def _onecycle(total: int, warmup: int, pct_start: float = 0.3, max_lr_factor: float = 1.0, **_):
    up = max(1, int(total * pct_start))
    start, end = 1 / 25.0, 1 / 1e4

    def f(s):
        if s < up:
            p = s / up
            return max_lr_factor * (start + (1 - start) * (1 - math.cos(math.pi * p)) / 2)
        p = min(1.0, (s - up) / max(1, total - up))
        return max_lr_factor * (end + (1 - end) * (1 + math.cos(math.pi * p)) / 2)
    return f


def create_lr_scheduler(optimizer, lr_scheduler_type: str = "linear", total_steps: int = 1000, warmup_steps: int = 0,
                        T_max: int | None = None, eta_min: float = 0.0, power: float = 1.0, step_size: int = 1,
                        gamma: float = 0.1, max_lr: float | None = None, pct_start: float = 0.3) -> LambdaLR:
    if lr_scheduler_type not in _REGISTRY:
        raise ValueError(f"unknown scheduler {lr_scheduler_type!r}; available: {available_schedulers()}")
    base = optimizer.param_groups[0]["lr"]
    fn = _REGISTRY[lr_scheduler_type](total=total_steps, warmup=warmup_steps, T_max=T_max, eta_min=eta_min,
                                      power=power, step_size=step_size, gamma=gamma, pct_start=pct_start,
                                      max_lr_factor=(max_lr / base) if max_lr else 1.0)
    return LambdaLR(optimizer, fn)

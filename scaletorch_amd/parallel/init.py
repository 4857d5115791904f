"""Parallelism-invariant weight initialisation.

Every parameter is initialised from a generator seeded by (global seed,
parameter's GLOBAL module name): the FULL tensor is generated and this rank
keeps its TP / EP shard.  Hence a TP2 x PP2 model starts from exactly the
weights of the single-GPU model with the same seed (the property the parity
tests check), which the reference did not have (per-shard RNG draws).
"""
from __future__ import annotations

import math
import zlib

import torch

_SEED = 1234


def set_init_seed(seed: int) -> None:
    global _SEED
    _SEED = int(seed)


def keyed_generator(key: str | None, device) -> torch.Generator | None:
    if key is None:
        return None
    dev = torch.device(device)
    g = torch.Generator(device=dev if dev.type == "cuda" else "cpu")
    g.manual_seed((_SEED * 1_000_003 + zlib.crc32(key.encode())) & ((1 << 62) - 1))
    return g


def init_full(shape, init: str, std: float, fan_in: int, key: str | None, device) -> torch.Tensor:
    """Full (unsharded) fp32 init tensor: 'normal' N(0, std) or 'uniform' U(+-1/sqrt(fan_in))."""
    g = keyed_generator(key, device)
    t = torch.empty(shape, dtype=torch.float32, device=device)
    if init == "normal":
        t.normal_(0.0, std, generator=g)
    else:
        b = 1.0 / math.sqrt(fan_in)
        t.uniform_(-b, b, generator=g)
    return t


def assign_init_keys(model: torch.nn.Module) -> None:
    for name, m in model.named_modules():
        m._st_init_key = name or "root"

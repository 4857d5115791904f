"""Device probing + peak-FLOPS registry (reference: scaletorch/utils/device.py:24-298).

MI355X (gfx950) dense bf16 peak ~2.5 PFLOP/s (AMD spec quotes ~5 PF *with*
2:1 sparsity; MFU is always priced against the dense figure).  Override with
``SCALETORCH_DEVICE_FLOPS`` (FLOP/s).
"""
from __future__ import annotations

import os

import torch

# dense bf16 FLOP/s
PEAK_FLOPS = {
    "mi355x": 2.5e15,
    "gfx950": 2.5e15,
    "mi350x": 2.3e15,
    "mi325x": 1.307e15,
    "mi300x": 1.307e15,
    "gfx942": 1.307e15,
    "h100": 989e12,
    "h200": 989e12,
    "a100": 312e12,
    "910b": 320e12,
    "cpu": 1e12,
}


def get_device_type() -> str:
    return "cuda" if torch.cuda.is_available() else "cpu"


def device_name() -> str:
    if not torch.cuda.is_available():
        return "cpu"
    try:
        props = torch.cuda.get_device_properties(0)
        arch = getattr(props, "gcnArchName", "") or ""
        return f"{props.name} {arch}".strip()
    except Exception:
        return "cuda"


def get_theoretical_flops(name: str | None = None) -> float:
    env = os.environ.get("SCALETORCH_DEVICE_FLOPS")
    if env:
        return float(env)
    n = (name or device_name()).lower()
    for k, v in PEAK_FLOPS.items():
        if k in n:
            return v
    if "instinct" in n or "amd" in n:
        return PEAK_FLOPS["mi355x"]
    return PEAK_FLOPS["cpu"]


def memory_reserved() -> float:
    return torch.cuda.memory_reserved() if torch.cuda.is_available() else 0.0


def memory_stats() -> dict:
    if not torch.cuda.is_available():
        return {}
    return {
        "allocated_gb": torch.cuda.memory_allocated() / 1e9,
        "reserved_gb": torch.cuda.memory_reserved() / 1e9,
        "peak_gb": torch.cuda.max_memory_allocated() / 1e9,
    }

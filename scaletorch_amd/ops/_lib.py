"""Loader for the in-tree HIP kernel library (``scaletorch_amd/_st_kernels.so``).

Policy: on a GPU the hand-written gfx950 kernels are THE
implementation -- if the library is missing or fails to load while a GPU
tensor reaches an op, the op raises instead of silently falling back to a
PyTorch composite.  The pure-PyTorch reference implementations in this
package are used only for CPU tensors (unit tests, gloo runs) or when the user
explicitly opts out with ``ST_DISABLE_NATIVE=1`` (debugging / A-B numerics).
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

# ST_KERNEL_LIB: load an alternative build (kernel A/B experiments, tools/bench_kernels.py)
_LIB_PATH = Path(os.environ.get("ST_KERNEL_LIB") or Path(__file__).resolve().parent.parent / "_st_kernels.so")
_lock = threading.Lock()
_loaded: bool | None = None
_load_error: str | None = None


def lib_path() -> Path:
    return _LIB_PATH


def load() -> bool:
    """Load the kernel library once; returns True on success."""
    global _loaded, _load_error
    if _loaded is not None:
        return _loaded
    with _lock:
        if _loaded is not None:
            return _loaded
        if not _LIB_PATH.exists():
            _load_error = f"{_LIB_PATH} not built (run `python -m scaletorch_amd._build`)"
            _loaded = False
            return False
        try:
            torch.ops.load_library(str(_LIB_PATH))
            _loaded = True
        except Exception as e:  # pragma: no cover - depends on environment
            _load_error = f"failed to load {_LIB_PATH}: {e}"
            _loaded = False
        return _loaded


def native_disabled() -> bool:
    return os.environ.get("ST_DISABLE_NATIVE", "0") == "1"


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` must go through the HIP kernels; raises if they are unavailable."""
    if t.device.type != "cuda" or native_disabled():
        return False
    if not load():
        raise RuntimeError(
            "scaletorch_amd: GPU tensor reached a fused op but the HIP kernel library is "
            f"unavailable ({_load_error}). Build it with `python -m scaletorch_amd._build` "
            "or set ST_DISABLE_NATIVE=1 to run the PyTorch reference path explicitly."
        )
    return True


def ops():
    load()
    return torch.ops.st_amd


def load_error() -> str | None:
    return _load_error


def is_probe_build() -> bool:
    """True when the loaded kernel library is the diagnostic build (``_build.py --probes``)."""
    return _LIB_PATH.stem == "probes" and _LIB_PATH.parent.name == "variants"


def probe_env(name: str) -> str | None:
    """Value of a timing-probe switch (``ST_*_PROBE*``: skips or fakes work, so the results are
    WRONG), or None when unset / "0".  Honoured only with the diagnostic library loaded; set on a
    production build it raises, so a stray variable can never corrupt a training run."""
    v = os.environ.get(name)
    if not v or v == "0":
        return None
    if not is_probe_build():
        raise RuntimeError(f"{name}={v} selects a timing probe with WRONG results; it runs only with the "
                           "diagnostic kernel library (python -m scaletorch_amd._build --probes; "
                           "ST_KERNEL_LIB=build/variants/probes.so)")
    return v

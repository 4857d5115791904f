"""Offline-tuned hipBLASLt / rocBLAS solutions for the library GEMMs (PyTorch TunableOp).

The plain library GEMMs of a step (forward projections, the TN data gradients on the
W^T copies, the fused LM head chunks) go through ``at::cuda::blas`` -> hipBLASLt with
its first heuristic solution.  TunableOp times every hipBLASLt and rocBLAS solution
for a GEMM signature once and records the fastest in a CSV keyed by (op, transposes,
M, N, K, dtype), validated against the PyTorch / ROCm / hipBLASLt versions and the GPU
architecture.  The table for the MI355X shapes this repository runs is committed
(``scaletorch_amd/tuning/gemm_gfx950.csv``) and produced by

    python bench.py --gemm_tuning tune --steps 1 --warmup 2 [--layout ...]

(each run ADDS the signatures it meets to the table).  Modes:

* ``auto`` (default): ``use`` on a gfx950 GPU when the committed table exists, else ``off``;
* ``use``: look solutions up in the table, never tune (a signature missing from it runs
  the default heuristic, unchanged);
* ``tune``: time every solution of each new signature during the run and write the table;
* ``off``: TunableOp disabled.

The reference has no counterpart (its GEMMs are whatever torch picks on CUDA / NPU).
"""
from __future__ import annotations

import os

import torch

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "gemm_gfx950.csv")
_STATE = {"mode": "off", "file": None}


def _gfx950() -> bool:
    try:
        return "gfx950" in torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
    except Exception:  # noqa: BLE001 - no GPU / no property
        return False


def configure(mode: str = "auto", path: str | None = None, max_tuning_ms: int = 30) -> str:
    """Set TunableOp up for this process; returns the effective mode."""
    path = path or os.environ.get("ST_GEMM_TUNING_FILE") or TABLE
    if mode not in ("auto", "use", "tune", "off"):
        raise ValueError(f"gemm_tuning must be auto | use | tune | off, got {mode!r}")
    if not torch.cuda.is_available():  # nothing to tune (and torch.cuda.tunable needs a device)
        _STATE.update(mode="off", file=None)
        return "off"
    if mode == "auto":
        mode = "use" if (os.path.exists(path) and _gfx950()) else "off"
    if mode == "use" and not os.path.exists(path):
        raise FileNotFoundError(f"gemm_tuning=use but {path} does not exist (run with --gemm_tuning tune first)")
    tun = torch.cuda.tunable
    if mode == "off":
        if tun.is_enabled():
            tun.enable(False)
        _STATE.update(mode="off", file=None)
        return mode
    tun.set_filename(path, False)
    tun.enable(True)
    tun.tuning_enable(mode == "tune")
    if mode == "tune":
        tun.set_max_tuning_duration(max_tuning_ms)
        os.makedirs(os.path.dirname(path), exist_ok=True)
    if os.path.exists(path):
        try:
            ok = tun.read_file(path)
        except Exception:  # noqa: BLE001 -- a table from another stack must never stop training
            ok = False
        if ok is False and mode == "use":
            # validators (PyTorch / ROCm / hipBLASLt versions, GPU arch) did not match: run the
            # library's default heuristics rather than half-applied or mismatched solutions
            tun.enable(False)
            _STATE.update(mode="off", file=None)
            return "off"
    _STATE.update(mode=mode, file=path)
    return mode


def finish() -> None:
    """Write the table after a tuning run (no-op otherwise).  PyTorch builds without
    ``torch.cuda.tunable.write_file`` write it when the process exits."""
    if _STATE["mode"] == "tune" and hasattr(torch.cuda.tunable, "write_file"):
        torch.cuda.tunable.write_file(_STATE["file"])


def state() -> dict:
    return {"mode": _STATE["mode"], "entries": len(torch.cuda.tunable.get_results()) if _STATE["mode"] != "off" else 0}

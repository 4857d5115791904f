"""Environment-variable names and a system-info dump.

Reference: scaletorch/env.py:7-29 (FLASH_ATTEN, CONTEXT_PARALLEL,
SEQUENCE_PARALLEL, VERBOSE, DTYPE, RANK, ...) and the deprecated
scaletorch/utils/env_utils.py:22-131 (``init_dist_pytorch`` / ``cleanup_dist``
shims, ``get_system_info``).  In this framework the reference's behaviour
toggles are CLI flags (trainer/config.py); the names below are the launcher /
runtime variables it reads, plus the ST_* tuning and debugging switches.
"""
from __future__ import annotations

import os
import platform
import socket

# launcher / rendezvous
RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE = "RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE"
MASTER_ADDR, MASTER_PORT = "MASTER_ADDR", "MASTER_PORT"
# reference behaviour toggles (accepted for compatibility; the CLI flags win)
FLASH_ATTEN, CONTEXT_PARALLEL, SEQUENCE_PARALLEL, VERBOSE, DTYPE = (
    "FLASH_ATTEN", "CONTEXT_PARALLEL", "SEQUENCE_PARALLEL", "VERBOSE", "DTYPE")
# this framework's switches
ST_DISABLE_NATIVE = "ST_DISABLE_NATIVE"   # 1: PyTorch reference ops instead of the HIP kernels (A/B numerics)
ST_KERNEL_LIB = "ST_KERNEL_LIB"           # path of an alternative kernel-library build (A/B)
ST_OVERLAP_OPT = "ST_OVERLAP_OPT"         # 0: optimizer step serial after backward
ST_WGRAD_KERNEL = "ST_WGRAD_KERNEL"       # 0: hipBLASLt for every weight-gradient GEMM
ST_WGRAD_TUNE = "ST_WGRAD_TUNE"           # 0: no per-shape HIP-vs-hipBLASLt timing
ST_WGRAD_FP32_GEMM = "ST_WGRAD_FP32_GEMM"  # 0: bf16 wgrad GEMM + separate fp32 add
ST_MOE_GROUPED_GEMM = "ST_MOE_GROUPED_GEMM"  # 0: per-expert GEMM loop
ST_ADAMW_BLOCKS = "ST_ADAMW_BLOCKS"       # cap the AdamW grid (overlap experiments)
ST_FAULT_STEP, ST_FAULT_RANK = "ST_FAULT_STEP", "ST_FAULT_RANK"  # fault injection (tools/train.py)
# RCCL / HIP
HSA_ENABLE_IPC_MODE_LEGACY = "HSA_ENABLE_IPC_MODE_LEGACY"  # must be 0 on dmabuf-only hosts
TORCH_NCCL_ASYNC_ERROR_HANDLING = "TORCH_NCCL_ASYNC_ERROR_HANDLING"


def env_flag(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    return default if v is None else v.strip().lower() in ("1", "true", "yes", "on")


def get_system_info() -> dict:
    """Host / ROCm / torch / GPU facts for run logs (no GPU initialisation needed)."""
    import torch

    info = {
        "hostname": socket.gethostname(), "platform": platform.platform(), "python": platform.python_version(),
        "torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
        "cpu_count": os.cpu_count(), "gpu_count": torch.cuda.device_count(),
        "rank": os.environ.get(RANK), "world_size": os.environ.get(WORLD_SIZE),
    }
    try:
        import torch.distributed as dist

        info["nccl_available"] = dist.is_nccl_available()
        info["gloo_available"] = dist.is_gloo_available()
    except Exception:  # pragma: no cover
        pass
    return info


def init_dist_pytorch(backend: str | None = None, **kw):
    """Deprecated reference shim (env_utils.init_dist_pytorch) -> dist.init_dist."""
    from .dist import init_dist

    return init_dist("pytorch", backend=backend, **kw)


def cleanup_dist() -> None:
    """Deprecated reference shim (env_utils.cleanup_dist)."""
    from .dist import cleanup_dist as _c

    _c()

"""Process-group initialisation for torchrun / SLURM / MPI launches.

Reference: ``init_dist`` and friends in scaletorch/dist/utils.py:67-276 and
``initialize_distributed_training`` in scaletorch/trainer/dist_setup.py:64-124.
On MI355X the device backend is ``nccl`` (= RCCL over xGMI); CPU runs use gloo.
RCCL-over-xGMI defaults are exported before the first communicator is created
(users' own env always wins).
"""
from __future__ import annotations

import datetime
import os
import re
import subprocess

import torch
import torch.distributed as dist

DEFAULT_TIMEOUT_S = 600

# Env for RCCL on a single 8x MI355X xGMI node.  setdefault only: anything the
# user exports wins.  HSA_ENABLE_IPC_MODE_LEGACY=0 is required on this fleet
# (dmabuf IPC only).
_RCCL_ENV = {
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
    "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1",
    "TORCH_NCCL_HIGH_PRIORITY": "1",  # comm kernels on a high-priority stream (overlap with compute)
}


def infer_launcher() -> str:
    if "WORLD_SIZE" in os.environ and "RANK" in os.environ:
        return "pytorch"
    if "SLURM_NTASKS" in os.environ:
        return "slurm"
    if "OMPI_COMM_WORLD_SIZE" in os.environ or "PMI_SIZE" in os.environ:
        return "mpi"
    return "none"


def device_backend(use_cpu: bool = False) -> str:
    if use_cpu or not torch.cuda.is_available():
        return "gloo"
    return "nccl"


def _apply_rccl_env() -> None:
    for k, v in _RCCL_ENV.items():
        os.environ.setdefault(k, v)


def _slurm_env(port: int | None) -> None:
    os.environ.setdefault("RANK", os.environ["SLURM_PROCID"])
    os.environ.setdefault("WORLD_SIZE", os.environ["SLURM_NTASKS"])
    os.environ.setdefault("LOCAL_RANK", os.environ.get("SLURM_LOCALID", "0"))
    if "MASTER_ADDR" not in os.environ:
        nodelist = os.environ.get("SLURM_NODELIST", "127.0.0.1")
        try:
            addr = subprocess.getoutput(f"scontrol show hostname {nodelist} | head -n1").strip()
        except Exception:
            addr = ""
        if not addr:
            addr = parse_slurm_nodelist(nodelist)[0]
        os.environ["MASTER_ADDR"] = addr
    os.environ.setdefault("MASTER_PORT", str(port or 29500))


def parse_slurm_nodelist(nodelist: str) -> list[str]:
    """Expand a SLURM nodelist like ``node[01-03,07],gpu5`` (reference: scaletorch/dist/utils.py:206-251)."""
    out = []
    for part in re.findall(r"[^,\[]+(?:\[[^\]]*\])?", nodelist):
        m = re.match(r"(.*)\[(.*)\]$", part)
        if not m:
            out.append(part)
            continue
        prefix, body = m.groups()
        for rng in body.split(","):
            if "-" in rng:
                a, b = rng.split("-")
                width = len(a)
                out.extend(f"{prefix}{i:0{width}d}" for i in range(int(a), int(b) + 1))
            else:
                out.append(prefix + rng)
    return out


def _mpi_env(port: int | None) -> None:
    os.environ.setdefault("RANK", os.environ.get("OMPI_COMM_WORLD_RANK", os.environ.get("PMI_RANK", "0")))
    os.environ.setdefault("WORLD_SIZE", os.environ.get("OMPI_COMM_WORLD_SIZE", os.environ.get("PMI_SIZE", "1")))
    os.environ.setdefault("LOCAL_RANK", os.environ.get("OMPI_COMM_WORLD_LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(port or 29500))


def init_dist(launcher: str | None = None, backend: str | None = None, use_cpu: bool = False,
              timeout_s: int = DEFAULT_TIMEOUT_S, port: int | None = None) -> tuple[int, int, int]:
    """Initialise the default process group; returns (rank, local_rank, world_size).

    A single process with no launcher env runs with world size 1 and NO
    process group (like the reference, parallel modules then see ``pgm`` unset).
    """
    if backend == "loopback":
        # one rank of a layout on one device (bench.py --slice): world / rank of the rank to
        # impersonate come from ST_LOOPBACK_WORLD / ST_LOOPBACK_RANK, collectives are local copies
        from .loopback import init_loopback

        world = int(os.environ.get("ST_LOOPBACK_WORLD", "1"))
        rank = int(os.environ.get("ST_LOOPBACK_RANK", "0"))
        if torch.cuda.is_available() and not use_cpu:
            torch.cuda.set_device(0)
        init_loopback(world, rank)
        return rank, 0, world
    launcher = launcher or infer_launcher()
    if launcher == "slurm":
        _slurm_env(port)
    elif launcher == "mpi":
        _mpi_env(port)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    backend = backend or device_backend(use_cpu)
    if backend == "hccl":  # reference-compat flag: HCCL does not exist here
        backend = device_backend(use_cpu)
    if backend == "nccl" and not torch.cuda.is_available():
        backend = "gloo"
    # ST_GPU_OVERSUBSCRIBE=1 (tests only): several ranks share the visible GPUs
    gpu = local_rank
    if os.environ.get("ST_GPU_OVERSUBSCRIBE", "0") == "1" and torch.cuda.is_available():
        gpu = local_rank % max(1, torch.cuda.device_count())
    if backend == "nccl":
        _apply_rccl_env()
        torch.cuda.set_device(gpu)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, init_method="env://", world_size=world, rank=rank,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", gpu)
        attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        if attempt > 0:
            # torchrun restart: the agent's store still holds the previous attempt's
            # rendezvous keys (peer addresses of dead ranks) -> namespace this attempt
            store, _, _ = next(dist.rendezvous("env://", rank=rank, world_size=world, timeout=kw["timeout"]))
            kw.pop("init_method")
            kw["store"] = dist.PrefixStore(f"/scaletorch_amd/attempt_{attempt}/", store)
        dist.init_process_group(**kw)
    return rank, local_rank, world


def cleanup_dist() -> None:
    if dist.is_available() and dist.is_initialized():
        try:
            dist.barrier()
        except Exception:
            pass
        dist.destroy_process_group()


def get_comm_device(group=None) -> torch.device:
    """Device on which tensors must live for ``group``'s backend."""
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")

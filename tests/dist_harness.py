"""Multi-process CPU/gloo harness: run ``fn(rank, world, *args)`` in ``world``
spawned processes on 127.0.0.1 and collect their return values."""
from __future__ import annotations

import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    import torch

    torch.set_num_threads(1)
    try:
        import io

        buf = io.BytesIO()
        torch.save(fn(rank, world, *args), buf)  # plain bytes: no shared-memory tensor handles
        q.put((rank, "ok", buf.getvalue()))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


def run_workers(fn, world: int, *args, timeout: float = 240.0) -> list:
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, val = q.get(timeout=timeout)
            if status == "err":
                raise RuntimeError(f"rank {rank} failed:\n{val}")
            import io

            import torch

            results[rank] = torch.load(io.BytesIO(val), weights_only=True)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]

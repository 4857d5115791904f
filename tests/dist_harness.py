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
    # the free port is only reserved until _free_port returns: under pytest -n another
    # worker's rendezvous can take it first (EADDRINUSE) -> retry on a fresh port
    for attempt in range(3):
        try:
            return _run_once(fn, world, args, timeout)
        except RuntimeError as e:
            if "EADDRINUSE" not in str(e) or attempt == 2:
                raise
    raise AssertionError("unreachable")


def _run_once(fn, world: int, args, timeout: float) -> list:
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results, errors = {}, {}
    try:
        import io
        import queue

        import torch

        for _ in range(world):
            try:
                rank, status, val = q.get(timeout=timeout if not errors else 20)
            except queue.Empty:
                if errors:
                    break
                raise
            if status == "err":
                errors[rank] = val
                continue
            results[rank] = torch.load(io.BytesIO(val), weights_only=True)
        if errors:
            # the root cause first: peers of a failed rank only see "Connection reset"
            first = sorted(errors, key=lambda r: ("Connection reset" in errors[r] or "Connection closed" in errors[r], r))
            dead = [r for r, p in enumerate(procs) if p.exitcode not in (None, 0)]
            raise RuntimeError(f"rank {first[0]} failed (errors from ranks {sorted(errors)}, "
                               f"abnormal exits {dead}):\n{errors[first[0]]}")
        missing = [r for r in range(world) if r not in results]
        if missing:
            codes = {r: procs[r].exitcode for r in missing}
            raise RuntimeError(f"ranks {missing} returned nothing (exit codes {codes})")
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]


def stage_gloo_cuda_p2p() -> None:
    """Test-only alias of scaletorch_amd.dist.gloo_staging.stage_gloo_cuda_p2p."""
    from scaletorch_amd.dist.gloo_staging import stage_gloo_cuda_p2p as _stage

    _stage()

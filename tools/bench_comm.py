#!/usr/bin/env python3
"""Collective bandwidth microbenchmark (RCCL over xGMI, or gloo on CPU).

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_comm.py \
      [--sizes 1M,16M,256M,1G] [--ops all_reduce,reduce_scatter,...] [--dtype bf16]

For every op and message size prints one JSON line with the time, the
algorithm bandwidth (bytes / time) and the bus bandwidth with the nccl-tests
conventions (all_reduce 2(n-1)/n, reduce_scatter / all_gather / all_to_all
(n-1)/n, broadcast and sendrecv 1), i.e. the per-link number to compare with
xGMI's ~50 GB/s/direction/link when choosing DP bucket sizes and TP/EP degree
(SURVEY.md §5.1 "comm-bandwidth microbenchmark").  Size = bytes of the full
(gathered / unsharded) buffer.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.realpath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

_FACT = {"all_reduce": lambda n: 2 * (n - 1) / n, "reduce_scatter": lambda n: (n - 1) / n,
         "all_gather": lambda n: (n - 1) / n, "all_to_all": lambda n: (n - 1) / n,
         "broadcast": lambda n: 1.0, "sendrecv": lambda n: 1.0}


def _parse_size(s: str) -> int:
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(float(s[:-1]) * mult[s[-1]]) if s[-1] in mult else int(s)


def run(argv=None) -> list[dict]:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1M,16M,128M,512M")
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather,all_to_all,broadcast,sendrecv")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--backend", default="nccl")
    args = ap.parse_args(argv)
    if not dist.is_initialized():
        from scaletorch_amd.dist.launch import init_dist

        init_dist(backend=args.backend, use_cpu=args.backend == "gloo")
    n, rank = dist.get_world_size(), dist.get_rank()
    gpu = args.backend == "nccl" and torch.cuda.is_available()
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}[args.dtype]
    if not gpu and dtype != torch.float32:
        dtype = torch.float32  # gloo reduces fp32
    esize = torch.tensor([], dtype=dtype).element_size()

    def sync():
        if gpu:
            torch.cuda.synchronize()

    rows = []
    for op in args.ops.split(","):
        for s in args.sizes.split(","):
            nbytes = _parse_size(s)
            numel = max(n, nbytes // esize // n * n)
            full = torch.ones(numel, dtype=dtype, device=dev)
            shard = torch.empty(numel // n, dtype=dtype, device=dev)
            out = torch.empty_like(full)
            peer_next, peer_prev = (rank + 1) % n, (rank - 1) % n

            def once():
                if op == "all_reduce":
                    dist.all_reduce(full)
                elif op == "reduce_scatter":
                    dist.reduce_scatter_tensor(shard, full)
                elif op == "all_gather":
                    dist.all_gather_into_tensor(out, shard)
                elif op == "all_to_all":
                    dist.all_to_all_single(out, full)
                elif op == "broadcast":
                    dist.broadcast(full, src=0)
                elif op == "sendrecv":
                    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, full, peer_next),
                                                   dist.P2POp(dist.irecv, out, peer_prev)])
                    for r in reqs:
                        r.wait()
                else:
                    raise ValueError(op)

            for _ in range(args.warmup):
                once()
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                once()
            sync()
            dt = (time.perf_counter() - t0) / args.iters
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
            size = numel * esize
            algbw = size / dt / 1e9
            rows.append({"op": op, "bytes": size, "n": n, "time_us": round(dt * 1e6, 2),
                         "algbw_GBps": round(algbw, 2), "busbw_GBps": round(algbw * _FACT[op](n), 2),
                         "dtype": str(dtype).replace("torch.", ""), "backend": dist.get_backend()})
            if rank == 0 and __name__ == "__main__":
                print(json.dumps(rows[-1]), flush=True)
            del full, shard, out
    return rows


if __name__ == "__main__":
    run()
    if dist.is_initialized():
        dist.destroy_process_group()

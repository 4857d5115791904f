#!/usr/bin/env python3
"""Collective smoke tests of ``scaletorch_amd.dist`` under a real launcher.

Reference: scripts/torch_dist/run_dist_test.py (14 assert-based collective tests
via scaletorch.dist under torchrun + nccl; its import of ``get_current_device``
is broken there).  Here every wrapper of dist/collectives.py is exercised with
exact integer-valued data, on RCCL (``--backend nccl``, one GPU per rank) or gloo
(``--backend gloo``, CPU; what tests/test_dist_smoke.py runs):

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 scripts/run_dist_test.py --backend nccl
  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 scripts/run_dist_test.py --backend gloo

Rank 0 prints one line per test and a final ``ALL N PASSED`` (exit 0) or the
failures (exit 1).  Every rank runs every test (collectives must match).
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from scaletorch_amd import dist as D  # noqa: E402


def _dev(backend: str) -> torch.device:
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def collective_cases(dev: torch.device):
    r, w = D.get_rank(), D.get_world_size()

    def t_all_reduce_sum():
        t = torch.full((5,), float(r + 1), device=dev)
        D.all_reduce(t, "sum")
        assert torch.all(t == w * (w + 1) / 2), t

    def t_all_reduce_mean_max_min():
        t = torch.full((3,), float(r), device=dev)
        D.all_reduce(t, "mean")
        assert torch.allclose(t, torch.full_like(t, (w - 1) / 2)), t
        t = torch.full((3,), float(r), device=dev)
        D.all_reduce(t, "max")
        assert torch.all(t == w - 1)
        t = torch.full((3,), float(r), device=dev)
        D.all_reduce(t, "min")
        assert torch.all(t == 0)

    def t_all_reduce_async():
        t = torch.full((4,), 2.0, device=dev)
        h = D.all_reduce(t, "sum", async_op=True)
        if h is not None:
            h.wait()
        assert torch.all(t == 2.0 * w)

    def t_broadcast():
        t = torch.arange(6, dtype=torch.float32, device=dev) if r == 0 else torch.zeros(6, device=dev)
        D.broadcast(t, src=0)
        assert torch.equal(t, torch.arange(6, dtype=torch.float32, device=dev))

    def t_all_gather():
        t = torch.full((2, 3), float(r), device=dev)
        out = D.all_gather(t, dim=0)
        assert out.shape == (2 * w, 3) and all(torch.all(out[2 * i: 2 * i + 2] == i) for i in range(w))
        lst = D.all_gather(t, as_list=True)
        assert len(lst) == w and all(torch.all(x == i) for i, x in enumerate(lst))

    def t_reduce_scatter():
        t = torch.arange(2 * w, dtype=torch.float32, device=dev)
        out = D.reduce_scatter(t, "sum", dim=0)
        assert torch.equal(out, torch.arange(2 * r, 2 * r + 2, dtype=torch.float32, device=dev) * w), out

    def t_reduce():
        t = torch.full((3,), float(r + 1), device=dev)
        D.reduce(t, dst=0, op="sum")
        if r == 0:
            assert torch.all(t == w * (w + 1) / 2)

    def t_scatter():
        data = [torch.full((4,), float(i), device=dev) for i in range(w)] if r == 0 else None
        out = torch.empty(4, device=dev)
        D.scatter(data, out, src=0)
        assert torch.all(out == r)

    def t_gather():
        got = D.gather(torch.full((2,), float(r), device=dev), dst=0)
        if r == 0:
            assert [int(x[0]) for x in got] == list(range(w))

    def t_all_to_all():
        t = torch.tensor([r * 100 + j for j in range(w)], dtype=torch.float32, device=dev)
        out = D.all_to_all(t)
        assert torch.equal(out, torch.tensor([j * 100 + r for j in range(w)], dtype=torch.float32, device=dev)), out

    def t_p2p_ring():
        nxt, prv = (r + 1) % w, (r - 1) % w
        send = torch.full((3,), float(r), device=dev)
        recv = torch.empty(3, device=dev)
        ops = [D.P2POp(dist.isend, send, nxt), D.P2POp(dist.irecv, recv, prv)]
        for req in D.batch_isend_irecv(ops):
            req.wait()
        assert torch.all(recv == prv)

    def t_object_collectives():
        objs = [{"rank": 0, "msg": "hello"}] if r == 0 else [None]
        D.broadcast_object_list(objs, src=0)
        assert objs[0] == {"rank": 0, "msg": "hello"}
        allv = D.all_gather_object({"r": r})
        assert [o["r"] for o in allv] == list(range(w))
        g = D.gather_object(r * 10, dst=0)
        if r == 0:
            assert g == [i * 10 for i in range(w)]

    def t_all_reduce_dict():
        d = {"a": torch.full((2,), float(r), device=dev), "b": torch.ones(3, device=dev)}
        out = D.all_reduce_dict(d, "sum")
        assert torch.all(out["a"] == w * (w - 1) / 2) and torch.all(out["b"] == w)

    def t_sync_random_seed_and_collect():
        s = D.sync_random_seed(device=dev)
        allv = D.all_gather_object(s)
        assert len(set(allv)) == 1
        part = [r * 10 + i for i in range(2)]
        tmp = tempfile.mkdtemp() if r == 0 else None
        tmp = D.all_gather_object(tmp)[0]
        res = D.collect_results(part, 2 * w, mode="cpu", tmpdir=tmp)
        if r == 0:
            assert sorted(res) == sorted(j * 10 + i for j in range(w) for i in range(2)), res

    def t_all_reduce_params_coalesced():
        # mixed dtypes + a 1-MB bucket limit: several flat buckets, each one collective
        ps = [torch.nn.Parameter(torch.full((300, 1000), float(r + 1), device=dev)),
              torch.full((5,), r, dtype=torch.int64, device=dev),
              torch.full((7, 3), float(2 * r), device=dev)]
        D.all_reduce_params(ps, bucket_size_mb=1)
        assert torch.all(ps[0].data == w * (w + 1) / 2)
        assert torch.all(ps[1] == w * (w - 1) // 2) and torch.all(ps[2] == w * (w - 1))
        qs = [torch.full((4,), float(r), device=dev) for _ in range(3)]
        D.all_reduce_params((q for q in qs), coalesce=False, op="max")
        assert all(torch.all(q == w - 1) for q in qs)
        xs = [torch.full((3,), float(r), device=dev), torch.ones(2, 2, device=dev)]
        D._all_reduce_coalesced(xs, op="mean")
        assert torch.allclose(xs[0], torch.full((3,), (w - 1) / 2, device=dev)) and torch.all(xs[1] == 1)

    def t_collect_results_names():
        part = [r * 10 + i for i in range(2)]
        res = D.collect_results_gpu(part, 2 * w)
        if r == 0:
            assert res == [j * 10 + i for i in range(2) for j in range(w)], res
        tmp = D.all_gather_object(tempfile.mkdtemp() if r == 0 else None)[0]
        res = D.collect_results_cpu(part, 2 * w - 1, tmpdir=tmp)
        if r == 0:
            assert res == [j * 10 + i for i in range(2) for j in range(w)][: 2 * w - 1], res

    def t_barrier_and_groups():
        D.barrier()
        g = D.new_group(list(range(w)))
        t = torch.ones(1, device=dev)
        D.all_reduce(t, group=g)
        assert t.item() == w
        assert D.global_rank_of(g, r) == r

    return [(f.__name__[2:], f) for f in (
        t_all_reduce_sum, t_all_reduce_mean_max_min, t_all_reduce_async, t_broadcast, t_all_gather,
        t_reduce_scatter, t_reduce, t_scatter, t_gather, t_all_to_all, t_p2p_ring, t_object_collectives,
        t_all_reduce_dict, t_sync_random_seed_and_collect, t_all_reduce_params_coalesced, t_collect_results_names,
        t_barrier_and_groups)]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    args = ap.parse_args()
    rank, _, world = D.init_dist(backend=args.backend, use_cpu=args.backend == "gloo")
    dev = _dev(args.backend)
    failed = []
    for name, fn in collective_cases(dev):
        try:
            fn()
            ok = True
        except Exception:  # noqa: BLE001
            ok = False
            failed.append((name, traceback.format_exc()))
        oks = D.all_gather_object(ok)
        if rank == 0:
            print(f"[{'PASS' if all(oks) else 'FAIL'}] {name} (world {world}, {args.backend})", flush=True)
    if rank == 0:
        if failed:
            for n, tb in failed:
                print(f"--- {n}\n{tb}")
        else:
            print(f"ALL {len(collective_cases(dev))} PASSED")
    all_failed = D.all_gather_object(len(failed))
    D.cleanup_dist()
    return 1 if any(all_failed) else 0


if __name__ == "__main__":
    sys.exit(main())

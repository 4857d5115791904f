"""Aux subsystems: collective-order race detection, step
watchdog, roctx ranges, comm benchmark -- CPU / gloo."""
from __future__ import annotations

import pytest
import torch

from tests.dist_harness import run_workers


def _mismatch_worker(rank, world):
    import torch.distributed as dist

    from scaletorch_amd.dist import debug

    dist.init_process_group("gloo", rank=rank, world_size=world)
    debug.enable(timeout_s=30)
    dist.all_reduce(torch.ones(3))  # same on both ranks: passes
    try:
        dist.all_reduce(torch.ones(4 + rank))  # shapes differ: must be caught, not hang
    except debug.CollectiveMismatch as e:
        return {"caught": True, "msg": str(e), "calls": debug.checked_calls()}
    return {"caught": False, "msg": "", "calls": debug.checked_calls()}


def test_collective_mismatch_is_reported_not_hung():
    res = run_workers(_mismatch_worker, 2, timeout=120)
    for r in res:
        assert r["caught"], r
        assert "all_reduce" in r["msg"] and "(4,)" in r["msg"] and "(5,)" in r["msg"]
        assert r["calls"] == 2


def _trainer_worker(rank, world):
    from scaletorch_amd.dist import debug
    from scaletorch_amd.trainer.config import ScaleTorchArguments
    from scaletorch_amd.trainer.engine import Trainer

    a = ScaleTorchArguments(model_name_or_path="tiny-llama", synthetic_data=True, sequence_length=32, use_cpu=True,
                            backend="gloo", dtype="float32", micro_batch_size=2, data_parallel_size=2,
                            total_train_steps=2, debug_collectives=True, zero_stage=1)
    tr = Trainer(a)
    loss = tr.reduced_loss(tr.train_step())
    return {"loss": loss, "calls": debug.checked_calls()}


def test_debug_collectives_on_a_zero1_training_step():
    res = run_workers(_trainer_worker, 2, timeout=180)
    assert res[0]["loss"] == res[1]["loss"]
    assert res[0]["calls"] > 3 and res[0]["calls"] == res[1]["calls"]


def test_step_watchdog_fires_and_kicks():
    """Load-tolerant: the deadline is 20x the kick period (a descheduled test process under
    ``pytest -n 8`` must not read as a hang), and the firing is awaited with a bounded poll
    instead of one fixed sleep."""
    import time

    from scaletorch_amd.utils.watchdog import StepWatchdog

    fired = []
    wd = StepWatchdog(2.0, on_timeout=lambda info: fired.append(info), poll_s=0.05)
    wd.start()
    try:
        t0 = time.monotonic()
        for _ in range(4):
            time.sleep(0.1)
            wd.kick(step=1)
        kicked_for = time.monotonic() - t0
        if kicked_for < 1.5:  # the kicks were on time, so nothing may have fired
            assert not fired
        fired.clear()
        wd.kick(step=1)
        deadline = time.monotonic() + 20.0
        while not fired and time.monotonic() < deadline:
            time.sleep(0.05)
        assert fired and "step 1" in fired[0]
    finally:
        wd.stop()


def test_roctx_ranges_are_noops_without_profiling():
    from scaletorch_amd.utils import profiling

    with profiling.range("fwd"):
        x = torch.ones(2) + 1
    assert x.sum().item() == 4
    profiling.set_enabled(True)
    with profiling.range("fwd"):  # CPU: nvtx/roctx unavailable -> still a no-op
        pass
    profiling.set_enabled(False)


def _comm_worker(rank, world):
    import sys

    sys.argv = ["bench_comm", "--sizes", "4K,64K", "--iters", "2", "--ops", "all_reduce,reduce_scatter,all_gather,"
                "all_to_all,broadcast,sendrecv", "--backend", "gloo"]
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location(
        "bench_comm", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "bench_comm.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.run()


@pytest.mark.slow
def test_bench_comm_gloo():
    res = run_workers(_comm_worker, 2, timeout=180)
    rows = res[0]
    ops = {r["op"] for r in rows}
    assert ops == {"all_reduce", "reduce_scatter", "all_gather", "all_to_all", "broadcast", "sendrecv"}
    assert all(r["busbw_GBps"] >= 0 and r["time_us"] > 0 for r in rows)


def test_benchmark_sweep_list_and_dry_run(capsys):
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location(
        "benchmark_sweep", os.path.join(os.path.dirname(os.path.dirname(__file__)), "scripts", "benchmark_sweep.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cfgs = mod.build_configs(8)
    names = [c["name"] for c in cfgs]
    assert "llama3-8b-dp8" in names and "qwen3-8b-tp2-dp4" in names and "mixtral-8x7b-ep8" in names
    assert all(8 % (c["tp"] * c["pp"] * c["cp"] * c["ep"]) == 0 for c in cfgs)
    assert mod.main(["--gpus", "8", "--dry-run", "--filter", "^llama3-8b-tp2-pp2"]) == 0
    out = capsys.readouterr().out
    assert "--tp 2" in out and "--pp 2" in out and "--nproc-per-node=8" in out
    assert mod.parse_result('noise\n{"metric": "x", "value": 1}\n') == {"metric": "x", "value": 1}

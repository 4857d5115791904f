"""Loopback process group (dist/loopback.py): one rank of an 8-rank layout runs its real
program in one process with every collective a same-shape local copy -- the machinery of
``bench.py --slice`` (per-rank compute slices of the BASELINE 8-GPU configs).  CPU only:
each case builds the rank's model through ``Trainer`` and takes two optimizer steps."""
from __future__ import annotations

import pytest
import torch

from tests.dist_harness import run_workers


def _slice_worker(rank, world, kw):
    import os

    lw, lr = kw.pop("world"), kw.pop("rank")
    os.environ["ST_LOOPBACK_WORLD"], os.environ["ST_LOOPBACK_RANK"] = str(lw), str(lr)
    from scaletorch_amd.parallel import mesh
    from scaletorch_amd.trainer.config import ScaleTorchArguments
    from scaletorch_amd.trainer.engine import Trainer

    base = dict(model_name_or_path=kw.pop("model", "tiny-llama"), synthetic_data=True, sequence_length=64,
                use_cpu=True, backend="loopback", dtype="float32", learning_rate=1e-3, total_train_steps=3, seed=7,
                micro_batch_size=2)
    base.update(kw)
    tr = Trainer(ScaleTorchArguments(**base))
    losses = [float(tr.train_step()) for _ in range(2)]
    pg = mesh.pgm
    import torch.distributed as dist

    return dict(losses=torch.tensor(losses), layers=len(tr.raw_model.decoder_layers), world=dist.get_world_size(),
                coords=torch.tensor([pg.dp_rank, pg.pp_rank, pg.cp_rank, pg.ep_rank, pg.tp_rank]))


@pytest.mark.parametrize("kw,layers,coords", [
    (dict(world=8, rank=0, data_parallel_size=8, zero_stage=1), 2, [0, 0, 0, 0, 0]),
    (dict(world=8, rank=2, tensor_parallel_size=2, pipeline_parallel_size=2, data_parallel_size=2,
          sequence_parallel=True, gradient_accumulation_steps=4, virtual_pipeline_size=2, num_hidden_layers=4),
     2, [0, 1, 0, 0, 0]),
    (dict(world=8, rank=0, context_parallel_size=8, sequence_length=256, micro_batch_size=1), 2, [0, 0, 0, 0, 0]),
    (dict(world=8, rank=0, expert_parallel_size=8, model="tiny-mixtral", gradient_accumulation_steps=2,
          micro_batch_size=1, zero_stage=1), 2, [0, 0, 0, 0, 0]),
], ids=["dp8_zero1", "tp2pp2dp2_last_stage", "cp8", "mixtral_ep8"])
def test_loopback_rank_runs_its_layout(kw, layers, coords):
    r = run_workers(_slice_worker, 1, dict(kw))[0]
    assert r["world"] == 8
    assert r["layers"] == layers
    assert r["coords"].tolist() == coords
    assert torch.isfinite(r["losses"]).all()


def _collectives_worker(rank, world):
    import torch.distributed as dist

    from scaletorch_amd.dist.loopback import init_loopback

    init_loopback(8, 3)
    out = {}
    o = torch.empty(4)
    dist.reduce_scatter_tensor(o, torch.arange(32.0))
    out["rs"] = o
    o = torch.full((16,), -1.0)
    dist.all_gather_into_tensor(o, torch.arange(2.0))
    out["ag"] = o
    o = torch.empty(10)
    dist.all_to_all_single(o, torch.arange(4.0))
    out["a2a"] = o
    r, s = torch.empty(3), torch.full((3,), 7.0)
    for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, r, 2), dist.P2POp(dist.isend, s, 4)]):
        w.wait()
    out["p2p"] = r
    return out


def test_loopback_collectives_are_same_shape_local_copies():
    r = run_workers(_collectives_worker, 1)[0]
    assert r["rs"].tolist() == [12.0, 13.0, 14.0, 15.0]  # rank 3's chunk of its own input
    assert r["ag"].tolist() == [0.0, 1.0] * 8
    assert r["a2a"].tolist() == [0.0, 1.0, 2.0, 3.0, 0.0, 1.0, 2.0, 3.0, 0.0, 1.0]
    assert r["p2p"].tolist() == [7.0, 7.0, 7.0]  # the batch's own send, looped back


@pytest.mark.parametrize("layout,model", [("tp2pp2dp2", "tiny-llama"), ("mixtral_ep8", "tiny-mixtral")])
def test_bench_slice_prints_its_own_kind(layout, model):
    """``bench.py --layout L --slice`` (CPU here): one JSON line of kind "per-rank compute slice",
    valid false, the impersonated rank's coordinates and its HBM estimate."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--layout", layout, "--slice", "--model", model,
                        "--steps", "1", "--warmup", "1", "--seq_len", "128", "--layers", "4"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["kind"] == "per-rank compute slice" and rec["valid"] is False
    assert rec["slice_world"] == 8 and rec["layers_total"] == 4
    if layout == "tp2pp2dp2":
        assert rec["rank_coords"]["pp"] == 1 and rec["layers_on_rank"] == 2
    assert rec["hbm_estimate_gb"] is not None and rec["ms_per_step"] > 0

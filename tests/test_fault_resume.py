"""Failure detection / elastic recovery: a rank is killed mid-run (ST_FAULT_STEP fault
injection), torchrun restarts the job (--max-restarts), and --auto_resume continues
from the newest COMPLETE checkpoint, data position included -- the resumed run ends
on the same loss as an uninterrupted one (CPU / gloo, 2 ranks, ZeRO-1 AdamW).
Reference: scripts/torch_dist/launch_single_node.sh:60-100 (restart launcher),
SURVEY.md §5.3 (no fault injection / resume test in the reference)."""
from __future__ import annotations

import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _train(work_dir: str, port: int, env_extra: dict, restarts: int = 0):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           f"--max-restarts={restarts}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           "tools/train.py", "--model_name_or_path", "tiny-llama", "--synthetic_data", "True", "--use_cpu", "True",
           "--backend", "gloo", "--dtype", "float32", "--data_parallel_size", "2", "--micro_batch_size", "2",
           "--sequence_length", "32", "--total_train_steps", "6", "--save_frequency", "2", "--learning_rate",
           "1e-2", "--zero_stage", "1", "--auto_resume", "True", "--work_dir", work_dir]
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)


def _losses(text: str) -> dict:
    return {int(m.group(1)): float(m.group(2)) for m in re.finditer(r"Step: (\d+)\s*\| Loss: ([0-9.]+)", text)}


def test_kill_restart_auto_resume(tmp_path):
    clean = _train(str(tmp_path / "clean"), 29761, {})
    assert clean.returncode == 0, clean.stderr[-3000:]
    faulted = _train(str(tmp_path / "faulted"), 29763, {"ST_FAULT_STEP": "3", "ST_FAULT_RANK": "1"}, restarts=1)
    out = faulted.stdout + faulted.stderr
    assert faulted.returncode == 0, out[-3000:]
    assert "fault injection: rank 1 exits at step 3" in out
    assert "resumed from" in out and "at step 2" in out
    ref, got = _losses(clean.stdout + clean.stderr), _losses(out)
    assert 6 in ref and 6 in got, (ref, got)
    assert got[6] == ref[6], (got, ref)
    # every saved step directory carries both ranks' completion markers
    from scaletorch_amd.utils.checkpoint import is_complete, latest_checkpoint

    assert is_complete(str(tmp_path / "faulted" / "6"))
    assert latest_checkpoint(str(tmp_path / "faulted")).endswith("/6")


def test_incomplete_checkpoint_is_skipped(tmp_path):
    from scaletorch_amd.utils.checkpoint import latest_checkpoint

    for step, ranks in ((2, (0, 1)), (4, (0,))):  # step 4: rank 1 died mid-save
        d = tmp_path / str(step)
        d.mkdir()
        (d / "weights_tp_rank_world_size=0_1_pp_rank_world_size=0_1.pth").write_bytes(b"x")
        for r in ranks:
            (d / f"complete_rank_world_size={r}_2").write_text("ok\n")
    assert latest_checkpoint(str(tmp_path)).endswith("/2")


def test_unmarked_legacy_checkpoint_is_accepted_visibly(tmp_path, monkeypatch):
    """A step directory written before completion markers existed is resumed from
    (with a warning) instead of silently restarting at step 0; ST_CKPT_ACCEPT_UNMARKED=0
    restores the strict behaviour."""
    from scaletorch_amd.utils.checkpoint import latest_checkpoint

    d = tmp_path / "3"
    d.mkdir()
    (d / "weights_tp_rank_world_size=0_1_pp_rank_world_size=0_1.pth").write_bytes(b"x")
    assert latest_checkpoint(str(tmp_path)).endswith("/3")
    monkeypatch.setenv("ST_CKPT_ACCEPT_UNMARKED", "0")
    assert latest_checkpoint(str(tmp_path)) is None


def test_zero_marker_crash_falls_back_to_marked_checkpoint(tmp_path):
    """A crash mid-save before any rank wrote its completion marker: with the
    save-started sentinel the directory is recognised as partial, and even without
    it (a crash before the sentinel existed) an unmarked directory next to marked
    ones is never preferred over the newest complete marked one."""
    from scaletorch_amd.utils.checkpoint import is_complete, latest_checkpoint

    w = "weights_tp_rank_world_size=0_1_pp_rank_world_size=0_1.pth"
    d2 = tmp_path / "2"
    d2.mkdir()
    (d2 / w).write_bytes(b"x")
    for r in (0, 1):
        (d2 / f"started_rank_world_size={r}_2").write_text("started\n")
        (d2 / f"complete_rank_world_size={r}_2").write_text("ok\n")
    d4 = tmp_path / "4"  # crash after rank 0's first file, no completion marker at all
    d4.mkdir()
    (d4 / w).write_bytes(b"x")
    (d4 / "started_rank_world_size=0_2").write_text("started\n")
    assert not is_complete(str(d4))
    assert latest_checkpoint(str(tmp_path)).endswith("/2")
    (d4 / "started_rank_world_size=0_2").unlink()  # no sentinel either: the sibling decides
    assert not is_complete(str(d4))
    assert latest_checkpoint(str(tmp_path)).endswith("/2")


def test_crash_in_first_marked_save_after_legacy_resume(tmp_path):
    """Legacy (unmarked) steps 1000 and 2000, then the current code crashes during its
    first save (step 2100: save-started sentinel, no completion marker): auto-resume
    falls back to legacy step 2000 -- an OLDER marked sibling is what disqualifies an
    unmarked directory, a newer partial one is not."""
    from scaletorch_amd.utils.checkpoint import is_complete, latest_checkpoint

    w = "weights_tp_rank_world_size=0_1_pp_rank_world_size=0_1.pth"
    for step in (1000, 2000, 2100):
        d = tmp_path / str(step)
        d.mkdir()
        (d / w).write_bytes(b"x")
    (tmp_path / "2100" / "started_rank_world_size=0_2").write_text("started\n")
    assert not is_complete(str(tmp_path / "2100"))
    assert is_complete(str(tmp_path / "2000"))
    assert latest_checkpoint(str(tmp_path)).endswith("/2000")
    # the current code then completes 2200 and crashes in 2300 before any marker: 2300 is
    # unmarked with an older marked sibling -> skipped; 2200 wins
    for step in (2200, 2300):
        d = tmp_path / str(step)
        d.mkdir()
        (d / w).write_bytes(b"x")
    for r in (0, 1):
        (tmp_path / "2200" / f"started_rank_world_size={r}_2").write_text("started\n")
        (tmp_path / "2200" / f"complete_rank_world_size={r}_2").write_text("ok\n")
    assert not is_complete(str(tmp_path / "2300"))
    assert latest_checkpoint(str(tmp_path)).endswith("/2200")


def _resume_corrupt_worker(rank, world, work_dir):
    import torch

    from scaletorch_amd.trainer.config import ScaleTorchArguments
    from scaletorch_amd.trainer.engine import Trainer
    from scaletorch_amd.utils.checkpoint import CheckpointManager

    a = ScaleTorchArguments(model_name_or_path="tiny-llama", synthetic_data=True, use_cpu=True, backend="gloo",
                            dtype="float32", data_parallel_size=2, micro_batch_size=1, sequence_length=16,
                            total_train_steps=4, zero_stage=1, num_hidden_layers=1)
    tr = Trainer(a)
    tr.train_step()
    ck = CheckpointManager(work_dir, async_save=False)
    path = os.path.dirname(ck.save_checkpoint(tr.model, tr.optimizer, 1, 0, lr_scheduler=tr.lr_scheduler))
    torch.distributed.barrier()
    if rank == 1:  # truncate this rank's ZeRO-1 optimizer shard: torch.load raises a non-RuntimeError
        shard = "optimizer_shard_rank_world_size=1_2.pth"
        with open(os.path.join(path, shard), "r+b") as f:
            f.truncate(37)
    torch.distributed.barrier()
    try:
        tr.resume(ck, path)
    except RuntimeError as e:
        return f"raised: {e}"
    return "resumed"


def test_resume_corrupt_shard_fails_on_every_rank(tmp_path):
    from tests.dist_harness import run_workers

    out = run_workers(_resume_corrupt_worker, 2, str(tmp_path), timeout=240)
    assert all(o.startswith("raised") for o in out), out

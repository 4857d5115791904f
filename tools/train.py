#!/usr/bin/env python3
"""Training entry point (reference: tools/train.py, root train.py -> symlink).

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py \
      --model_name_or_path llama3-8b --synthetic_data True \
      --data_parallel_size 8 --micro_batch_size 2 --sequence_length 4096 --total_train_steps 100

Prints the reference's per-step line (parsed by its benchmark scripts):
  [rank r] Step: N | Loss: x | LR: x | GradNorm: x | Global batch size: x | Tokens/s: x |
  Tokens/s/GPU: x | Tokens: x | MFU: x% | Memory: xGB
but the timing covers the FULL step (fwd, bwd, grad all-reduce, clip, optimizer).
Honours --save_frequency/--resume_path/--auto_resume (reference checkpoint
layout), --profile (torch.profiler, ROCm/roctracer), --use_wandb, and the
fault-injection env ST_FAULT_STEP / ST_FAULT_RANK used by the resume tests.
"""
from __future__ import annotations

import json
import math
import os
import signal
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.realpath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# one hardware queue per stream (compute, optimizer side stream, W^T, RCCL): see bench.py
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import torch  # noqa: E402

from scaletorch_amd.dist import collectives as C  # noqa: E402
from scaletorch_amd.dist.launch import cleanup_dist  # noqa: E402
from scaletorch_amd.parallel import mesh  # noqa: E402
from scaletorch_amd.trainer.config import parse_args  # noqa: E402
from scaletorch_amd.trainer.engine import Trainer  # noqa: E402
from scaletorch_amd.utils.checkpoint import CheckpointManager, latest_checkpoint  # noqa: E402
from scaletorch_amd.utils.device import get_theoretical_flops  # noqa: E402
from scaletorch_amd.dist import trace as comm_trace  # noqa: E402
from scaletorch_amd.utils.logger import PerformanceMonitor, get_logger  # noqa: E402
from scaletorch_amd.utils.misc import comm_per_step, pipeline_bubble_fraction  # noqa: E402
from scaletorch_amd.utils.misc import flops_per_token, rank_print, to_readable_format  # noqa: E402


def _is_log_rank() -> bool:
    pg = mesh.pgm
    if not pg:
        return True
    return pg.tp_rank == 0 and pg.dp_rank == 0 and pg.cp_rank == 0 and pg.ep_rank == 0 and pg.pp_is_last_stage


def main(argv=None) -> int:
    args = parse_args(argv)
    log = get_logger()
    tr = Trainer(args)
    cfg = tr.model_config
    world = tr.world
    log.info("config: %s", json.dumps({k: v for k, v in vars(args).items()}, default=str)[:2000])
    log.info("model %s: %.2fB params (%.2fB active)", cfg.name, cfg.num_params() / 1e9, cfg.active_params() / 1e9)

    ckpt = CheckpointManager(args.work_dir, async_save=args.async_save)
    resume = args.resume_path or (latest_checkpoint(args.work_dir) if args.auto_resume else None)
    if args.auto_resume and not args.resume_path and world > 1:
        resume = C.broadcast_object_list([resume], src=0)[0]  # one decision for every rank
    if resume:
        tr.resume(ckpt, resume)  # fatal on every rank if any rank cannot load
        log.info("resumed from %s at step %d", resume, tr.step)

    wandb = None
    if args.use_wandb and _is_log_rank():
        try:
            import wandb as _wb

            _wb.init(project=args.project_name, name=args.experiment_name, config=vars(args))
            wandb = _wb
        except Exception as e:  # no network here; keep training
            log.warning("wandb unavailable: %s", e)

    total = args.total_train_steps or 1000
    # fault injection (tests): on the first launch only, so a torchrun restart can resume
    fault_step = int(os.environ.get("ST_FAULT_STEP", "-1"))
    if int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0:
        fault_step = -1
    fault_rank = int(os.environ.get("ST_FAULT_RANK", "0"))
    monitor = PerformanceMonitor(warmup_steps=2, rank=tr.rank)
    monitor.extra["pp_bubble_fraction"] = round(pipeline_bubble_fraction(
        args.pipeline_parallel_size, args.gradient_accumulation_steps, args.virtual_pipeline_size), 4)
    comm0 = None  # (step, trace.stats()) once the monitor's warm-up is over
    n_active = cfg.active_params()
    fpt = flops_per_token(n_active, cfg.num_hidden_layers, cfg.num_attention_heads, cfg.head_dim,
                          args.sequence_length)
    peak = get_theoretical_flops()
    prof = None
    if args.profile:
        from torch.profiler import ProfilerActivity, profile, schedule, tensorboard_trace_handler

        prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                       schedule=schedule(wait=2, warmup=1, active=3, repeat=1),
                       on_trace_ready=tensorboard_trace_handler(args.profile_dir), record_shapes=False)
        prof.start()
        from scaletorch_amd.utils import profiling

        profiling.set_enabled(True)  # roctx ranges around fwd / bwd / optimizer in the trace
    watchdog = None
    if args.watchdog_s and args.watchdog_s > 0:
        from scaletorch_amd.utils.watchdog import StepWatchdog

        watchdog = StepWatchdog(args.watchdog_s).start()
    epoch_bound = not args.total_train_steps and not args.max_tokens
    stop = {"flag": False}
    signal.signal(signal.SIGTERM, lambda *_: stop.__setitem__("flag", True))
    try:
        while tr.step < total and not stop["flag"]:
            if args.max_tokens and tr.trained_tokens >= args.max_tokens:
                break
            # --epochs bounds the run only when neither --total_train_steps nor --max_tokens is
            # given (reference precedence: trainer/config.py:321-325)
            if epoch_bound and getattr(tr.data, "epoch", 0) >= args.epochs:
                log.info("completed %d epochs", args.epochs)
                break
            if tr.step == fault_step and tr.rank == fault_rank:
                log.error("fault injection: rank %d exits at step %d", tr.rank, tr.step)
                os._exit(17)
            monitor.start_iteration()
            loss_t = tr.train_step()
            log_now = tr.step % max(1, args.log_interval) == 0 or tr.step == total
            rec = monitor.end_iteration(tr.tokens_per_step, sync=log_now)  # events only: no device-wide sync
            if comm0 is None and tr.step >= monitor.warmup:
                comm0 = (tr.step, comm_trace.stats())
            if watchdog is not None:
                watchdog.kick(tr.step)
            if prof is not None:
                prof.step()
            if log_now:
                tr.health_check()  # xGMI collective timeouts -> non-zero exit (restart + --auto_resume)
                loss = tr.reduced_loss(loss_t)
                if args.nan_check and loss != loss:
                    raise FloatingPointError(f"non-finite loss at step {tr.step}")
                gn = tr.optimizer.last_grad_norm
                gn = float(gn.item()) if gn is not None else None
                if args.nan_check and gn is not None and not math.isfinite(gn):
                    raise FloatingPointError(f"non-finite gradient norm {gn} at step {tr.step}")
                tok_s = rec["tokens_per_s"]
                per_gpu = tok_s / world
                mfu = per_gpu * fpt / peak * 100
                if _is_log_rank():
                    mt = ("/" + to_readable_format(args.max_tokens)) if args.max_tokens else ""
                    parts = [f"[rank {tr.rank}]", f"Step: {tr.step:<5d}", f"Loss: {loss:6.4f}",
                             f"LR: {tr.lr_scheduler.get_last_lr()[0]:.2e}"]
                    if gn is not None:
                        parts.append(f"GradNorm: {gn:.2f}")
                    parts += [f"Global batch size: {to_readable_format(tr.tokens_per_step):>7s}",
                              f"Tokens/s: {to_readable_format(tok_s):>7s}",
                              f"Tokens/s/GPU: {to_readable_format(per_gpu):>7s}",
                              f"Tokens: {to_readable_format(tr.trained_tokens):>7s}{mt}",
                              f"MFU: {mfu:5.2f}%"]
                    if torch.cuda.is_available():
                        parts.append(f"Memory: {torch.cuda.memory_reserved() / 1e9:6.2f}GB")
                    rank_print(" | ".join(parts))
                    if wandb is not None:
                        wandb.log({"loss": loss, "tokens_per_second": tok_s, "tokens_per_second_per_gpu": per_gpu,
                                   "mfu": mfu, "grad_norm": gn, "trained_tokens": tr.trained_tokens}, step=tr.step)
            if args.eval_interval > 0 and tr.step % args.eval_interval == 0:
                vloss = tr.evaluate()
                if _is_log_rank():
                    rank_print(f"[rank {tr.rank}] Step: {tr.step:<5d} | Eval loss: {vloss:6.4f} | "
                               f"Eval sequences: {args.test_batch_size}")
            if args.save_model_checkpoint and args.save_frequency > 0 and tr.step % args.save_frequency == 0:
                ckpt.save_checkpoint(tr.model, tr.optimizer, tr.step, tr.trained_tokens, lr_scheduler=tr.lr_scheduler)
    except KeyboardInterrupt:
        log.warning("interrupted; cleaning up")
    finally:
        if watchdog is not None:
            watchdog.stop()
        if prof is not None:
            prof.stop()
        ckpt.wait()
        if comm0 is not None and tr.step > comm0[0]:
            monitor.extra["comm_per_step"] = comm_per_step(comm0[1], comm_trace.stats(), tr.step - comm0[0])
        if tr.rank == 0 or _is_log_rank():
            s = monitor.summary()
            if s:
                log.info("performance: %s", json.dumps(s))
            monitor.dump(os.path.join(args.work_dir, "perf"))
        if wandb is not None:
            wandb.finish()
        cleanup_dist()
    return 0


if __name__ == "__main__":
    sys.exit(main())

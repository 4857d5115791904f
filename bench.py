#!/usr/bin/env python3
"""Headline benchmark: Llama-3-8B training throughput on MI355X (synthetic data, random init).

Metric (BASELINE.json): tokens/sec (+ MFU) of a full Llama-3-8B training step
-- forward, backward, DP gradient all-reduce, global grad-norm clip and the
fused AdamW update are ALL inside the timed region (the reference timed only
fwd+bwd).  Weak scaling: every GPU processes
``--micro_batch_size x --seq_len`` tokens per micro-batch; N GPUs = DP=N
(override the layout with --tp/--pp/--cp/--ep).

Default micro-batch is 6 x 4096 tokens with the fused chunked LM head + CE (the
[tokens, vocab] logits never exist; the head's dW goes straight into main_grad):
271.0 GB peak at DP=1 of 288 GB (utils/memory.py estimates 271.4; less under
ZeRO-1 at DP > 1).  Same-box A/B on one MI355X (profiles/r02/mbs6_fused_head_ab.log):
mbs 4 + logits/CE 700.8 ms = 23.38k tok/s, mbs 6 + fused head 1025-1033 ms =
23.78-23.98k tok/s (+1.7-2.5 %); mbs 6 with materialised logits does not fit.

Usage:
  python bench.py --gpus 1 --steps 10 --warmup 3
  python bench.py --gpus 8 --steps 10 --warmup 3      # starts 8 ranks itself (torchrun child process)
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --steps 10 --warmup 3
  torchrun --nproc-per-node 8 ... bench.py --gpus 8 --layout tp2pp2dp2   # BASELINE.json 8-GPU configs:
      dp (default) | tp2pp2dp2 | cp8_32k | mixtral_ep8  (explicit flags override a preset)

Every run prints its per-rank HBM estimate (utils/memory.py) to stderr before
building anything and refuses a layout that would not fit in 288 GB.

Rank 0 prints ONE JSON line; ``value`` = whole-job tokens/s (all GPUs).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4); past that,
# streams share a queue and their kernels run in submission order.  A step drives the
# compute stream, the optimizer side stream, the W^T stream and, at DP > 1, RCCL's
# streams (one per communicator): give each its own queue so a collective waiting on a
# peer never sits in front of compute.  Read when the HIP runtime starts: set before torch.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

# Qwen3-8B TP2-DP4 S2048, 8x Ascend 910B: 1,391 tok/s/GPU (README.md:84 of the
# reference) -- the nearest published 8B row whose step does
# real DP/TP work.  vs_baseline compares per-GPU throughput against it.
BASELINE_TOK_S_PER_GPU = 1391.0

# BASELINE.json's 8-GPU configurations (reference scripts/benchmark_comprehensive.py:54-173
# layouts).  Sizes are per GPU; the data-parallel width absorbs the rest of the job.
LAYOUTS = {
    "dp": dict(),
    # 3-D: TP inside an xGMI pair, 2 pipeline stages, DP over the rest; 8 micro-batches through
    # the interleaved 1F1B schedule with 2 chunks per stage keep the bubble at
    # (pp-1)/(V*M+pp-1) = 6 % (11 % plain 1F1B); sequence parallel shards norm/residual activations.
    # Layers per chunk 9,8,8,7 (stage 0: 17, last stage: 15 + final norm, LM head and loss): the
    # per-rank slices ran the even split at 1333 / 1487 ms per stage and this one at 1417 / 1401,
    # so the pipeline's pace (its slowest stage) drops 4.7 % (profiles/r06/pp_balance/)
    "tp2pp2dp2": dict(tp=2, pp=2, sp=True, micro_batch_size=4, grad_acc=8, vpp=2, layer_distribution="9,8,8,7"),
    # long context: 32K tokens over 8 CP ranks (4K local), zig-zag chunks, GQA-sized K/V
    "cp8_32k": dict(cp=-1, seq_len=32768, micro_batch_size=1),
    # Mixtral 8x7B: one expert per GPU (EP carved out of DP), dense weights ZeRO-1 over DP x EP;
    # DROPLESS dispatch with the routing counts on the device (models/moe.py): exchange buffers
    # sized by the worst case ep*T*min(k, E/ep) rows, so nothing is dropped and -- over the xGMI
    # push exchange -- no count is read by the host.  mbs 1 x GA 2 (the R_max buffers of mbs 2
    # would not fit in 288 GB: utils/memory.py), the same 8192 tokens per GPU per step
    # EP transport: RCCL (host counts -> exact-row expert buffers: 140 vs 179 GB peak per rank),
    # the path the per-rank slices measured; --ep_comm auto / xgmi select the push exchange
    "mixtral_ep8": dict(model="mixtral-8x7b", ep=-1, micro_batch_size=1, grad_acc=2, moe_capacity_factor=0.0,
                        ep_comm="rccl"),
}


def _tp_transport() -> dict:
    """TP transport the trainer chose (tensor_parallel.select_tp_transport) + its self-test."""
    from scaletorch_amd.parallel.tensor_parallel import TRANSPORT

    return dict(TRANSPORT)


def _planned_ipc(args, mcfg) -> int:
    """IPC areas the start-up transport self-tests may keep (utils/memory.py comm term)."""
    if args.tp <= 1 and args.ep <= 1:
        return 0
    from scaletorch_amd.dist.xgmi import planned_ipc_bytes

    tokens = args.micro_batch_size * (args.seq_len // max(1, args.cp))
    area = None
    if args.ep > 1 and mcfg.is_moe:
        from scaletorch_amd.models.moe import ep_area_bytes

        area = ep_area_bytes(tokens, args.ep, mcfg.num_experts_per_tok, mcfg.num_experts, mcfg.hidden_size,
                             args.moe_capacity_factor)
    return planned_ipc_bytes(args.tp, args.ep, tokens * mcfg.hidden_size * 2,
                             moe_dropless=args.moe_capacity_factor == 0 and args.ep > 1, ep_area=area)


def _visible_gpus() -> int:
    """GPUs this process may use, counted WITHOUT the HIP runtime (so the parent that
    starts the ranks never initialises a GPU): the KFD topology nodes that have SIMDs
    (GPU agents; CPU nodes report simd_count 0), narrowed by the visible-devices
    variables.  Falls back to torch.cuda.device_count() (hipGetDeviceCount, which does
    initialise HIP in this process) only when the topology is unreadable."""
    import glob

    n = 0
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(props) as f:
                kv = dict(line.split(None, 1) for line in f if line.strip())
            n += int(kv.get("simd_count", "0").strip()) > 0
        except (OSError, ValueError):
            continue
    if n == 0:
        import torch

        return torch.cuda.device_count()
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def _self_launch(n: int, argv: list[str], backend: str) -> int:
    """``python bench.py --gpus N`` without a launcher: start N ranks as one torchrun
    CHILD process (never exec: the parent must not replace itself) on 127.0.0.1,
    let rank 0's JSON line through and return the child's exit code.
    Mirrors the reference driver building its own torchrun command per config
    (scripts/benchmark_comprehensive.py:177-215)."""
    import socket
    import subprocess

    if backend != "gloo":
        have = _visible_gpus()
        if n > have:
            print(f"bench: --gpus {n} but only {have} GPU(s) visible; refusing to start", file=sys.stderr)
            return 2
    with socket.socket() as s:  # a free rendezvous port
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", ST_BENCH_SELF_LAUNCHED="1")
    print(f"[bench] --gpus {n} with no WORLD_SIZE: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr,
          flush=True)
    return subprocess.call(cmd, env=env)


def _slice_record(out: dict, args, est, est_run, tr, dp: int, world: int, elapsed: float) -> dict:
    """The JSON of a per-rank compute slice: its own kind, never a throughput result."""
    import torch

    from scaletorch_amd.parallel import mesh

    pg = mesh.pgm
    coords = {k: getattr(pg, f"{k}_rank") for k in ("dp", "pp", "cp", "ep", "tp")} if pg else {}
    peak_gb = torch.cuda.max_memory_allocated() / 1e9 if torch.cuda.is_available() else 0.0
    est_gb = float(est.total_gb)
    rec = {
        "kind": "per-rank compute slice",
        "valid": False,
        "why_not_a_result": "one rank of an 8-GPU layout on one GPU; collectives are same-shape local copies "
                            "(dist/loopback.py), no communication, no pipeline bubble",
        "layout": args.layout, "slice_world": world, "rank": int(os.environ.get("ST_LOOPBACK_RANK", "0")),
        "rank_coords": coords, "model": args.model, "layers_total": tr.model_config.num_hidden_layers,
        "layers_on_rank": len(tr.raw_model.decoder_layers),
        "ms_per_step": round(elapsed / args.steps * 1000, 2), "steps": args.steps, "warmup": args.warmup,
        "tokens_per_step_global": tr.tokens_per_step,
        "tokens_per_s_per_gpu_upper_bound": out["tokens_per_s_per_gpu"],
        "mfu_pct_per_rank_upper_bound": out["mfu_pct"], "mfu_pct_strict_per_rank_upper_bound": out["mfu_pct_strict"],
        "peak_hbm_gb": round(peak_gb, 2), "hbm_estimate_gb": round(est_gb, 2) if est_gb else None,
        "hbm_estimate_err_pct": round(100 * (peak_gb - est_gb) / est_gb, 1) if est_gb else None,
        "hbm_estimate": est.summary(),
        "hbm_estimate_8gpu_worst_rank_gb": round(float(est_run.total_gb), 2),
        "comm_mb_per_step_rank": out["comm_mb_per_step_rank0"],
        "moe_dispatch": out["moe_dispatch"], "config": out["config"], "final_loss": out["final_loss"],
        "dtype": "bf16", "data": out["data"],
    }
    return rec


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Without torchrun (no WORLD_SIZE) and N > 1, bench.py starts "
                         "the N ranks itself; under torchrun it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layout", default="dp", choices=sorted(LAYOUTS))
    ap.add_argument("--model", default=None, help="default llama3-8b")
    ap.add_argument("--micro_batch_size", type=int, default=None, help="default 6 (layout presets set their own)")
    ap.add_argument("--seq_len", type=int, default=None, help="default 4096")
    ap.add_argument("--grad_acc", type=int, default=None, help="default 1")
    ap.add_argument("--tp", type=int, default=None)
    ap.add_argument("--pp", type=int, default=None)
    ap.add_argument("--cp", type=int, default=None)
    ap.add_argument("--ep", type=int, default=None)
    ap.add_argument("--sp", action="store_true", default=None)
    ap.add_argument("--vpp", type=int, default=None, help="model chunks per pipeline stage (interleaved 1F1B)")
    ap.add_argument("--layer_distribution", default=None,
                    help="comma list of layers per pipeline chunk (global chunk order with --vpp > 1)")
    ap.add_argument("--cp_comm", default="auto", help="auto | allgather | ring | ulysses")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) | gloo (debug rehearsals only)")
    ap.add_argument("--gc", action="store_true", help="activation checkpointing")
    ap.add_argument("--recompute", default="selective", help="with --gc: full | selective (norm+MLP only)")
    ap.add_argument("--grad_reduce_dtype", default="bf16")
    ap.add_argument("--bucket_mb", type=float, default=256)
    ap.add_argument("--zero", type=int, default=1, help="ZeRO stage when DP > 1 (0: replicated optimizer, "
                                                         "1: sharded optimizer / reduce-scatter + all-gather)")
    ap.add_argument("--fused_head", type=int, default=1,
                    help="1: fused chunked LM head + CE (no logits tensor, dW straight into main_grad); "
                         "0: logits + vocab-parallel CE")
    ap.add_argument("--head_chunk", type=int, default=4096, help="tokens per fused LM-head chunk")
    ap.add_argument("--layers", type=int, default=None, help="(debug only; result marked invalid)")
    ap.add_argument("--moe_capacity_factor", type=float, default=None,
                    help="EP dispatch: 0 dropless (one host read of the counts per layer), > 0 static capacity")
    ap.add_argument("--gemm_tuning", default="auto", choices=["auto", "use", "tune", "off"],
                    help="TunableOp table for the library GEMMs (utils/gemm_tuning.py); tune: time every "
                         "solution of each new GEMM signature in the warm-up and add it to the table")
    ap.add_argument("--opt_state_dtype", default="bf16", choices=["fp32", "bf16"],
                    help="AdamW moment dtype: bf16 (default) = the reference's own optimizer-state precision "
                         "(torch AdamW on its bf16 model keeps bf16 exp_avg / exp_avg_sq and NO master "
                         "weights); ours keeps fp32 master weights either way")
    ap.add_argument("--moe_ep_chunks", type=int, default=None, help="EP dispatch chunks (capacity mode)")
    ap.add_argument("--slice", action="store_true",
                    help="per-rank compute slice: run ONE rank of the --layout on this GPU at full depth, with every "
                         "collective replaced by a same-shape local copy (dist/loopback.py); prints its own JSON "
                         "kind, valid: false -- per-rank kernels and HBM of a layout no 8-GPU box is here to run")
    ap.add_argument("--slice_world", type=int, default=8, help="world size of the sliced layout")
    ap.add_argument("--slice_stage", default="last", choices=["first", "last"],
                    help="pipeline stage the slice impersonates: last (final norm + LM head + loss, the "
                         "heavier compute) or first (embedding, the most micro-batches in flight: peak HBM)")
    ap.add_argument("--tp_comm", default="auto", choices=["auto", "rccl", "xgmi"],
                    help="TP / SP transport: auto (self-tested xGMI paths at start-up, RCCL fallback), rccl, xgmi")
    ap.add_argument("--ep_comm", default=None, choices=["auto", "rccl", "xgmi"],
                    help="EP exchange transport: rccl (host counts, exact-row expert buffers), xgmi (push "
                         "exchange, device counts, R_max-row buffers), auto (xgmi when its self-test passes)")
    args = ap.parse_args()
    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.slice:
        if launched and world > 1:
            raise SystemExit("--slice runs ONE rank in one process; do not start it under a launcher")
        world = args.slice_world
        args.gpus = world
        args.backend = "loopback"
    if args.gpus is None:
        args.gpus = world
    if not launched and args.gpus > 1 and not args.slice:
        return _self_launch(args.gpus, sys.argv[1:], args.backend)
    if args.gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {args.gpus})")
    if world != args.gpus and not args.slice:
        # a mismatch would report a different job size than the one asked for
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    preset = dict(model="llama3-8b", micro_batch_size=6, seq_len=4096, grad_acc=1, tp=1, pp=1, cp=1, ep=1, sp=False,
                  vpp=1, moe_capacity_factor=0.0, moe_ep_chunks=1, layer_distribution=None, ep_comm="auto")
    preset.update({k: (world if v == -1 else v) for k, v in LAYOUTS[args.layout].items()})
    user_dist = args.layer_distribution
    for k, v in preset.items():
        if getattr(args, k) is None:
            setattr(args, k, v)

    import torch
    import torch.distributed as dist

    from scaletorch_amd.trainer.config import ScaleTorchArguments
    from scaletorch_amd.trainer.engine import Trainer
    from scaletorch_amd.utils.device import get_theoretical_flops
    from scaletorch_amd.utils.misc import flops_per_token

    mp = args.tp * args.pp * args.cp * args.ep
    if world % mp:
        raise SystemExit(f"world {world} not divisible by tp*pp*cp*ep={mp}")
    dp = world // mp
    ga = args.grad_acc
    if args.slice:
        # the rank to impersonate: the LAST pipeline stage (embedding-free, final norm + LM head:
        # the heavier stage), first of every other axis.  Mesh order [dp, pp, cp, ep, tp], TP fastest.
        stage = args.pp - 1 if args.slice_stage == "last" else 0
        rep = stage * args.cp * args.ep * args.tp
        os.environ["ST_LOOPBACK_WORLD"], os.environ["ST_LOOPBACK_RANK"] = str(world), str(rep)
    if args.pp > 1:
        # the (interleaved) 1F1B schedule needs >= pp micro-batches in flight -- a multiple of
        # pp with virtual stages; fewer is an error, never silently raised
        if ga < args.pp or (args.vpp > 1 and ga % args.pp):
            raise SystemExit(f"--grad_acc {ga} with pp={args.pp} vpp={args.vpp}: need a multiple of pp "
                             f"(>= {args.pp}); >= {4 * args.pp} keeps the bubble under ~20 %")
        if ga < 4 * args.pp and int(os.environ.get("RANK", "0")) == 0:
            print(f"[bench] note: grad_acc {ga} < 4*pp: pipeline bubble (pp-1)/(vpp*M+pp-1) = "
                  f"{(args.pp - 1) / (args.vpp * ga + args.pp - 1):.0%}", file=sys.stderr)
    from scaletorch_amd.models import get_model_config
    from scaletorch_amd.utils.memory import estimate_rank_memory

    mcfg = get_model_config(args.model, num_hidden_layers=args.layers)
    if args.layer_distribution:
        d = [int(x) for x in args.layer_distribution.split(",")]
        nchunks = args.pp * (args.vpp if args.pp > 1 else 1)
        if args.pp == 1 or len(d) != nchunks or sum(d) != mcfg.num_hidden_layers:
            if user_dist:
                raise SystemExit(f"--layer_distribution {user_dist}: need {nchunks} entries summing to "
                                 f"{mcfg.num_hidden_layers} layers")
            args.layer_distribution = None  # the preset's split is for its own model / layout
    def estimate(slice_rank: bool):
        """HBM of the 8-GPU run's worst rank (first stage, planned IPC areas, the transport's
        expert buffers) or, ``slice_rank``, of the rank this slice runs (no IPC areas, RCCL EP)."""
        return estimate_rank_memory(
            mcfg, tp=args.tp, pp=args.pp, cp=args.cp, ep=args.ep, dp=dp, micro_batch=args.micro_batch_size,
            seq_len=args.seq_len, grad_acc=ga, zero1=args.zero >= 1 and dp * args.cp * args.ep > 1,
            sequence_parallel=args.sp, gradient_checkpointing=(args.recompute if args.gc else False),
            grad_reduce_dtype=args.grad_reduce_dtype, fused_head_chunk=args.head_chunk if args.fused_head else 0,
            moe_dropless=args.moe_capacity_factor == 0 and args.ep > 1, optimizer_state_dtype=args.opt_state_dtype,
            xgmi_ipc_bytes=0 if slice_rank else _planned_ipc(args, mcfg),
            pp_rank=(args.pp - 1 if slice_rank and args.slice_stage == "last" else 0),
            virtual_pipeline=args.vpp if args.pp > 1 else 1,
            moe_exact_rows=args.ep_comm == "rccl" or slice_rank,
            layer_distribution=[int(x) for x in args.layer_distribution.split(",")] if args.layer_distribution else None)

    est_run = estimate(False)
    est = estimate(True) if args.slice else est_run
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] layout {args.layout}: {args.model} tp{args.tp} pp{args.pp} cp{args.cp} ep{args.ep} dp{dp} "
              f"mbs{args.micro_batch_size} ga{ga} seq{args.seq_len}; HBM estimate {est.summary()}",
              file=sys.stderr, flush=True)
    if not est.fits() or not est_run.fits():
        raise SystemExit(f"layout {args.layout} would not fit: {est_run.summary()}")
    a = ScaleTorchArguments(
        model_name_or_path=args.model, synthetic_data=True, micro_batch_size=args.micro_batch_size,
        sequence_length=args.seq_len, gradient_accumulation_steps=ga, total_train_steps=args.warmup + args.steps,
        tensor_parallel_size=args.tp, pipeline_parallel_size=args.pp, context_parallel_size=args.cp,
        virtual_pipeline_size=args.vpp if args.pp > 1 else 1, layer_distribution=args.layer_distribution,
        expert_parallel_size=args.ep, data_parallel_size=dp, sequence_parallel=args.sp,
        cp_comm=args.cp_comm, backend=args.backend,
        gradient_checkpointing=args.gc, recompute_granularity=args.recompute, learning_rate=3e-4, lr_scheduler_type="cosine", warmup_steps=0,
        max_grad_norm=1.0, grad_reduce_dtype=args.grad_reduce_dtype, bucket_size_mb=args.bucket_mb,
        num_hidden_layers=args.layers, dtype="bfloat16", weight_decay=0.1, betas=(0.9, 0.95),
        zero_stage=args.zero, fused_lm_head=bool(args.fused_head), lm_head_chunk_tokens=args.head_chunk,
        moe_capacity_factor=args.moe_capacity_factor, moe_ep_chunks=args.moe_ep_chunks,
        optimizer_state_dtype=args.opt_state_dtype, gemm_tuning=args.gemm_tuning, ep_comm=args.ep_comm,
        tp_comm=args.tp_comm,
    )
    if args.backend == "gloo" and torch.cuda.is_available():  # 1-GPU multi-rank rehearsal
        from scaletorch_amd.dist.gloo_staging import stage_gloo_cuda_p2p

        stage_gloo_cuda_p2p()
    tr = Trainer(a)
    mem_built = torch.cuda.memory_allocated() / 1e9 if torch.cuda.is_available() else 0.0
    rank = tr.rank
    dev = tr.device
    # ranks that really take part in the backend's collectives: an 8-byte all-reduce of ones
    ranks_seen = torch.ones(1, dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(ranks_seen)
    ranks_seen = int(ranks_seen.item())
    if args.slice:
        ranks_seen = 1  # loopback: this process is the only rank that exists
    elif ranks_seen != world:
        raise SystemExit(f"all-reduce saw {ranks_seen} ranks, WORLD_SIZE={world}")

    def sync():
        if dist.is_initialized():
            dist.barrier(device_ids=[dev.index]) if dev.type == "cuda" else dist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        loss = tr.train_step()
    sync()
    if tr.gemm_tuning == "tune":  # tuned in the warm-up (a tuning run's timing is not a result)
        from scaletorch_amd.utils import gemm_tuning

        if rank == 0:
            gemm_tuning.finish()
    from scaletorch_amd.dist import trace as comm_trace

    comm0 = comm_trace.stats()  # host-side counters only (a dict increment per collective)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = tr.train_step()
    sync()
    elapsed = time.perf_counter() - t0
    from scaletorch_amd.utils.misc import comm_per_step

    comm = {op: round(v["bytes"] / 1e6, 1) for op, v in
            sorted(comm_per_step(comm0, comm_trace.stats(), args.steps).items())}
    # max over ranks
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    final_loss = tr.reduced_loss(loss)
    tr.health_check()
    moe_info = None
    if tr.model_config.is_moe:  # EP dispatch counters of the last step (device values, read after the timing)
        layers = [m for m in tr.raw_model.modules() if getattr(m, "dropped_rows", None) is not None]
        sent = [m.ep_rows_sent for m in layers if getattr(m, "ep_rows_sent", None) is not None]
        from scaletorch_amd.models.moe import EP_TRANSPORT

        moe_info = {"capacity_factor": args.moe_capacity_factor, "ep_chunks": args.moe_ep_chunks,
                    "dispatch": "capacity" if args.moe_capacity_factor > 0 else "dropless",
                    "dropped_rows_last_step": int(sum(int(m.dropped_rows) for m in layers)) if layers else 0,
                    "rows_sent_off_rank_last_micro_batch": int(sum(int(x) for x in sent)) if sent else None,
                    "ep_transport": dict(EP_TRANSPORT) if args.ep > 1 else None}
    tokens_per_step = tr.tokens_per_step  # global: dp*ep*mbs*ga*seq
    tok_s = tokens_per_step * args.steps / elapsed
    cfg = tr.model_config
    n_params = cfg.active_params()
    fpt = flops_per_token(n_params, cfg.num_hidden_layers, cfg.num_attention_heads, cfg.head_dim, args.seq_len)
    fpt_causal = flops_per_token(n_params, cfg.num_hidden_layers, cfg.num_attention_heads, cfg.head_dim,
                                 args.seq_len, causal=True)
    # strict: GEMM parameters only (no input-embedding gather) and causal attention FLOPs
    fpt_strict = flops_per_token(cfg.matmul_params(), cfg.num_hidden_layers, cfg.num_attention_heads, cfg.head_dim,
                                 args.seq_len, causal=True)
    peak = get_theoretical_flops()
    per_gpu = tok_s / world
    mfu = per_gpu * fpt / peak * 100
    par = "".join(f"{k}{v}" for k, v in (("dp", dp), ("tp", args.tp), ("pp", args.pp), ("cp", args.cp),
                                         ("ep", args.ep)) if v > 1 or k == "dp")
    valid = args.layers is None
    names = {"llama3-8b": "Llama-3-8B", "mixtral-8x7b": "Mixtral-8x7B"}
    out = {
        "metric": f"tokens/sec ({names.get(args.model, args.model)} training, full step)",
        "value": round(tok_s, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1000, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(per_gpu / BASELINE_TOK_S_PER_GPU, 3),
        "dtype": "bf16",
        "data": "synthetic (random tokens), random-init weights",
        "config": {"model": args.model, "global_batch": dp * args.ep * args.micro_batch_size * ga,
                   "micro_batch": args.micro_batch_size, "grad_accum": ga, "seq_len": args.seq_len,
                   "parallelism": par, "layout": args.layout, "sequence_parallel": args.sp, "activation_checkpointing": args.gc,
                   "virtual_pipeline": args.vpp if args.pp > 1 else 1, "layer_distribution": args.layer_distribution,
                   "lm_head": f"fused, {args.head_chunk}-token chunks" if args.fused_head else "logits + CE",
                   "grad_reduce_dtype": args.grad_reduce_dtype, "zero_stage": args.zero if dp * args.cp * args.ep > 1 else 0,
                   "optimizer": f"AdamW, fp32 master, {args.opt_state_dtype} moments",
                   "gemm_tuning": tr.gemm_tuning},
        "tokens_per_s_per_gpu": round(per_gpu, 1),
        "mfu_pct": round(mfu, 2),
        "mfu_pct_causal_flops": round(per_gpu * fpt_causal / peak * 100, 2),
        "mfu_pct_strict": round(per_gpu * fpt_strict / peak * 100, 2),
        "mfu_basis": "mfu_pct: 6N + 12LHdS per token, N incl. the input embedding (reference misc.py:136-174); "
                     "mfu_pct_strict: N without the input-embedding gather, causal attention (6LHdS)",
        "peak_flops": peak,
        "baseline_tok_s_per_gpu": BASELINE_TOK_S_PER_GPU,
        "vs_baseline_basis": "context only: per-GPU tok/s over the reference's Qwen3-8B TP2-DP4 S2048 row on "
                             "8x Ascend 910B (README.md:84); BASELINE.json publishes no MI355X/Llama-3-8B number",
        "final_loss": round(final_loss, 4),
        "valid": valid,
        "max_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1) if dev.type == "cuda" else 0.0,
        "comm_mb_per_step_rank0": comm,  # bytes handed to each collective per step on rank 0 (dist/trace.py)
        "moe_dispatch": moe_info,
        "tp_transport": _tp_transport() if args.tp > 1 else None,
        "dist_world_size": dist.get_world_size() if dist.is_initialized() else 1,
        "backend": (("rccl" if a.backend == "nccl" else a.backend) if dist.is_initialized() else "none"),
        "collective_ranks_seen": ranks_seen,
        "launcher": "bench.py self-launch" if os.environ.get("ST_BENCH_SELF_LAUNCHED") else
                    ("torchrun" if launched else "single process"),
    }
    if args.slice:
        out = _slice_record(out, args, est, est_run, tr, dp, world, elapsed)
        # where the bytes sit: after the build (weights, grads, buffers) and between steps
        # (+ optimizer state), against the estimate's resident terms -- the rest of the peak is
        # the step's activations and workspaces
        out["hbm_after_build_gb"] = round(mem_built, 2)
        out["hbm_resident_between_steps_gb"] = round(
            torch.cuda.memory_allocated() / 1e9 if torch.cuda.is_available() else 0.0, 2)
        out["hbm_estimate_resident_gb"] = round(est.params_gb + est.grads_gb + est.optimizer_gb + est.comm_gb, 2)
    if rank == 0 or args.slice:
        print(json.dumps(out), flush=True)
        if os.environ.get("ST_WGRAD_TUNE_LOG") == "1":  # the per-shape weight-gradient picks (stderr)
            from scaletorch_amd.ops import grad as G

            for k, v in G._WGRAD_TIMES.items():
                print("wgrad tune", k[0], k[2], {a: round(b, 3) for a, b in v.items()}, "->", G._WGRAD_CHOICE.get(k),
                      file=sys.stderr, flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

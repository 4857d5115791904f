"""Trainer: builds mesh / model / arenas / optimizer / data and runs training steps.

Reference flow: tools/train.py:55-418 + scaletorch/trainer/{dist_setup,model_builder,train_step}.py.
Build order here: dist init -> mesh -> seed -> model built sharded on the
meta-free path directly in bf16 on the GPU -> TP tags -> DataParallel arenas
(flat bf16 params, fp32 main_grad) -> arena optimizer -> LR schedule -> data.

One training step (non-PP):
  for each micro-batch: forward -> vocab-parallel CE (+ MoE aux loss) -> backward
  (DP buckets all-reduce asynchronously during the LAST micro-batch's backward)
  -> global grad-norm (device) -> fused AdamW (clip coefficient read on device)
  -> LR schedule.  Losses stay on device; ``.item()`` happens only when logging.
"""
from __future__ import annotations

import contextlib
import logging
import math
import os
import time

import torch

from .. import ops
from ..data.loader import DeviceSyntheticLoader, MicroBatchDataLoader, SyntheticTokenDataset
from ..dist import collectives as C
from ..dist.launch import init_dist
from ..models import build_model, get_model_config
from ..optim import create_optimizer
from ..parallel import mesh
from ..parallel.data_parallel import DataParallel, mark_tp_sharded
from ..parallel.pipeline_parallel import PipelineEngine
from ..utils import profiling
from ..utils.misc import set_all_seed
from .lr_scheduler import create_lr_scheduler

logger = logging.getLogger(__name__)

_DTYPES = {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float16": torch.float16, "fp16": torch.float16,
           "float32": torch.float32, "fp32": torch.float32}


_COMPUTE_STREAMS: dict = {}
# ST_DEBUG_FINITE=1: name the parameters whose gradient (before clipping) or value (after the
# update) holds a non-finite element, and print the clipped-over grad norm -- host syncs, debug only
_DEBUG_FINITE = os.environ.get("ST_DEBUG_FINITE", "0") == "1"


def _report_nonfinite(model, what: str, step: int) -> None:
    bad = []
    for name, p in model.named_parameters():
        t = p.grad if what == "grad" else p
        if t is not None and t.numel() and not bool(torch.isfinite(t).all()):
            bad.append(f"{name}({int((~torch.isfinite(t)).sum())})")
    r = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
    print(f"[finite] step {step} rank {r} non-finite {what}s: {len(bad)} {bad[:6]}", flush=True)


class Trainer:
    def __init__(self, args, device_data: bool | None = None, build_data: bool = True):
        self.args = args
        a = args
        self.rank, self.local_rank, self.world = init_dist(backend=a.backend, use_cpu=a.use_cpu, timeout_s=a.timeout_s)
        a.validate_world_size(self.world)
        if self.world > 1:
            mesh.setup_process_group_manager(a.tensor_parallel_size, a.context_parallel_size,
                                             a.pipeline_parallel_size, a.data_parallel_size, a.expert_parallel_size)
            if a.debug_collectives:
                from ..dist import debug

                debug.enable(timeout_s=a.timeout_s)
        if a.tensor_parallel_size > 1:
            from ..parallel.tensor_parallel import select_tp_transport, set_tp_comm

            if torch.cuda.is_available() and not a.use_cpu and (a.backend == "nccl" or a.tp_comm == "xgmi"
                                                                 or os.environ.get("ST_GPU_OVERSUBSCRIBE") == "1"):
                # collective over the world, before any model code: "auto" self-tests the
                # 7-link pair path for tp = 2 against RCCL and keeps the faster correct one
                msg = None
                if a.micro_batch_size and a.sequence_length:
                    # the row-parallel all-reduce / SP reduce-scatter input: [mbs, S/cp, h] bf16
                    h = get_model_config(a.model_name_or_path).hidden_size
                    msg = a.micro_batch_size * (a.sequence_length // max(1, a.context_parallel_size)) * h * 2
                select_tp_transport(mesh.tp_group(), a.tp_comm, msg_bytes=msg)
            else:
                set_tp_comm("rccl" if a.tp_comm == "auto" else a.tp_comm)
        from ..models.attention_backends import set_use_flash_attention
        from ..models.moe import set_moe_dispatch

        set_moe_dispatch(a.moe_capacity_factor, a.moe_ep_chunks, "rccl" if a.ep_comm == "auto" else a.ep_comm)
        if a.expert_parallel_size > 1 and a.sequence_length and a.micro_batch_size:
            from ..models.moe import set_ep_token_bound

            # every micro-batch holds exactly this many tokens per rank (loaders drop ragged
            # tails), so the EP exchange buffers need no per-call agreement
            set_ep_token_bound(a.micro_batch_size * a.sequence_length // max(1, a.context_parallel_size))
        if a.expert_parallel_size > 1 and torch.cuda.is_available() and not a.use_cpu and a.ep_comm != "rccl" \
                and (a.backend == "nccl" or os.environ.get("ST_GPU_OVERSUBSCRIBE", "0") == "1"):
            from ..models.moe import select_ep_transport

            # collective over each EP group, at start-up: "auto" self-tests the xGMI push
            # exchange (dropless, device counts) against RCCL and keeps it when it matches
            area = None
            if a.sequence_length and a.micro_batch_size:
                mc = get_model_config(a.model_name_or_path)
                if mc.is_moe:
                    from ..models.moe import ep_area_bytes

                    area = ep_area_bytes(a.micro_batch_size * a.sequence_length // max(1, a.context_parallel_size),
                                         a.expert_parallel_size, mc.num_experts_per_tok, mc.num_experts,
                                         mc.hidden_size, a.moe_capacity_factor)
            select_ep_transport(mesh.pgm.ep_group, a.ep_comm, area_bytes=area)

        set_use_flash_attention(a.use_flash_attention)
        if a.context_parallel_size > 1:
            from ..parallel.context_parallel import set_cp_comm, set_cp_zigzag

            set_cp_zigzag(a.cp_zigzag)
            set_cp_comm(a.cp_comm)
        self.device = torch.device("cuda", torch.cuda.current_device()) if (torch.cuda.is_available() and not a.use_cpu) \
            else torch.device("cpu")
        if self.device.type == "cuda":
            from ..utils.gemm_tuning import configure as _tune_gemms

            self.gemm_tuning = _tune_gemms(a.gemm_tuning)
        else:
            self.gemm_tuning = "off"
        self.dtype = _DTYPES[a.dtype]
        if self.device.type == "cpu" and self.dtype == torch.float16:
            self.dtype = torch.float32
        set_all_seed(a.seed)
        from ..parallel.init import set_init_seed

        set_init_seed(a.seed)
        overrides = dict(num_hidden_layers=a.num_hidden_layers, num_attention_heads=a.num_attention_heads,
                         num_key_value_heads=a.num_key_value_heads)
        self.model_config = get_model_config(a.model_name_or_path, **overrides)
        cfg = self.model_config
        if a.sequence_length and a.sequence_length > cfg.max_position_embeddings:
            cfg.max_position_embeddings = a.sequence_length
        dist_ = [int(x) for x in a.layer_distribution.split(",")] if a.layer_distribution else None
        # build directly on the target device in the compute dtype (no meta/CPU materialisation)
        with torch.device(self.device):
            prev = torch.get_default_dtype()
            torch.set_default_dtype(self.dtype if self.dtype.is_floating_point else torch.float32)
            try:
                model = build_model(cfg, sequence_parallel=a.sequence_parallel, layer_distribution=dist_,
                                    virtual_stages=a.virtual_pipeline_size)
            finally:
                torch.set_default_dtype(prev)
        model.cos, model.sin = model.cos.float(), model.sin.float()
        # HF safetensors (single file or sharded index) when model_name_or_path holds them:
        # loaded before the DP arena / optimizer exist, so the arena and the fp32 masters
        # are built from the loaded weights (reference model_builder.py:82-84)
        from ..utils.checkpoint import maybe_load_hf_weights

        self.hf_tensors_loaded = maybe_load_hf_weights(model, a.model_name_or_path, getattr(a, "hf_weights", "auto"))
        mark_tp_sharded(model)
        self.raw_model = model
        bucket = max(1, int(a.bucket_size_mb * 1024 * 1024) // 4)
        self.model = DataParallel(model, bucket_size=bucket, reduce_dtype=a.grad_reduce_dtype,
                                  zero1=a.zero_stage >= 1)
        self.optimizer = create_optimizer(self.model, a.optimizer_type, a.learning_rate, a.weight_decay,
                                          a.betas, a.adam_eps, a.use_fused_adam,
                                          state_dtype=a.optimizer_state_dtype)
        self.total_steps = a.total_train_steps or 1000
        self.lr_scheduler = create_lr_scheduler(self.optimizer, a.lr_scheduler_type, self.total_steps,
                                                a.warmup_steps, a.T_max, a.eta_min, a.power, a.step_size, a.gamma,
                                                a.max_lr, a.pct_start)
        pg = mesh.pgm
        self.tp_group = pg.tp_group if pg else None
        self.mp_group = pg.mp_group if pg else None
        self.pp = pg.pp_world_size if pg else 1
        self.cp = pg.cp_world_size if pg else 1
        self.cp_rank = pg.cp_rank if pg else 0
        self.tokens_per_step = a.global_batch_size * (a.sequence_length or 0)
        # activation checkpointing mode handed to the model: False | "full" | "selective"
        self.gc_mode = (a.recompute_granularity if a.recompute_granularity in ("full", "selective") else "full") \
            if a.gradient_checkpointing else False
        self.step = 0
        self.trained_tokens = 0
        self.data = None
        if build_data:
            self.data = self._build_data(device_data if device_data is not None else a.synthetic_data)
        if self.pp > 1:
            S = a.sequence_length // self.cp
            if a.sequence_parallel and mesh.tp_size() > 1:
                S //= mesh.tp_size()
            self.pipeline = PipelineEngine(self.model, self._loss, (a.micro_batch_size, S, cfg.hidden_size),
                                           dtype=self.dtype, device=self.device,
                                           gradient_checkpointing=self.gc_mode,
                                           aux_loss_fn=model.aux_loss if cfg.is_moe else None,
                                           head_kwargs_fn=self._head_kwargs,
                                           virtual_stages=a.virtual_pipeline_size)

    # ---------------------------------------------------------------- data
    def _build_data(self, synthetic: bool):
        a, pg = self.args, mesh.pgm
        data_rank = pg.data_rank if pg else 0
        data_world = pg.data_world_size if pg else 1
        if synthetic and self.device.type == "cuda":
            return DeviceSyntheticLoader(self.model_config.vocab_size, a.micro_batch_size, a.sequence_length,
                                         self.device, a.gradient_accumulation_steps, self.cp, self.cp_rank,
                                         a.cp_zigzag, seed=a.seed, data_rank=data_rank)
        if synthetic:
            ds = SyntheticTokenDataset(self.model_config.vocab_size, a.sequence_length, seed=a.seed)
        else:
            from ..data.dataset import build_dataset

            ds = build_dataset(a, a.sequence_length)
        return MicroBatchDataLoader(ds, a.micro_batch_size, a.sequence_length, a.gradient_accumulation_steps,
                                    data_rank, data_world, self.cp_rank, self.cp, a.cp_zigzag, seed=a.seed,
                                    num_workers=0 if synthetic else a.num_workers,
                                    pin_memory=a.pin_memory and self.device.type == "cuda")

    def _to_device(self, batch: dict) -> dict:
        out = {}
        for k, v in batch.items():
            out[k] = v.to(self.device, non_blocking=True) if isinstance(v, torch.Tensor) else v
        return out

    # ---------------------------------------------------------------- loss
    def _head_kwargs(self, batch: dict) -> dict:
        """Model kwargs that make the last stage return the fused head's loss."""
        a = self.args
        if not getattr(a, "fused_lm_head", False):
            return {}
        # the loss is divided by the micro-batch count before backward, so that is the
        # head's upstream gradient: its weight gradient goes straight into main_grad
        return {"labels": batch["target_ids"], "lm_head_chunk": a.lm_head_chunk_tokens,
                "lm_head_grad_scale": 1.0 / a.gradient_accumulation_steps}

    def _loss(self, logits: torch.Tensor, batch: dict) -> torch.Tensor:
        if logits.dim() == 0:  # the fused LM head already produced the loss
            return logits
        tgt = batch["target_ids"].to(logits.device)
        group = self.tp_group if mesh.tp_size() > 1 else None
        return ops.cross_entropy(logits, tgt, vocab_start=self.raw_model.vocab_start, group=group)

    # ---------------------------------------------------------------- step
    def train_step(self) -> torch.Tensor:
        """One optimizer step; returns the mean loss as a DEVICE tensor.

        ``ST_COMPUTE_STREAM_PRIORITY`` < 0 runs the step on a high-priority HIP
        stream, so the side streams (optimizer update, W^T copies) -- default
        priority -- are dispatched behind the forward/backward kernels they
        overlap.  The caller's stream waits for it before the loss is returned."""
        prio = int(os.environ.get("ST_COMPUTE_STREAM_PRIORITY", "0")) if self.device.type == "cuda" else 0
        if prio == 0:
            return self._train_step()
        key = (self.device.index, prio)
        st = _COMPUTE_STREAMS.get(key)
        if st is None:
            st = _COMPUTE_STREAMS[key] = torch.cuda.Stream(device=self.device, priority=prio)
        caller = torch.cuda.current_stream(self.device)
        st.wait_stream(caller)
        with torch.cuda.stream(st):
            loss = self._train_step()
        caller.wait_stream(st)
        return loss

    def _train_step(self) -> torch.Tensor:
        a = self.args
        ga = a.gradient_accumulation_steps
        self.optimizer.zero_grad()
        if self.pp > 1:
            it = (self._to_device(next(self.data)) for _ in iter(int, 1))
            eng = self.pipeline
            if a.virtual_pipeline_size > 1:
                loss = eng.train_step_interleaved(it, ga)
            elif a.pipeline_parallel_engine == "1f1b":
                loss = eng.train_step_1f1b(it, ga)
            else:
                loss = eng.train_step_afab(it, ga)
        else:
            loss = torch.zeros((), dtype=torch.float32, device=self.device)
            for i in range(ga):
                batch = self._to_device(next(self.data))
                ctx = self.model.no_sync() if i < ga - 1 else contextlib.nullcontext()
                with ctx:
                    with profiling.range("forward"):
                        logits = self.model(input_ids=batch["input_ids"], position_ids=batch["position_ids"],
                                            gradient_checkpointing=self.gc_mode, **self._head_kwargs(batch))
                        l = self._loss(logits, batch) / ga
                        del logits
                        if self.model_config.is_moe:
                            aux = self.raw_model.aux_loss()
                            if aux is not None:
                                l = l + aux / ga
                    with profiling.range("backward"):
                        l.backward()
                loss += l.detach().float()
        with profiling.range("optimizer"):
            if _DEBUG_FINITE:
                _report_nonfinite(self.raw_model, "grad", self.step)
            gn = self.optimizer.clip_grad_norm_(a.max_grad_norm, self.mp_group)
            if _DEBUG_FINITE:
                print(f"[finite] step {self.step} rank {self.rank} grad norm {float(gn) if gn is not None else None}",
                      flush=True)
            self.optimizer.step()
            if _DEBUG_FINITE:
                _report_nonfinite(self.raw_model, "param", self.step)
        self.lr_scheduler.step()
        self.step += 1
        self.trained_tokens += self.tokens_per_step
        return loss

    @torch.no_grad()
    def evaluate(self, num_sequences: int | None = None) -> float:
        """Mean held-out loss over ``num_sequences`` (default ``--test_batch_size``)
        sequences, sharded over the data-parallel replicas, forward only, in
        micro-batches of ``--micro_batch_size``.  The held-out stream is a separate
        synthetic stream (seed + 1) or the dataset's ``validation`` split."""
        a = self.args
        if self.pp > 1:
            raise NotImplementedError("evaluation with pipeline parallelism is not supported; use pp = 1")
        n = num_sequences or a.test_batch_size
        pg = mesh.pgm
        data_world = pg.data_world_size if pg else 1
        per_rank = max(1, n // data_world)
        steps = max(1, per_rank // a.micro_batch_size)
        loader = getattr(self, "_eval_data", None)
        if loader is None:
            loader = self._eval_data = self._build_eval_data()
        was_training = self.raw_model.training
        self.raw_model.eval()
        total = torch.zeros((), dtype=torch.float32, device=self.device)
        try:
            for _ in range(steps):
                batch = self._to_device(next(loader))
                logits = self.model(input_ids=batch["input_ids"], position_ids=batch["position_ids"],
                                    **self._head_kwargs(batch))
                total += self._loss(logits, batch).float()
        finally:
            self.raw_model.train(was_training)
        return self.reduced_loss(total / steps)

    def _build_eval_data(self):
        a, pg = self.args, mesh.pgm
        data_rank = pg.data_rank if pg else 0
        data_world = pg.data_world_size if pg else 1
        if a.synthetic_data or a.use_cpu and not a.dataset_name:
            ds = SyntheticTokenDataset(self.model_config.vocab_size, a.sequence_length, seed=a.seed + 1)
        else:
            from ..data.dataset import build_dataset

            import copy

            b = copy.copy(a)
            b.split = "validation"
            ds = build_dataset(b, a.sequence_length)
        return MicroBatchDataLoader(ds, a.micro_batch_size, a.sequence_length, 1, data_rank, data_world,
                                    self.cp_rank, self.cp, a.cp_zigzag, shuffle=False, seed=a.seed)

    def resume(self, ckpt_manager, path: str) -> None:
        """Load a checkpoint on EVERY rank or fail on every rank: a rank that could not
        load (missing shard, bad file) must not continue from step 0 while its peers
        resume at step N (different LR schedule / step counts -> hang or divergence).
        The data loaders are advanced past the consumed micro-batches."""
        ok, err = 1, None
        try:
            self.step, self.trained_tokens = ckpt_manager.load_checkpoint(self.model, self.optimizer, path,
                                                                          self.lr_scheduler)
        except Exception as e:  # noqa: BLE001 -- any local failure (corrupt/truncated file, unpickling,
            ok, err = 0, e      # permissions) must reach the collective below, or the peers hang in it
        flag = torch.tensor([ok], dtype=torch.int32, device=self.device if C.get_world_size() > 1 else "cpu")
        if C.get_world_size() > 1:
            C.all_reduce(flag, op="min")
        if int(flag.item()) != 1:
            raise RuntimeError(f"resume from {path} failed on at least one rank"
                               + (f" (this rank: {err})" if err is not None else ""))
        if self.data is not None and hasattr(self.data, "skip_batches"):
            self.data.skip_batches(self.step * self.args.gradient_accumulation_steps)

    def health_check(self) -> None:
        """Raise if a custom xGMI collective timed out since the last check (its
        outputs are invalid); called at logging steps by tools/train.py and at the
        end of bench.py so the job exits non-zero instead of training on garbage."""
        from ..parallel.tensor_parallel import TRANSPORT

        if TRANSPORT["tp"] == "xgmi":
            from ..parallel.tensor_parallel import check_xgmi

            check_xgmi()
        from ..models.moe import check_ep_xgmi

        check_ep_xgmi()
        if getattr(self.args, "fused_lm_head", False):
            from ..ops.fused_head import check_grad_scale

            check_grad_scale()

    def reduced_loss(self, loss: torch.Tensor) -> float:
        """Mean loss over data-parallel replicas (last PP stage holds it); host sync."""
        pg = mesh.pgm
        t = loss.detach().float().clone().reshape(1)
        if pg:
            if pg.pp_world_size > 1:
                C.all_reduce(t, group=pg.pp_group)  # only the last stage is non-zero
            C.all_reduce(t, op="mean", group=pg.dense_dp_group)
        return float(t.item())

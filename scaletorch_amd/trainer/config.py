"""Training configuration / CLI.

Same flag names and defaults as the reference ``ScaleTorchArguments``
(scaletorch/trainer/config.py:31-461) so existing launch scripts work; the
reference's env toggles (FLASH_ATTEN, CONTEXT_PARALLEL, SEQUENCE_PARALLEL, DTYPE)
are CLI flags here, read once.  Flags the reference parsed but ignored
 are wired up: ``use_flash_attention`` selects the flash or sdpa
attention backend (models/attention_backends.py), ``epochs`` bounds training by
data passes, ``test_batch_size`` is the number of held-out sequences per
evaluation (``eval_interval``), ``dtype``/``backend``/``pin_memory``/
``log_interval``/``save_model_checkpoint`` are read by the trainer and
tools/train.py.  Extra MI355X-side flags are grouped in ``SystemArguments``.
"""
from __future__ import annotations

import dataclasses
import json
import logging
from dataclasses import dataclass, field

logger = logging.getLogger(__name__)

_VALID_LR_SCHEDULERS = {"linear", "cosine", "polynomial", "step", "onecycle", "constant"}
_VALID_OPTIMIZERS = {"adamw", "adam", "sgd", "lamb"}


@dataclass
class DataArguments:
    data_path: str = field(default="./data", metadata={"help": "local dataset dir / file"})
    dataset_name: str = field(default="wikitext2", metadata={"help": "dataset name (local only, no hub access)"})
    tokenizer_name_or_path: str = field(default="facebook/opt-125m", metadata={"help": "local tokenizer path"})
    subset_name: str | None = field(default=None)
    split: str = field(default="train")
    num_proc: int = field(default=1)
    num_workers: int = field(default=2)
    num_samples: int | None = field(default=None)
    pin_memory: bool = field(default=True)
    synthetic_data: bool = field(default=False, metadata={"help": "random tokens, no dataset/tokenizer needed"})


@dataclass
class ModelArguments:
    model_name_or_path: str = field(default="facebook/opt-125m",
                                    metadata={"help": "registry name (llama3-8b, qwen3-8b, mixtral-8x7b, ...) "
                                                      "or local HF config dir"})
    num_hidden_layers: int | None = field(default=None)
    num_attention_heads: int | None = field(default=None)
    num_key_value_heads: int | None = field(default=None)
    use_flash_attention: bool = field(default=True)
    dtype: str = field(default="bfloat16")
    hf_weights: str = field(default="auto",
                            metadata={"help": "auto: load *.safetensors when model_name_or_path is a dir holding "
                                              "them (reference model_builder.py:82-84) | required: fail without "
                                              "them | off: random init"})


@dataclass
class ParallelArguments:
    tensor_parallel_size: int = field(default=1)
    pipeline_parallel_size: int = field(default=1)
    data_parallel_size: int = field(default=1)
    context_parallel_size: int = field(default=1)
    expert_parallel_size: int = field(default=1)
    pipeline_parallel_engine: str = field(default="1f1b", metadata={"help": "1f1b | afab"})
    virtual_pipeline_size: int = field(default=1, metadata={"help": "model chunks per pipeline rank: > 1 runs the "
                                                                      "interleaved 1F1B schedule (needs 1f1b and "
                                                                      "gradient_accumulation_steps % pp == 0)"})
    backend: str = field(default="nccl", metadata={"help": "nccl (=RCCL) | gloo | hccl (maps to nccl) | loopback "
                                                           "(one rank of a layout on one GPU, dist/loopback.py)"})
    sequence_parallel: bool = field(default=False, metadata={"help": "Megatron-SP over the TP group"})
    cp_zigzag: bool = field(default=True, metadata={"help": "zig-zag load-balanced CP chunks"})
    tp_comm: str = field(default="auto", metadata={"help": "TP transport: auto (one node: tp = 2 self-tests the 7-link xGMI pair path, tp 4 / 8 the TP-group communicator's all-reduce / all-gather / reduce-scatter at the run's real message size, each against RCCL at start-up, keeping every collective that is correct and faster) | rccl | xgmi (custom one-/two-shot all-reduce + all-gather / reduce-scatter over IPC peer memory, dist/xgmi.py)"})
    cp_comm: str = field(default="auto", metadata={"help": "CP transport: auto (= allgather: RCCL drives all 7 xGMI links) | allgather (overlapped K/V all-gather) | ring (p2p rotation overlapped with block compute) | ulysses (head all-to-all)"})
    layer_distribution: str | None = field(default=None, metadata={"help": "comma list of layers per PP stage"})
    moe_capacity_factor: float = field(default=0.0, metadata={
        "help": "EP dispatch: 0 = dropless (exchange buffers sized by the worst case ep*T*min(k, E/ep) rows, "
                "routing counts stay on the device; over xGMI no host sync at all, over RCCL one host read "
                "of the count matrix per layer for the splits); > 0 = static per-(source, destination) "
                "capacity ceil(f * T * k / ep) rows: rows past it are dropped (counted in dropped_rows)"})
    ep_comm: str = field(default="auto", metadata={
        "help": "EP transport: auto (one node: self-test the xGMI push exchange against RCCL at start-up and "
                "keep it when it matches) | rccl | xgmi (push into IPC peer memory, dist/xgmi.py)"})
    moe_ep_chunks: int = field(default=1, metadata={
        "help": "EP dispatch pipelining (capacity mode): the tokens are dispatched in this many chunks, each "
                "chunk's all-to-all overlapping the previous chunk's expert GEMMs"})

    def __post_init__(self) -> None:
        for name in ("data_parallel_size", "tensor_parallel_size", "pipeline_parallel_size",
                     "context_parallel_size", "expert_parallel_size"):
            if getattr(self, name) < 1:
                raise ValueError(f"{name} must be >= 1, got {getattr(self, name)}")
        if self.pipeline_parallel_engine not in {"1f1b", "afab"}:
            raise ValueError(f'pipeline_parallel_engine must be "1f1b" or "afab", got {self.pipeline_parallel_engine}')
        if self.virtual_pipeline_size < 1:
            raise ValueError("virtual_pipeline_size must be >= 1")
        if self.virtual_pipeline_size > 1:
            if self.pipeline_parallel_size < 2 or self.pipeline_parallel_engine != "1f1b":
                raise ValueError("virtual_pipeline_size > 1 needs pipeline_parallel_size > 1 and the 1f1b engine")
            if getattr(self, "gradient_accumulation_steps", 1) % self.pipeline_parallel_size:
                raise ValueError("interleaved 1F1B needs gradient_accumulation_steps divisible by "
                                 "pipeline_parallel_size")
        if self.tp_comm not in {"auto", "rccl", "xgmi"}:
            raise ValueError(f"tp_comm must be auto, rccl or xgmi, got {self.tp_comm}")
        if self.ep_comm not in {"auto", "rccl", "xgmi"}:
            raise ValueError(f"ep_comm must be auto, rccl or xgmi, got {self.ep_comm}")
        if self.moe_capacity_factor < 0 or self.moe_ep_chunks < 1:
            raise ValueError("moe_capacity_factor must be >= 0 and moe_ep_chunks >= 1")
        if self.backend not in {"nccl", "gloo", "hccl", "loopback"}:
            raise ValueError(f"backend must be one of {{nccl, gloo, hccl, loopback}}, got {self.backend}")


@dataclass
class LrSchedulerArguments:
    lr_scheduler_type: str = field(default="linear")
    warmup_steps: int = field(default=0)
    T_max: int | None = field(default=None)
    eta_min: float = field(default=0.0)
    power: float = field(default=1.0)
    step_size: int = field(default=1)
    gamma: float = field(default=0.1)
    max_lr: float | None = field(default=None)
    pct_start: float = field(default=0.3)

    def __post_init__(self) -> None:
        if self.lr_scheduler_type not in _VALID_LR_SCHEDULERS:
            raise ValueError(f"lr_scheduler_type must be one of {sorted(_VALID_LR_SCHEDULERS)}, got {self.lr_scheduler_type}")
        if self.warmup_steps < 0:
            raise ValueError(f"warmup_steps must be >= 0, got {self.warmup_steps}")
        t = self.lr_scheduler_type
        if t == "cosine" and self.eta_min < 0:
            raise ValueError(f"eta_min must be >= 0, got {self.eta_min}")
        if t == "polynomial" and self.power <= 0:
            raise ValueError(f"power must be > 0, got {self.power}")
        if t == "step":
            if self.step_size <= 0:
                raise ValueError(f"step_size must be > 0, got {self.step_size}")
            if not 0 < self.gamma <= 1:
                raise ValueError(f"gamma must be in (0, 1], got {self.gamma}")
        if t == "onecycle" and not 0 < self.pct_start < 1:
            raise ValueError(f"pct_start must be in (0, 1), got {self.pct_start}")


@dataclass
class OptimizerArguments:
    optimizer_type: str = field(default="adamw")
    weight_decay: float = field(default=0.0)
    use_fused_adam: bool = field(default=True)
    betas: list[float] = field(default_factory=lambda: [0.9, 0.999], metadata={"help": "two floats"})
    learning_rate: float = field(default=1e-3)
    adam_eps: float = field(default=1e-8)
    gemm_tuning: str = field(
        default="auto", metadata={"help": "library GEMM solutions (utils/gemm_tuning.py): auto | use | tune | off"})
    optimizer_state_dtype: str = field(
        default="fp32", metadata={"help": "AdamW exp_avg / exp_avg_sq dtype: fp32 | bf16 (the reference's own "
                                          "state precision; fp32 master weights are kept either way)"})

    def __post_init__(self) -> None:
        if self.optimizer_state_dtype not in ("fp32", "bf16"):
            raise ValueError(f"optimizer_state_dtype must be fp32 or bf16, got {self.optimizer_state_dtype!r}")
        if self.optimizer_type not in _VALID_OPTIMIZERS:
            raise ValueError(f"optimizer_type must be one of {sorted(_VALID_OPTIMIZERS)}, got {self.optimizer_type}")
        if self.learning_rate <= 0:
            raise ValueError(f"learning_rate must be > 0, got {self.learning_rate}")
        self.betas = tuple(self.betas)


@dataclass
class TrainingArguments:
    batch_size: int = field(default=64)
    test_batch_size: int = field(default=1000, metadata={"help": "held-out sequences per evaluation"})
    micro_batch_size: int | None = field(default=None)
    gradient_accumulation_steps: int = field(default=1)
    gradient_checkpointing: bool = field(default=False)
    recompute_granularity: str = field(default="full", metadata={"help": "with --gradient_checkpointing: full "
                                                                      "(whole layer) | selective (norm+MLP "
                                                                      "only; attention activations kept)"})
    fused_lm_head: bool = field(default=True, metadata={"help": "LM head + cross-entropy fused and chunked "
                                                                "(ops/fused_head.py): the [tokens, vocab] logits "
                                                                "are never materialised"})
    lm_head_chunk_tokens: int = field(default=4096, metadata={"help": "tokens per fused LM-head chunk"})
    max_grad_norm: float | None = field(default=1.0)
    epochs: int = field(default=5, metadata={"help": "stop after this many passes over the dataset"})
    seed: int = field(default=1)
    sequence_length: int | None = field(default=1024)
    log_interval: int = field(default=1)
    max_tokens: int | None = field(default=None)
    total_train_steps: int | None = field(default=None)
    use_cpu: bool = field(default=False)
    eval_interval: int = field(default=0, metadata={"help": "evaluate held-out loss every N steps (0 = off)"})

    def __post_init__(self) -> None:
        if self.gradient_accumulation_steps < 1:
            raise ValueError(f"gradient_accumulation_steps must be >= 1, got {self.gradient_accumulation_steps}")
        if self.micro_batch_size is not None and self.micro_batch_size < 1:
            raise ValueError(f"micro_batch_size must be >= 1, got {self.micro_batch_size}")
        if self.sequence_length is not None and self.sequence_length < 1:
            raise ValueError(f"sequence_length must be >= 1, got {self.sequence_length}")


@dataclass
class CheckpointArguments:
    work_dir: str = field(default="./work_dir")
    save_model_checkpoint: bool = field(default=True)
    save_frequency: int = field(default=300)
    resume_path: str = field(default="")
    auto_resume: bool = field(default=False, metadata={"help": "resume from the newest step dir in work_dir"})
    async_save: bool = field(default=True, metadata={"help": "write checkpoints from a background thread"})

    def __post_init__(self) -> None:
        if self.save_frequency < 0:
            raise ValueError(f"save_frequency must be >= 0, got {self.save_frequency}")


@dataclass
class LoggingArguments:
    use_wandb: bool = field(default=False)
    project_name: str = field(default="scaletorch")
    experiment_name: str | None = field(default=None)


@dataclass
class SystemArguments:
    grad_reduce_dtype: str = field(default="fp32", metadata={"help": "fp32 | bf16 gradient all-reduce"})
    bucket_size_mb: float = field(default=256, metadata={"help": "DP bucket size (MiB of fp32 gradient)"})
    zero_stage: int = field(default=0, metadata={"help": "0: replicated optimizer; 1: ZeRO-1 distributed "
                                                         "optimizer (reduce-scatter grads, sharded states, "
                                                         "all-gather params)"})
    profile: bool = field(default=False, metadata={"help": "torch.profiler trace of steps 3-5"})
    profile_dir: str = field(default="./profiles/trace")
    nan_check: bool = field(default=True, metadata={"help": "abort on non-finite loss"})
    timeout_s: int = field(default=600)
    watchdog_s: float = field(default=0.0, metadata={"help": "abort (exit 75, torchrun restarts + --auto_resume) "
                                                            "when a step makes no progress for this long; 0 = off"})
    debug_collectives: bool = field(default=False, metadata={"help": "cross-check collective order across ranks"})


@dataclass
class ScaleTorchArguments(DataArguments, ModelArguments, ParallelArguments, LrSchedulerArguments,
                          OptimizerArguments, TrainingArguments, CheckpointArguments, LoggingArguments,
                          SystemArguments):
    global_batch_size: int = field(init=False, default=0)
    global_batch_size_token: int | None = field(init=False, default=None)

    def __post_init__(self) -> None:
        ParallelArguments.__post_init__(self)
        LrSchedulerArguments.__post_init__(self)
        OptimizerArguments.__post_init__(self)
        TrainingArguments.__post_init__(self)
        CheckpointArguments.__post_init__(self)
        if self.micro_batch_size is None:
            self.micro_batch_size = self.batch_size
        if self.hf_weights not in ("auto", "required", "off"):
            raise ValueError(f"hf_weights must be auto, required or off, got {self.hf_weights!r}")
        cp = self.context_parallel_size
        if self.sequence_length and cp > 1:
            div = 2 * cp if self.cp_zigzag else cp
            if self.sequence_length % div:
                raise ValueError(f"sequence_length ({self.sequence_length}) must be divisible by {div} "
                                 f"(context_parallel_size={cp}, zigzag={self.cp_zigzag})")
        # EP ranks are data-parallel replicas (mesh.py)
        self.global_batch_size = (self.data_parallel_size * self.expert_parallel_size * self.micro_batch_size
                                  * self.gradient_accumulation_steps)
        if self.sequence_length is not None:
            self.global_batch_size_token = self.global_batch_size * self.sequence_length

    def validate_world_size(self, world_size: int) -> None:
        expected = (self.tensor_parallel_size * self.pipeline_parallel_size * self.data_parallel_size
                    * self.context_parallel_size * self.expert_parallel_size)
        if world_size != expected:
            raise ValueError(f"world_size ({world_size}) != TP({self.tensor_parallel_size}) * "
                             f"PP({self.pipeline_parallel_size}) * DP({self.data_parallel_size}) * "
                             f"CP({self.context_parallel_size}) * EP({self.expert_parallel_size}) = {expected}")

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), indent=2, default=str)


def parse_args(argv: list[str] | None = None) -> ScaleTorchArguments:
    from transformers import HfArgumentParser

    parser = HfArgumentParser(ScaleTorchArguments)
    (args,) = parser.parse_args_into_dataclasses(args=argv)
    return args

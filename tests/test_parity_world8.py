"""World-8 parity of the COMBINED layouts the 8-GPU benchmark runs (CPU / gloo).

Each case is one of BASELINE.json's 8-GPU configs scaled down to a tiny model
(or a layout that composes the same axes) and is compared against the
single-process run on the same global batch: loss and updated weights (TP
shards against slices of the full tensors, local experts against their global
index).  Reference layouts: scripts/benchmark_comprehensive.py:54-173 of the
reference (TP/PP/CP/DP mixes) and its 1F1B schedule
(scaletorch/parallel/pipeline_parallel/pipeline_parallel.py:457-671).
"""
from __future__ import annotations

import pytest

from tests.dist_harness import run_workers
from tests.test_parallel_parity import _ADAM, _compare, _compare_moe, _reference, _worker

pytestmark = pytest.mark.slow

GB = 8  # global batch (rows of SEQ+1 tokens): divisible by every data-parallel width used here


@pytest.mark.parametrize("kw", [
    dict(data_parallel_size=8, micro_batch_size=1, zero_stage=1),
    dict(data_parallel_size=8, micro_batch_size=1, zero_stage=1, bucket_size_mb=0.05, grad_reduce_dtype="fp32"),
], ids=["dp8_zero1", "dp8_zero1_buckets"])
def test_dp8_zero1(kw):
    ref = _reference("tiny-llama", 1, GB, **_ADAM)
    res = run_workers(_worker, 8, "tiny-llama", dict(kw, global_b=GB, **_ADAM))
    _compare(ref, res, atol=5e-5, rtol=5e-3)


_TPPPDP = dict(tensor_parallel_size=2, pipeline_parallel_size=2, data_parallel_size=2, micro_batch_size=1,
               gradient_accumulation_steps=4, global_b=GB)


@pytest.mark.parametrize("kw", [
    dict(),
    dict(sequence_parallel=True),
    dict(pipeline_parallel_engine="afab"),
], ids=["tp2_pp2_dp2_1f1b", "tp2_pp2_dp2_1f1b_sp", "tp2_pp2_dp2_afab"])
def test_tp2_pp2_dp2(kw):
    ref = _reference("tiny-llama", 4, GB)
    res = run_workers(_worker, 8, "tiny-llama", dict(_TPPPDP, **kw))
    _compare(ref, res)


def test_tp2_pp2_dp2_zero1_adamw():
    ref = _reference("tiny-llama", 4, GB, **_ADAM)
    res = run_workers(_worker, 8, "tiny-llama", dict(_TPPPDP, sequence_parallel=True, zero_stage=1, **_ADAM))
    _compare(ref, res, atol=5e-5, rtol=5e-3)


def test_tp2_pp2_dp2_interleaved_zero1_adamw():
    """Interleaved 1F1B (2 chunks per pipeline rank, 4 layers) with SP and ZeRO-1 over
    2 AdamW steps equals the single-process run."""
    ref = _reference("tiny-llama", 4, GB, num_hidden_layers=4, **_ADAM)
    res = run_workers(_worker, 8, "tiny-llama", dict(_TPPPDP, sequence_parallel=True, zero_stage=1,
                                                     virtual_pipeline_size=2, num_hidden_layers=4, **_ADAM))
    _compare(ref, res, atol=5e-5, rtol=5e-3)


@pytest.mark.parametrize("comm", ["allgather", "ring"])
def test_cp8(comm):
    """cp=8 (zig-zag: 16 chunks of 2 tokens) with the GQA-sized K/V transports."""
    ref = _reference("tiny-llama", 1, GB)
    res = run_workers(_worker, 8, "tiny-llama", dict(context_parallel_size=8, micro_batch_size=GB, cp_comm=comm,
                                                      global_b=GB))
    _compare(ref, res)


def test_cp8_ulysses():
    """Ulysses needs heads % cp == 0: 8 query heads, 2 kv heads replicated 4x."""
    heads = dict(num_attention_heads=8, num_key_value_heads=2)
    ref = _reference("tiny-llama", 1, GB, **heads)
    res = run_workers(_worker, 8, "tiny-llama", dict(context_parallel_size=8, micro_batch_size=GB,
                                                      cp_comm="ulysses", global_b=GB, **heads))
    _compare(ref, res)


def test_tp2_cp2_dp2():
    ref = _reference("tiny-llama", 1, GB)
    res = run_workers(_worker, 8, "tiny-llama", dict(tensor_parallel_size=2, context_parallel_size=2,
                                                      data_parallel_size=2, micro_batch_size=4, global_b=GB))
    _compare(ref, res)


@pytest.mark.parametrize("kw", [
    dict(expert_parallel_size=8, micro_batch_size=1),
    dict(expert_parallel_size=4, data_parallel_size=2, micro_batch_size=1),
    dict(expert_parallel_size=4, tensor_parallel_size=2, micro_batch_size=2),
    dict(expert_parallel_size=8, micro_batch_size=1, moe_capacity_factor=8.0, moe_ep_chunks=2),
    dict(expert_parallel_size=4, tensor_parallel_size=2, micro_batch_size=2, moe_capacity_factor=4.0),
], ids=["ep8", "ep4_dp2", "ep4_tp2", "ep8_capacity_chunked", "ep4_tp2_capacity"])
def test_mixtral_ep(kw):
    """Mixtral-style MoE (8 experts, top-2): EP carved out of data parallelism, dense
    grads reduced over DP x EP, expert grads over expert-DP."""
    ref = _reference("tiny-mixtral", 1, GB)
    res = run_workers(_worker, 8, "tiny-mixtral", dict(kw, global_b=GB))
    _compare_moe(ref, res)


def test_mixtral_ep8_zero1_adamw():
    """2 AdamW steps: the dense arena sharded over DP x EP (8 ranks), experts unsharded.
    Compared rank-wise with the replicated-optimizer EP=8 run: AdamW amplifies the
    ~1e-6 fp32 reordering of the MoE combine, which can flip a step-2 top-k choice
    against the single process (see test_zero1_moe_ep2_dense_sharded)."""
    kw = dict(expert_parallel_size=8, micro_batch_size=1, global_b=GB, **_ADAM)
    base = run_workers(_worker, 8, "tiny-mixtral", dict(kw, zero_stage=0))
    res = run_workers(_worker, 8, "tiny-mixtral", dict(kw, zero_stage=1))
    for b, r in zip(base, res):
        _compare(b, [r], atol=1e-5, rtol=1e-4)

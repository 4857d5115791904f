"""utils/memory.py against the peaks measured on one MI355X by the per-rank slices of the
8-GPU layouts (bench.py --slice, profiles/r06/slices/*.json): each estimate within 5 %."""
from __future__ import annotations

import pytest

from scaletorch_amd.models import get_model_config
from scaletorch_amd.utils.memory import estimate_rank_memory

# layout -> (estimate kwargs, measured peak GB of the slice rank)
MEASURED = {
    "dp8_zero1": (dict(model="llama3-8b", dp=8, micro_batch=6, zero1=True), 201.18),
    "tp2pp2dp2_first_stage": (dict(model="llama3-8b", tp=2, pp=2, dp=2, micro_batch=4, grad_acc=8, zero1=True,
                                   sequence_parallel=True, virtual_pipeline=2, pp_rank=0), 78.51),
    "tp2pp2dp2_last_stage": (dict(model="llama3-8b", tp=2, pp=2, dp=2, micro_batch=4, grad_acc=8, zero1=True,
                                  sequence_parallel=True, virtual_pipeline=2, pp_rank=1), 60.69),
    "tp2pp2dp2_9_8_8_7_first": (dict(model="llama3-8b", tp=2, pp=2, dp=2, micro_batch=4, grad_acc=8, zero1=True,
                                     sequence_parallel=True, virtual_pipeline=2, pp_rank=0,
                                     layer_distribution=[9, 8, 8, 7]), 84.71),
    "tp2pp2dp2_9_8_8_7_last": (dict(model="llama3-8b", tp=2, pp=2, dp=2, micro_batch=4, grad_acc=8, zero1=True,
                                    sequence_parallel=True, virtual_pipeline=2, pp_rank=1,
                                    layer_distribution=[9, 8, 8, 7]), 59.06),
    "cp8_32k": (dict(model="llama3-8b", cp=8, micro_batch=1, seq_len=32768, zero1=True), 115.89),
    "mixtral_ep8_rccl": (dict(model="mixtral-8x7b", ep=8, micro_batch=1, grad_acc=2, zero1=True, moe_dropless=True,
                              moe_exact_rows=True), 140.18),
}


@pytest.mark.parametrize("name", sorted(MEASURED))
def test_estimate_matches_slice_peak(name):
    kw, peak = MEASURED[name]
    kw = dict(kw)
    cfg = get_model_config(kw.pop("model"))
    est = estimate_rank_memory(cfg, fused_head_chunk=4096, optimizer_state_dtype="bf16", **kw)
    assert abs(est.total_gb - peak) / peak < 0.05, (name, est.summary(), peak)


def test_first_stage_is_the_worst_rank_and_exact_rows_shrink_moe():
    m = get_model_config("llama3-8b")
    kw = dict(tp=2, pp=2, dp=2, micro_batch=4, grad_acc=8, zero1=True, sequence_parallel=True)
    for v in (1, 2):
        first = estimate_rank_memory(m, virtual_pipeline=v, pp_rank=0, **kw).activations_gb
        last = estimate_rank_memory(m, virtual_pipeline=v, pp_rank=1, **kw).activations_gb
        assert first > last
    x = get_model_config("mixtral-8x7b")
    kw = dict(ep=8, micro_batch=1, grad_acc=2, zero1=True, moe_dropless=True)
    assert (estimate_rank_memory(x, moe_exact_rows=True, **kw).activations_gb
            < 0.5 * estimate_rank_memory(x, moe_exact_rows=False, **kw).activations_gb)

"""Numerical parity of every parallel mode against a single-process run (CPU / gloo).

The reference had NO parity tests, which is how its DP+GA,
CP and EP bugs survived.  Each case runs one SGD step of a tiny model on a
fixed global batch and compares the loss and the updated weights (in the
reference checkpoint layout, TP shards compared to slices of the full model)
with the single-process result.
"""
from __future__ import annotations

import pytest
import torch

from tests.dist_harness import run_workers

pytestmark = pytest.mark.slow

SEQ = 32
GLOBAL_B = 4


def _global_batch(vocab: int, n: int = GLOBAL_B):
    g = torch.Generator().manual_seed(99)
    return torch.randint(0, vocab, (n, SEQ + 1), generator=g)


def _make_args(model: str, **kw):
    from scaletorch_amd.trainer.config import ScaleTorchArguments

    base = dict(model_name_or_path=model, synthetic_data=True, sequence_length=SEQ, use_cpu=True, backend="gloo",
                dtype="float32", optimizer_type="sgd", learning_rate=0.5, lr_scheduler_type="constant",
                max_grad_norm=None, total_train_steps=2, seed=7)
    base.update(kw)
    return ScaleTorchArguments(**base)


def _batches_for(tr, X):
    """Yield this rank's micro-batches of the global batch X (DP/EP shard + CP slice)."""
    from scaletorch_amd.data.loader import cp_slice_indices
    from scaletorch_amd.parallel import mesh

    a = tr.args
    pg = mesh.pgm
    data_rank = pg.data_rank if pg else 0
    data_world = pg.data_world_size if pg else 1
    per = X.shape[0] // data_world
    mine = X[data_rank * per:(data_rank + 1) * per]
    cp = pg.cp_world_size if pg else 1
    cpr = pg.cp_rank if pg else 0
    idx = cp_slice_indices(SEQ, cp, cpr, a.cp_zigzag)
    mbs = a.micro_batch_size
    out = []
    for i in range(0, mine.shape[0], mbs):
        ids = mine[i:i + mbs]
        out.append({"input_ids": ids[:, :-1][:, idx].contiguous(), "target_ids": ids[:, 1:][:, idx].contiguous(),
                    "position_ids": idx.unsqueeze(0).expand(ids.shape[0], -1).contiguous(), "hidden_states": None})
    return out


def _run_one_step(model: str, **kw):
    from scaletorch_amd.trainer.engine import Trainer

    steps = kw.pop("steps", 1)
    global_b = kw.pop("global_b", GLOBAL_B)
    import os

    os.environ.update(kw.pop("env", {}))
    tr = Trainer(_make_args(model, **kw), build_data=False)
    X = _global_batch(tr.model_config.vocab_size, global_b)
    batches = _batches_for(tr, X)
    tr.data = iter(batches * 4 * steps)
    for _ in range(steps):
        loss = tr.reduced_loss(tr.train_step())
    tr.model.wait_params()
    sd = {k: v.detach().clone() for k, v in tr.raw_model.reference_state_dict().items()}
    from scaletorch_amd.parallel import mesh

    pg = mesh.pgm
    coords = dict(tp=pg.tp_rank if pg else 0, tp_size=pg.tp_world_size if pg else 1,
                  ep=pg.ep_rank if pg else 0, ep_size=pg.ep_world_size if pg else 1)
    return loss, sd, coords


def _worker(rank, world, model, kw):
    return _run_one_step(model, **kw)


_REF_CACHE = {}


def _reference(model: str, ga: int = 1, global_b: int = GLOBAL_B, **extra):
    key = (model, ga, global_b, tuple(sorted(extra.items())))
    if key not in _REF_CACHE:
        _REF_CACHE[key] = run_workers(_worker, 1, model, dict(micro_batch_size=global_b // ga, global_b=global_b,
                                                                gradient_accumulation_steps=ga, **extra))[0]
    return _REF_CACHE[key]


def _tp_slice(full: torch.Tensor, name: str, tp: int, r: int) -> torch.Tensor:
    col = any(s in name for s in ("q_proj", "k_proj", "v_proj", "gate_proj", "up_proj", "final_proj", "embedding"))
    row = any(s in name for s in ("out_proj", "down_proj"))
    if tp == 1 or not (col or row) or "experts" in name:
        return full
    if col:
        return full.chunk(tp, dim=0)[r]
    return full.chunk(tp, dim=1)[r]


def _compare(ref, results, atol=2e-5, rtol=2e-3, loss_rtol=1e-4):
    ref_loss, ref_sd, _ = ref
    for loss, sd, c in results:
        assert abs(loss - ref_loss) < loss_rtol * max(1, abs(ref_loss)), (loss, ref_loss)
        for k, v in sd.items():
            if k not in ref_sd:
                continue
            exp = _tp_slice(ref_sd[k], k, c["tp_size"], c["tp"])
            assert exp.shape == v.shape, (k, exp.shape, v.shape)
            torch.testing.assert_close(v, exp, atol=atol, rtol=rtol, msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("kw", [
    dict(data_parallel_size=2, micro_batch_size=2),
    dict(data_parallel_size=2, micro_batch_size=1, gradient_accumulation_steps=2),
    dict(tensor_parallel_size=2, micro_batch_size=4),
    dict(tensor_parallel_size=2, micro_batch_size=4, sequence_parallel=True),
    dict(tensor_parallel_size=2, micro_batch_size=4, sequence_parallel=True, env={"ST_SP_CHUNKS": "2"}),
    dict(tensor_parallel_size=2, micro_batch_size=4, sequence_parallel=True, env={"ST_SP_OVERLAP": "0"}),
    dict(tensor_parallel_size=2, micro_batch_size=4, sequence_parallel=True, fused_lm_head=False),
    dict(tensor_parallel_size=2, micro_batch_size=4, fused_lm_head=False),
    dict(tensor_parallel_size=2, micro_batch_size=4, lm_head_chunk_tokens=5),
    dict(tensor_parallel_size=2, micro_batch_size=4, env={"ST_TP_AR_CHUNKS": "3"}),
    dict(data_parallel_size=2, micro_batch_size=2, gradient_checkpointing=True),
    dict(data_parallel_size=2, micro_batch_size=2, gradient_checkpointing=True, recompute_granularity="selective"),
    dict(context_parallel_size=2, micro_batch_size=4),
    dict(context_parallel_size=2, micro_batch_size=4, cp_comm="ring"),
    dict(context_parallel_size=2, micro_batch_size=4, cp_comm="ring", cp_zigzag=False),
    dict(context_parallel_size=2, micro_batch_size=4, cp_comm="ulysses"),
    dict(context_parallel_size=2, micro_batch_size=4, cp_comm="ulysses", cp_zigzag=False),
    dict(pipeline_parallel_size=2, micro_batch_size=2, gradient_accumulation_steps=2),
    dict(pipeline_parallel_size=2, micro_batch_size=2, gradient_accumulation_steps=2, pipeline_parallel_engine="afab"),
], ids=["dp2", "dp2_ga2", "tp2", "tp2_sp", "tp2_sp_chunked", "tp2_sp_serial", "tp2_sp_logits_head", "tp2_logits_head", "tp2_head_chunk5",
        "tp2_chunked_ar", "dp2_gc_full", "dp2_gc_selective", "cp2", "cp2_ring", "cp2_ring_contig", "cp2_ulysses",
        "cp2_ulysses_contig", "pp2_1f1b", "pp2_afab"])
def test_dense_parity_world2(kw):
    ref = _reference("tiny-llama")
    res = run_workers(_worker, 2, "tiny-llama", kw)
    _compare(ref, res)


@pytest.mark.parametrize("pp,v,ga,extra", [(2, 2, 2, {}), (2, 2, 4, {}), (4, 2, 4, {}),
                                           (2, 2, 2, {"tensor_parallel_size": 2, "sequence_parallel": True})],
                         ids=["pp2v2_ga2", "pp2v2_ga4", "pp4v2_ga4", "tp2_sp_pp2v2"])
def test_interleaved_1f1b_parity(pp, v, ga, extra):
    """Interleaved 1F1B (v model chunks per rank over pp x v chunks of the layers)
    equals the single-process step on loss and every weight."""
    layers = pp * v
    ref = _reference("tiny-llama", ga, num_hidden_layers=layers)
    world = pp * extra.get("tensor_parallel_size", 1)
    res = run_workers(_worker, world, "tiny-llama", dict(pipeline_parallel_size=pp, micro_batch_size=GLOBAL_B // ga,
                                                         gradient_accumulation_steps=ga, virtual_pipeline_size=v,
                                                         num_hidden_layers=layers, **extra))
    _compare(ref, res)


def test_interleaved_uneven_layer_distribution_parity():
    """Interleaved 1F1B with an uneven per-chunk layer distribution (global chunk order:
    chunk v * pp + stage) -- "2,1,2,1": stage 0 holds 4 layers, the last stage (LM head) 2 --
    equals the single-process step on loss and every weight."""
    ref = _reference("tiny-llama", 2, num_hidden_layers=6)
    res = run_workers(_worker, 2, "tiny-llama", dict(pipeline_parallel_size=2, micro_batch_size=GLOBAL_B // 2,
                                                     gradient_accumulation_steps=2, virtual_pipeline_size=2,
                                                     num_hidden_layers=6, layer_distribution="2,1,2,1"))
    _compare(ref, res)


@pytest.mark.parametrize("engine", ["1f1b", "afab"])
def test_pp3_parity(engine):
    """Three pipeline stages (a middle stage that both receives and sends in each
    direction) on per-channel communicators equal the single-process step."""
    ref = _reference("tiny-llama", 4, num_hidden_layers=3)
    res = run_workers(_worker, 3, "tiny-llama", dict(pipeline_parallel_size=3, micro_batch_size=1,
                                                     gradient_accumulation_steps=4, num_hidden_layers=3,
                                                     pipeline_parallel_engine=engine))
    _compare(ref, res)


def test_interleaved_schedules_deadlock_free_with_posted_receives():
    """The engine's model (pipeline_parallel.py): one communicator per direction and ring
    seam, receives posted 1-3 ahead, sends issued after their compute step -- every
    (P, V, M) completes with every channel matched in order."""
    from scaletorch_amd.parallel import interleaved as I

    for P in (2, 3, 4, 8):
        for V in (1, 2, 3, 4):
            for M in (P, 2 * P, 4 * P):
                for depth in (1, 2, 3):
                    I.simulate_channels(P, V, M, depth)


def test_pipeline_engine_streams_deadlock_free_on_rccl_layout():
    """Stream-level replay of the engine's host issue order under RCCL semantics (one
    ordered stream per rank per communicator, comm streams fenced on compute): with one
    2-rank communicator per directed stage pair (the mesh layout) AFAB, 1F1B and
    interleaved 1F1B complete for P 2-8 and depth 1-3; the round-3 layout (one
    whole-pipeline communicator per direction) deadlocks at P >= 3 with receives
    posted two ahead, which the replay must detect."""
    from scaletorch_amd.parallel import interleaved as I

    for sched in ("afab", "1f1b", "interleaved"):
        for P in (2, 3, 4, 8):
            for V in ((1, 2, 3) if sched == "interleaved" else (1,)):
                for M in (P, 2 * P, 4 * P):
                    for depth in (1, 2, 3):
                        I.simulate_streams(I.engine_programs(P, V, M, sched, depth, I.channel_layout))
    for sched in ("1f1b", "interleaved"):
        with pytest.raises(AssertionError, match="deadlock"):
            I.simulate_streams(I.engine_programs(3, 1, 6, sched, 2, I.shared_layout))
    I.simulate_streams(I.engine_programs(2, 1, 4, "1f1b", 2, I.shared_layout))  # pp = 2 was safe


def test_mesh_pp_channels_are_two_rank_directed():
    """Every pipeline channel a rank holds is a distinct 2-rank group of (sender,
    receiver) stages, fwd i: i -> i+1 and bwd i: i+1 -> i (mod P)."""
    from unittest import mock

    from scaletorch_amd.parallel.mesh import ProcessGroupManager

    made = []

    def fake_new_group(ranks):
        made.append(tuple(ranks))
        return ("g", len(made), tuple(ranks))

    for P, dp, tp in ((3, 2, 2), (2, 1, 1), (4, 1, 2)):
        world = P * dp * tp
        for rank in range(world):
            made.clear()
            with mock.patch("scaletorch_amd.dist.collectives.is_distributed", return_value=True), \
                    mock.patch("scaletorch_amd.dist.collectives.new_group", side_effect=fake_new_group):
                pg = ProcessGroupManager(tp_size=tp, pp_size=P, dp_size=dp, rank=rank, world_size=world)
            chans = pg.pp_channels
            r = pg.pp_rank
            assert set(chans) == {("fwd", r), ("fwd", (r - 1) % P), ("bwd", r), ("bwd", (r - 1) % P)}
            assert len(set(chans.values())) == 4
            for (kind, i), g in chans.items():
                assert len(g[2]) == 2 and rank in g[2]
                send_stage, recv_stage = (i, (i + 1) % P) if kind == "fwd" else ((i + 1) % P, i)
                assert sorted((x // tp) % P for x in g[2]) == sorted((send_stage, recv_stage))


def test_interleaved_schedules_are_deadlock_free():
    """Every (P, V, M) schedule replays without deadlock under ordered-stream p2p
    semantics, every message matched in order, every step's input present; a
    schedule with one receive dropped is caught."""
    from scaletorch_amd.parallel import interleaved as I

    for P in (2, 3, 4, 8):
        for V in (1, 2, 3, 4):
            for mult in (1, 2, 3):
                I.simulate(P, V, P * mult)
    real = I.build_schedule

    def broken(P, V, M, r):
        acts = real(P, V, M, r)
        if r == 1:
            for a in acts:
                if isinstance(a, I.Exchange) and a.recv:
                    a.recv.pop()
                    break
        return acts

    I.build_schedule = broken
    try:
        with pytest.raises(AssertionError):
            I.simulate(4, 2, 8)
    finally:
        I.build_schedule = real


@pytest.mark.parametrize("comm", ["ulysses", "allgather"])
def test_cp4_parity_world4(comm):
    """cp=4 > Hkv=2: Ulysses replicates each kv head over 2 ranks and sums their dK/dV."""
    ref = _reference("tiny-llama")
    res = run_workers(_worker, 4, "tiny-llama", dict(context_parallel_size=4, micro_batch_size=4, cp_comm=comm))
    _compare(ref, res)


_ADAM = dict(optimizer_type="adamw", learning_rate=1e-2, max_grad_norm=0.05, steps=2)


@pytest.mark.parametrize("kw", [
    dict(data_parallel_size=2, micro_batch_size=2, zero_stage=1),
    dict(data_parallel_size=2, micro_batch_size=2, zero_stage=1, bucket_size_mb=0.02),
    dict(data_parallel_size=2, micro_batch_size=1, gradient_accumulation_steps=2, zero_stage=1, bucket_size_mb=0.05),
], ids=["dp2_zero1", "dp2_zero1_buckets", "dp2_ga2_zero1"])
def test_zero1_adamw_parity(kw):
    """ZeRO-1 (reduce-scatter, sharded AdamW + global clip, param all-gather) over 2
    optimizer steps equals the single-process replicated AdamW run."""
    ga = kw.get("gradient_accumulation_steps", 1)
    ref = _reference("tiny-llama", ga, **_ADAM)
    res = run_workers(_worker, 2, "tiny-llama", dict(kw, **_ADAM))
    _compare(ref, res, atol=5e-5, rtol=5e-3)


def test_zero1_adamw_bf16_moments_parity():
    """bf16 AdamW moments (``optimizer_state_dtype="bf16"``, the bench default) under ZeRO-1:
    the shard-sized bf16 states give the same 2 steps as the replicated bf16-moment run."""
    kw = dict(data_parallel_size=2, micro_batch_size=2, zero_stage=1, bucket_size_mb=0.02)
    ref = _reference("tiny-llama", 1, optimizer_state_dtype="bf16", **_ADAM)
    res = run_workers(_worker, 2, "tiny-llama", dict(kw, optimizer_state_dtype="bf16", **_ADAM))
    _compare(ref, res, atol=5e-5, rtol=5e-3)


def test_zero1_moe_ep2_dense_sharded():
    """EP=2: the dense arena shards over DP x EP, the expert arena (world 1) does not.
    Compared with the replicated-optimizer EP=2 run (the MoE combine's fp32 summation
    order already differs from the single process by ~1e-5, which AdamW amplifies)."""
    kw = dict(expert_parallel_size=2, micro_batch_size=2, **_ADAM)
    base = run_workers(_worker, 2, "tiny-moe", dict(kw, zero_stage=0))
    res = run_workers(_worker, 2, "tiny-moe", dict(kw, zero_stage=1))
    for b, r in zip(base, res):  # rank-wise: each EP rank holds different experts
        _compare(b, [r], atol=1e-5, rtol=1e-4)


def test_xgmi_default_timeout(monkeypatch):
    """The spin-wait bound guards against a dead peer, not a slow one: 60 s by default and
    300 s when ranks time-share one GPU (the old 2 s fired in the 8-rank one-GPU Mixtral
    rehearsal and left EP exchange rows unwritten)."""
    from scaletorch_amd.dist.xgmi import _default_timeout

    monkeypatch.delenv("ST_GPU_OVERSUBSCRIBE", raising=False)
    assert float(_default_timeout()) == 60
    monkeypatch.setenv("ST_GPU_OVERSUBSCRIBE", "1")
    assert float(_default_timeout()) == 300


def _ckpt_worker(rank, world, tmpdir):
    from scaletorch_amd.trainer.engine import Trainer
    from scaletorch_amd.utils.checkpoint import CheckpointManager

    kw = dict(data_parallel_size=2, micro_batch_size=2, zero_stage=1, optimizer_type="adamw", learning_rate=1e-2)
    tr = Trainer(_make_args("tiny-llama", **kw), build_data=False)
    X = _global_batch(tr.model_config.vocab_size)
    tr.data = iter(_batches_for(tr, X) * 8)
    tr.train_step()
    cm = CheckpointManager(tmpdir, async_save=False)
    cm.save_checkpoint(tr.model, tr.optimizer, 1, 0)
    l_cont = tr.reduced_loss(tr.train_step())
    tr2 = Trainer(_make_args("tiny-llama", **kw), build_data=False)
    tr2.data = iter(_batches_for(tr2, X) * 8)
    cm.load_checkpoint(tr2.model, tr2.optimizer, f"{tmpdir}/1")
    l_resumed = tr2.reduced_loss(tr2.train_step())
    return l_cont, l_resumed


def test_zero1_checkpoint_roundtrip(tmp_path):
    """Each rank writes / reads its own optimizer shard; a resumed run continues bit-identically."""
    for l_cont, l_resumed in run_workers(_ckpt_worker, 2, str(tmp_path)):
        assert l_cont == l_resumed, (l_cont, l_resumed)


def test_qwen3_tied_tp2_parity():
    ref = _reference("tiny-qwen3")
    res = run_workers(_worker, 2, "tiny-qwen3", dict(tensor_parallel_size=2, micro_batch_size=4))
    _compare(ref, res)


def _expert_global_key(k: str, sd: dict, ep_rank: int) -> str:
    """Local expert e on ep rank r is global expert r*E_local + e."""
    parts = k.split(".")
    i = parts.index("experts") + 2
    e = int(parts[i])
    e_local = sum(1 for kk in sd if kk.endswith("gate_proj.weight") and parts[:i - 1] == kk.split(".")[:i - 1])
    parts[i] = str(ep_rank * e_local + e)
    return ".".join(parts)


def _compare_moe(ref, res, atol=1e-4, rtol=2e-3):
    ref_loss, ref_sd, _ = ref
    for loss, sd, c in res:
        assert abs(loss - ref_loss) < 1e-4 * max(1, abs(ref_loss)), (loss, ref_loss)
        for k, v in sd.items():
            if ".experts.experts." in k:
                exp = ref_sd[_expert_global_key(k, sd, c["ep"])]
                exp = exp.chunk(c["tp_size"], dim=1 if "down_proj" in k else 0)[c["tp"]]
            elif k in ref_sd:
                exp = _tp_slice(ref_sd[k], k, c["tp_size"], c["tp"])
            else:
                continue
            torch.testing.assert_close(v, exp, atol=atol, rtol=rtol, msg=lambda m: f"{k}: {m}")


def test_moe_ep2_parity():
    ref = _reference("tiny-moe")
    res = run_workers(_worker, 2, "tiny-moe", dict(expert_parallel_size=2, micro_batch_size=2))
    _compare_moe(ref, res)


@pytest.mark.parametrize("chunks", [1, 3])
def test_moe_ep2_capacity_dispatch_parity(chunks):
    """Sync-free static-capacity dispatch (capacity = every row: nothing dropped), with the
    tokens pipelined in chunks through async all-to-alls: same step as one process."""
    ref = _reference("tiny-moe")
    res = run_workers(_worker, 2, "tiny-moe", dict(expert_parallel_size=2, micro_batch_size=2,
                                                   moe_capacity_factor=2.0, moe_ep_chunks=chunks))
    _compare_moe(ref, res)


class _RcclSemantics:
    """Stands in for torch.distributed inside data_parallel.py: forwards everything,
    but executes all_reduce / reduce_scatter_tensor with RCCL's contract (ReduceOp.AVG,
    in-place reduce-scatter when recv == send + rank * count) on top of gloo SUM, and
    asserts that an aliased output is exactly this rank's chunk."""

    class _Done:
        def wait(self):
            return None

    def __init__(self):
        import torch.distributed as dist

        self._d = dist
        self.calls = {"avg_all_reduce": 0, "avg_reduce_scatter": 0, "inplace_reduce_scatter": 0}

    def __getattr__(self, k):
        return getattr(self._d, k)

    def all_reduce(self, t, op=None, group=None, async_op=False):
        d = self._d
        if op == d.ReduceOp.AVG:
            self.calls["avg_all_reduce"] += 1
            d.all_reduce(t, op=d.ReduceOp.SUM, group=group)
            t.div_(d.get_world_size(group))
            return self._Done() if async_op else None
        return d.all_reduce(t, op=op, group=group, async_op=async_op)

    def reduce_scatter_tensor(self, out, inp, op=None, group=None, async_op=False):
        d = self._d
        w, r = d.get_world_size(group), d.get_rank(group)
        n = out.numel()
        lo, hi = inp.data_ptr(), inp.data_ptr() + inp.numel() * inp.element_size()
        if lo <= out.data_ptr() < hi:
            assert out.data_ptr() == lo + r * n * inp.element_size(), "in-place output is not this rank's chunk"
            self.calls["inplace_reduce_scatter"] += 1
        src = inp.clone()
        tmp = torch.empty_like(out)
        d.reduce_scatter_tensor(tmp, src, op=d.ReduceOp.SUM, group=group)
        if op == d.ReduceOp.AVG:
            self.calls["avg_reduce_scatter"] += 1
            tmp.div_(w)
        out.copy_(tmp)
        return self._Done() if async_op else None


def _rccl_worker(rank, world, model, kw):
    from scaletorch_amd.parallel import data_parallel as dp_mod

    shim = _RcclSemantics()
    dp_mod.dist = shim
    dp_mod._is_rccl = lambda group: True
    out = _run_one_step(model, **kw)
    return out + (shim.calls,)


@pytest.mark.parametrize("kw,expect", [
    (dict(data_parallel_size=2, micro_batch_size=2, grad_reduce_dtype="fp32"), "avg_all_reduce"),
    (dict(data_parallel_size=2, micro_batch_size=2, zero_stage=1, grad_reduce_dtype="fp32", bucket_size_mb=0.05),
     "inplace_reduce_scatter"),
    (dict(data_parallel_size=2, micro_batch_size=2, zero_stage=1, grad_reduce_dtype="bf16"), "avg_reduce_scatter"),
], ids=["avg_allreduce", "zero1_inplace_rs", "zero1_bf16_rs"])
def test_rccl_only_branches(kw, expect):
    """The RCCL-only reduction branches of GradArena.launch (AVG, in-place
    reduce-scatter, bf16 comm buffer) against the single-process step."""
    # bf16 reduction: one SGD step (AdamW would amplify bf16 rounding of near-zero grads)
    opt = _ADAM if kw["grad_reduce_dtype"] == "fp32" else {}
    ref = _reference("tiny-llama", **opt)
    res = run_workers(_rccl_worker, 2, "tiny-llama", dict(kw, **opt))
    for r in res:
        assert r[3][expect] > 0, r[3]
    tol = dict(atol=5e-5, rtol=5e-3) if opt else dict(atol=2e-3, rtol=2e-2, loss_rtol=1e-3)
    _compare(ref, [r[:3] for r in res], **tol)


def _cover_worker(rank, world, model, kw):
    from scaletorch_amd.trainer.engine import Trainer

    tr = Trainer(_make_args(model, **kw), build_data=False)
    X = _global_batch(tr.model_config.vocab_size)
    b = _batches_for(tr, X)[0]
    return tr.model.uncovered_params(lambda: tr.model(input_ids=b["input_ids"], position_ids=b["position_ids"]))


@pytest.mark.parametrize("model,world,kw", [
    ("tiny-llama", 1, dict(micro_batch_size=4)),
    ("tiny-qwen3", 1, dict(micro_batch_size=4)),
    ("tiny-moe", 1, dict(micro_batch_size=4)),
    ("tiny-llama", 2, dict(tensor_parallel_size=2, sequence_parallel=True, micro_batch_size=4)),
    ("tiny-qwen3", 2, dict(tensor_parallel_size=2, sequence_parallel=True, micro_batch_size=4)),
], ids=["llama", "qwen3", "moe", "llama_tp2_sp", "qwen3_tied_tp2_sp"])
def test_every_weight_read_waits_for_its_bucket(model, world, kw):
    """Every trainable weight is covered by the forward pre-hook bucket wait of a module
    that actually runs (the SP LM head and the fused QK-norm read weights
    without calling their owning module, racing the side-stream optimizer update)."""
    for missing in run_workers(_cover_worker, world, model, kw):
        assert missing == [], missing


def _dropless_uneven_worker(rank, world):
    """EP=2 MoE layer on a rank-dependent token count vs the same layer with every expert
    local (ep = 1 math, built from the same full weights)."""
    import torch.distributed as dist

    from scaletorch_amd.models.config import get_model_config
    from scaletorch_amd.models.moe import MoELayer
    from scaletorch_amd.parallel import mesh

    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = get_model_config("tiny-moe")
    torch.manual_seed(0)
    ref_layer = MoELayer(cfg).float()  # ep = 1: all 8 experts here (mesh not installed yet)
    mesh.setup_process_group_manager(ep_size=world)
    layer = MoELayer(cfg).float()
    with torch.no_grad():
        layer.router.gate.weight.copy_(ref_layer.router.gate.weight)
        El = layer.num_local
        layer.experts.w_gate_up.copy_(ref_layer.experts.w_gate_up[rank * El:(rank + 1) * El])
        layer.experts.w_down.copy_(ref_layer.experts.w_down[rank * El:(rank + 1) * El])
    T = 5 + 7 * rank  # different token counts on the two ranks
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(1, T, cfg.hidden_size, generator=g)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya = layer(xa)
    yb = ref_layer(xb)
    ya.square().sum().backward()
    yb.square().sum().backward()
    gw = ref_layer.experts.w_gate_up.grad.clone()
    dist.all_reduce(gw)  # every rank's tokens reach the owner's experts: sum the per-rank references
    gw = gw[rank * El:(rank + 1) * El]
    return (ya.detach(), yb.detach(), xa.grad, xb.grad, layer.experts.w_gate_up.grad, gw,
            int(layer.dropped_rows))


def _dropless_ragged_steps_worker(rank, world):
    import torch.distributed as dist

    from scaletorch_amd.models.config import get_model_config
    from scaletorch_amd.models.moe import MoELayer
    from scaletorch_amd.parallel import mesh

    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = get_model_config("tiny-moe")
    torch.manual_seed(0)
    ref_layer = MoELayer(cfg).float()
    mesh.setup_process_group_manager(ep_size=world)
    layer = MoELayer(cfg).float()
    with torch.no_grad():
        layer.router.gate.weight.copy_(ref_layer.router.gate.weight)
        El = layer.num_local
        layer.experts.w_gate_up.copy_(ref_layer.experts.w_gate_up[rank * El:(rank + 1) * El])
        layer.experts.w_down.copy_(ref_layer.experts.w_down[rank * El:(rank + 1) * El])
    # one rank's token count repeats while its peer's changes (and the reverse): a bound
    # cached on the local count would desynchronise the EP collectives here
    counts = [[5, 5, 9, 9], [12, 20, 20, 6]][rank]
    out = []
    for step, T in enumerate(counts):
        g = torch.Generator().manual_seed(1000 * step + rank)
        x = torch.randn(1, T, cfg.hidden_size, generator=g)
        xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
        ya, yb = layer(xa), ref_layer(xb)
        ya.square().sum().backward()
        yb.square().sum().backward()
        out.append((ya.detach(), yb.detach(), xa.grad, xb.grad))
    return out


def test_moe_dropless_ragged_counts_across_steps():
    """Several dropless EP forwards/backwards where each rank's token count changes between
    calls independently of its peer's: every call agrees on the buffer bound, so the EP
    collectives stay in step and each call matches the all-experts-local computation."""
    res = run_workers(_dropless_ragged_steps_worker, 2)
    for steps in res:
        assert len(steps) == 4
        for ya, yb, ga, gb in steps:
            torch.testing.assert_close(ya, yb, atol=1e-5, rtol=1e-4)
            torch.testing.assert_close(ga, gb, atol=1e-5, rtol=1e-4)


def test_moe_dropless_uneven_token_counts():
    """Dropless EP dispatch with device counts when EP ranks hold DIFFERENT token counts
    (ragged batches): outputs, input gradients and expert weight gradients equal the
    all-experts-local computation; nothing is dropped."""
    res = run_workers(_dropless_uneven_worker, 2)
    for ya, yb, ga, gb, wa, wb, dropped in res:
        torch.testing.assert_close(ya, yb, atol=1e-5, rtol=1e-4)
        torch.testing.assert_close(ga, gb, atol=1e-5, rtol=1e-4)
        torch.testing.assert_close(wa, wb, atol=1e-5, rtol=1e-4)
        assert dropped == 0


def _tp_vote_worker(rank, world):
    import torch.distributed as dist

    from scaletorch_amd.parallel import tensor_parallel as TP

    dist.init_process_group("gloo", rank=rank, world_size=world)
    names = ["all_reduce", "all_gather", "reduce_scatter"]
    # rank 2 saw its all-gather lose to RCCL; rank 3's reduce-scatter failed correctness
    flags = [1, 0 if rank == 2 else 1, 0 if rank == 3 else 1]
    voted = TP._vote(names, flags)

    class FakeComm:
        closed = 0

        def close(self):
            FakeComm.closed += 1

    TP._XGMI[1] = FakeComm()
    TP._XGMI[2] = FakeComm()
    TP._close_tp_xgmi()
    TP.set_tp_comm("xgmi" if any(voted.values()) else "rccl", voted)
    routed = {op: TP._TP_XGMI_OPS[op] for op in names}
    out = (voted, FakeComm.closed, len(TP._XGMI), dict(TP.TRANSPORT), routed)
    TP.set_tp_comm("rccl")
    return out


def test_tp_transport_vote_is_min_over_ranks_and_losers_are_closed():
    """tp 4 / 8 auto transport: each collective keeps xGMI only if EVERY rank's self-test
    passed it (MIN vote), the per-collective routing follows the vote, and closing the
    losing communicators releases every TP IPC area."""
    res = run_workers(_tp_vote_worker, 4)
    for voted, closed, left, transport, routed in res:
        assert voted == {"all_reduce": True, "all_gather": False, "reduce_scatter": False}
        assert closed == 2 and left == 0
        assert transport["tp"] == "xgmi" and transport["ops"] == ["all_reduce"]
        assert routed == {"all_reduce": True, "all_gather": False, "reduce_scatter": False}

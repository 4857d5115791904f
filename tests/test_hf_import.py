"""HF safetensors import on the model-build path (reference model_builder.py:82-84,
utils/checkpoint.py:64-464).

Tiny Llama / tied Qwen3 / Mixtral (``w1/w2/w3``) / Qwen3-MoE checkpoints are written
in HF naming with ``safetensors`` (one file, or two shards + ``model.safetensors.index.json``),
then built through ``Trainer`` with ``model_name_or_path=<dir>``:

* world 1: every internal tensor equals its HF source (exact), and the loss differs
  from the random-init build (so the load really happened);
* gloo tp2 / pp2 / ep2 / tp2 x pp2: the first-step loss equals the world-1 load
  (each rank reads only its PP stage, EP experts and TP slice).
"""
from __future__ import annotations

import json
import os

import pytest
import torch

from tests.dist_harness import run_workers

pytestmark = pytest.mark.slow

SEQ = 32
GLOBAL_B = 4

H, HEADS, KV, D, INTER, VOCAB, LAYERS, EXPERTS = 64, 4, 2, 16, 128, 256, 2, 4

_CONFIGS = {
    "llama": dict(model_type="llama", vocab_size=VOCAB, hidden_size=H, intermediate_size=INTER,
                  num_hidden_layers=LAYERS, num_attention_heads=HEADS, num_key_value_heads=KV,
                  max_position_embeddings=256, rms_norm_eps=1e-5, rope_theta=10000.0, tie_word_embeddings=False),
    "qwen3": dict(model_type="qwen3", vocab_size=VOCAB, hidden_size=H, intermediate_size=INTER,
                  num_hidden_layers=LAYERS, num_attention_heads=HEADS, num_key_value_heads=KV, head_dim=D,
                  max_position_embeddings=256, rms_norm_eps=1e-6, rope_theta=1e6, tie_word_embeddings=True),
    "mixtral": dict(model_type="mixtral", vocab_size=VOCAB, hidden_size=H, intermediate_size=INTER,
                    num_hidden_layers=LAYERS, num_attention_heads=HEADS, num_key_value_heads=KV,
                    max_position_embeddings=256, rms_norm_eps=1e-5, rope_theta=1e6, num_local_experts=EXPERTS,
                    num_experts_per_tok=2, tie_word_embeddings=False),
    "qwen3_moe": dict(model_type="qwen3_moe", vocab_size=VOCAB, hidden_size=H, intermediate_size=INTER,
                      moe_intermediate_size=INTER // 2, num_hidden_layers=LAYERS, num_attention_heads=HEADS,
                      num_key_value_heads=KV, head_dim=D, max_position_embeddings=256, rms_norm_eps=1e-6,
                      rope_theta=1e6, num_experts=EXPERTS, num_experts_per_tok=2, norm_topk_prob=True,
                      tie_word_embeddings=False),
}


def _hf_tensors(kind: str, seed: int = 0) -> dict[str, torch.Tensor]:
    """HF-named weights exactly as transformers' Llama / Qwen3 / Mixtral / Qwen3-MoE save them."""
    g = torch.Generator().manual_seed(seed)

    def w(*shape, scale=0.08):
        return (torch.randn(*shape, generator=g) * scale).contiguous()

    def norm(n):
        return (1.0 + 0.1 * torch.randn(n, generator=g)).contiguous()

    d = D if kind in ("qwen3", "qwen3_moe") else H // HEADS
    t = {"model.embed_tokens.weight": w(VOCAB, H, scale=0.5), "model.norm.weight": norm(H)}
    if kind != "qwen3":
        t["lm_head.weight"] = w(VOCAB, H)
    for i in range(LAYERS):
        p = f"model.layers.{i}."
        t[p + "input_layernorm.weight"] = norm(H)
        t[p + "post_attention_layernorm.weight"] = norm(H)
        t[p + "self_attn.q_proj.weight"] = w(HEADS * d, H)
        t[p + "self_attn.k_proj.weight"] = w(KV * d, H)
        t[p + "self_attn.v_proj.weight"] = w(KV * d, H)
        t[p + "self_attn.o_proj.weight"] = w(H, HEADS * d)
        t[p + "self_attn.rotary_emb.inv_freq"] = torch.arange(d // 2).float()  # unmapped: ignored
        if kind in ("qwen3", "qwen3_moe"):
            t[p + "self_attn.q_norm.weight"] = norm(d)
            t[p + "self_attn.k_norm.weight"] = norm(d)
        if kind == "mixtral":
            t[p + "block_sparse_moe.gate.weight"] = w(EXPERTS, H, scale=0.3)
            for e in range(EXPERTS):
                q = p + f"block_sparse_moe.experts.{e}."
                t[q + "w1.weight"] = w(INTER, H)
                t[q + "w3.weight"] = w(INTER, H)
                t[q + "w2.weight"] = w(H, INTER)
        elif kind == "qwen3_moe":
            I = INTER // 2
            t[p + "mlp.gate.weight"] = w(EXPERTS, H, scale=0.3)
            for e in range(EXPERTS):
                q = p + f"mlp.experts.{e}."
                t[q + "gate_proj.weight"] = w(I, H)
                t[q + "up_proj.weight"] = w(I, H)
                t[q + "down_proj.weight"] = w(H, I)
        else:
            t[p + "mlp.gate_proj.weight"] = w(INTER, H)
            t[p + "mlp.up_proj.weight"] = w(INTER, H)
            t[p + "mlp.down_proj.weight"] = w(H, INTER)
    return t


def write_hf_checkpoint(root: str, kind: str, sharded: bool = False) -> str:
    from safetensors.torch import save_file

    path = os.path.join(root, f"{kind}{'_sharded' if sharded else ''}")
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(_CONFIGS[kind], f)
    t = _hf_tensors(kind)
    if not sharded:
        save_file(t, os.path.join(path, "model.safetensors"))
        return path
    names = sorted(t)
    halves = [names[: len(names) // 2], names[len(names) // 2:]]
    wmap = {}
    for j, part in enumerate(halves):
        fn = f"model-{j + 1:05d}-of-00002.safetensors"
        save_file({n: t[n] for n in part}, os.path.join(path, fn))
        wmap.update({n: fn for n in part})
    with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": 0}, "weight_map": wmap}, f)
    return path


def _first_step(path: str, **kw):
    from tests.test_parallel_parity import _batches_for, _make_args

    from scaletorch_amd.parallel import mesh
    from scaletorch_amd.trainer.engine import Trainer

    kw.setdefault("micro_batch_size", GLOBAL_B)
    tr = Trainer(_make_args(path, **kw), build_data=False)
    g = torch.Generator().manual_seed(5)
    X = torch.randint(0, VOCAB, (GLOBAL_B, SEQ + 1), generator=g)
    tr.data = iter(_batches_for(tr, X) * 4)
    loss = tr.reduced_loss(tr.train_step())
    pg = mesh.pgm
    return dict(loss=loss, loaded=tr.hf_tensors_loaded, pp=pg.pp_rank if pg else 0)


def _worker(rank, world, path, kw):
    return _first_step(path, **kw)


def _world1_state(rank, world, path, mode):
    from tests.test_parallel_parity import _make_args

    from scaletorch_amd.trainer.engine import Trainer

    tr = Trainer(_make_args(path, micro_batch_size=GLOBAL_B, hf_weights=mode), build_data=False)
    return {k: v.detach().clone() for k, v in tr.raw_model.reference_state_dict().items()}


@pytest.mark.parametrize("kind", ["llama", "qwen3", "mixtral", "qwen3_moe"])
def test_world1_load_is_exact(tmp_path, kind):
    from scaletorch_amd.utils.checkpoint import hf_to_internal_name

    path = write_hf_checkpoint(str(tmp_path), kind, sharded=(kind in ("qwen3", "mixtral")))
    sd = run_workers(_world1_state, 1, path, "required")[0]
    hf = _hf_tensors(kind)
    seen = set()
    for name, t in hf.items():
        iname = hf_to_internal_name(name)
        if iname is None:
            assert "inv_freq" in name
            continue
        assert iname in sd, f"{name} -> {iname} not a model parameter"
        torch.testing.assert_close(sd[iname], t, rtol=0, atol=0, msg=lambda m: f"{iname}: {m}")
        seen.add(iname)
    assert seen == set(sd), f"parameters not loaded: {sorted(set(sd) - seen)}"
    # random init differs: the load is what produced these values
    rnd = run_workers(_world1_state, 1, path, "off")[0]
    assert not torch.equal(rnd["decoder_layers.0.attention.q_proj.weight"], sd["decoder_layers.0.attention.q_proj.weight"])


_LAYOUTS = {
    "llama": [dict(tensor_parallel_size=2), dict(pipeline_parallel_size=2, micro_batch_size=2,
                                                 gradient_accumulation_steps=2),
              dict(tensor_parallel_size=2, pipeline_parallel_size=2, micro_batch_size=2,
                   gradient_accumulation_steps=2)],
    "qwen3": [dict(tensor_parallel_size=2), dict(pipeline_parallel_size=2, micro_batch_size=2,
                                                 gradient_accumulation_steps=2)],
    "mixtral": [dict(expert_parallel_size=2, micro_batch_size=2), dict(tensor_parallel_size=2)],
    "qwen3_moe": [dict(expert_parallel_size=2, micro_batch_size=2)],
}


@pytest.mark.parametrize("kind,kw", [(k, kw) for k, v in _LAYOUTS.items() for kw in v],
                         ids=[f"{k}-" + "-".join(f"{n.split('_')[0]}{x}" for n, x in kw.items()
                                                 if n.endswith("parallel_size"))
                              for k, v in _LAYOUTS.items() for kw in v])
def test_sharded_load_first_step_loss_matches_world1(tmp_path, kind, kw):
    path = write_hf_checkpoint(str(tmp_path), kind, sharded=True)
    ref = run_workers(_worker, 1, path, {})[0]
    assert ref["loaded"] > 0
    world = kw.get("tensor_parallel_size", 1) * kw.get("pipeline_parallel_size", 1) * kw.get("expert_parallel_size", 1)
    res = run_workers(_worker, world, path, dict(kw))
    for r in res:
        assert r["loaded"] > 0
        assert abs(r["loss"] - ref["loss"]) < 1e-4 * max(1.0, abs(ref["loss"])), (r, ref)


def test_unmatched_checkpoint_fails_loudly(tmp_path):
    from safetensors.torch import save_file

    path = write_hf_checkpoint(str(tmp_path), "llama")
    os.remove(os.path.join(path, "model.safetensors"))
    save_file({"transformer.h.0.attn.c_attn.weight": torch.zeros(4, 4)}, os.path.join(path, "model.safetensors"))
    with pytest.raises(RuntimeError, match="none of their tensors"):
        run_workers(_world1_state, 1, path, "auto")


def test_missing_shard_and_required_mode(tmp_path):
    path = write_hf_checkpoint(str(tmp_path), "llama", sharded=True)
    os.remove(os.path.join(path, "model-00002-of-00002.safetensors"))
    with pytest.raises(RuntimeError, match="not present"):
        run_workers(_world1_state, 1, path, "auto")
    empty = tmp_path / "cfg_only"
    empty.mkdir()
    (empty / "config.json").write_text(json.dumps(_CONFIGS["llama"]))
    with pytest.raises(RuntimeError, match="holds no"):
        run_workers(_world1_state, 1, str(empty), "required")
    # auto without weights: random init, nothing loaded
    assert run_workers(_world1_state, 1, str(empty), "auto")[0]

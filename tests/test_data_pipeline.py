"""Real-data path, hermetic: a local WordLevel tokenizer + a jsonl corpus through
``load_tokenizer`` (rank-0 build + broadcast), ``DatasetProcessor`` / ``build_dataset``
(concat_chunk), ``MicroBatchDataLoader`` (DP shard, CP slice, shifted targets, global
positions) and a ``Trainer`` step on it.  Reference: scaletorch/data/dataset.py:89-489,
scaletorch/data/dataloader.py:16-292, scaletorch/data/pretrain_dataset.py:13-107."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest
import torch

from tests.dist_harness import run_workers

WORDS = [f"w{i}" for i in range(60)]


def _write_corpus(root: str, n_docs: int = 40) -> tuple[str, str]:
    from tokenizers import Tokenizer, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast

    vocab = {"[UNK]": 0, "[EOS]": 1}
    vocab.update({w: i + 2 for i, w in enumerate(WORDS)})
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="[UNK]"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    tok_dir = os.path.join(root, "tok")
    PreTrainedTokenizerFast(tokenizer_object=tk, unk_token="[UNK]", eos_token="[EOS]").save_pretrained(tok_dir)
    rng = np.random.default_rng(0)
    data = os.path.join(root, "corpus.jsonl")
    with open(data, "w") as f:
        for _ in range(n_docs):
            f.write(json.dumps({"text": " ".join(rng.choice(WORDS, size=rng.integers(5, 30)))}) + "\n")
    return tok_dir, data


def _expected_chunks(data: str, seq: int) -> np.ndarray:
    flat = []
    with open(data) as f:
        for line in f:
            flat += [WORDS.index(w) + 2 for w in json.loads(line)["text"].split()] + [1]
    n = len(flat) // (seq + 1)
    return np.asarray(flat[: n * (seq + 1)]).reshape(n, seq + 1)


def _args(tok_dir, data, **kw):
    from scaletorch_amd.trainer.config import ScaleTorchArguments

    base = dict(model_name_or_path="tiny-llama", tokenizer_name_or_path=tok_dir, data_path=data,
                dataset_name="local", synthetic_data=False, sequence_length=16, micro_batch_size=2, use_cpu=True,
                backend="gloo", dtype="float32", num_workers=0, total_train_steps=2, seed=3)
    base.update(kw)
    return ScaleTorchArguments(**base)


def test_concat_chunk_dataset_matches_tokenized_corpus(tmp_path):
    from scaletorch_amd.data.dataset import available_strategies, build_dataset

    tok_dir, data = _write_corpus(str(tmp_path))
    ds = build_dataset(_args(tok_dir, data), 16)
    exp = _expected_chunks(data, 16)
    assert "concat_chunk" in available_strategies()
    assert len(ds) == exp.shape[0] > 10
    got = np.stack([ds[i]["input_ids"].numpy() for i in range(len(ds))])
    np.testing.assert_array_equal(got, exp)
    # num_samples subset: fewer documents -> fewer chunks
    assert len(build_dataset(_args(tok_dir, data, num_samples=10), 16)) < len(ds)


def test_npy_dataset_is_memory_mapped(tmp_path):
    from scaletorch_amd.data.dataset import build_dataset

    arr = np.arange(5 * 17, dtype=np.int64).reshape(5, 17)
    p = str(tmp_path / "chunks.npy")
    np.save(p, arr)
    ds = build_dataset(_args("unused", p), 16)
    assert isinstance(ds.chunks, np.memmap) and len(ds) == 5
    np.testing.assert_array_equal(ds[3]["input_ids"].numpy(), arr[3])


def test_pretrain_dataset_pads_and_masks(tmp_path):
    from transformers import AutoTokenizer

    from scaletorch_amd.data.dataset import PretrainDataset

    tok_dir, data = _write_corpus(str(tmp_path), n_docs=6)
    tok = AutoTokenizer.from_pretrained(tok_dir, local_files_only=True)
    tok.pad_token = "[EOS]"
    ds = PretrainDataset(data, tok, max_length=40)
    item = ds[0]
    n = int(item["attention_mask"].sum())
    assert item["input_ids"].shape == (40,) and 0 < n <= 40
    assert (item["labels"][n:] == -100).all() and (item["labels"][:n] == item["input_ids"][:n]).all()


def _loader_worker(rank, world, tok_dir, data, cp, zigzag):
    from scaletorch_amd.data.dataset import build_dataset, load_tokenizer
    from scaletorch_amd.data.loader import MicroBatchDataLoader
    from scaletorch_amd.dist.launch import init_dist

    init_dist(backend="gloo", use_cpu=True)
    # rank 1 never reads the tokenizer directory: the object is broadcast from rank 0
    tok = load_tokenizer(tok_dir if rank == 0 else "/nonexistent")
    ids = tok("w3 w7 w59", add_special_tokens=False)["input_ids"]
    args = _args(tok_dir, data)
    ds = build_dataset(args, 16)
    dp = world // cp
    dl = MicroBatchDataLoader(ds, 2, 16, 1, data_rank=rank // cp, data_world_size=dp, cp_rank=rank % cp,
                              cp_size=cp, zigzag=zigzag, shuffle=False)
    b = next(dl)
    return dict(ids=torch.tensor(ids), inp=b["input_ids"], tgt=b["target_ids"], pos=b["position_ids"])


@pytest.mark.parametrize("cp,zigzag", [(1, True), (2, True), (2, False)])
def test_loader_world2_tokenizer_broadcast_and_cp_slices(tmp_path, cp, zigzag):
    from scaletorch_amd.data.loader import cp_slice_indices

    tok_dir, data = _write_corpus(str(tmp_path))
    exp = torch.from_numpy(_expected_chunks(data, 16))
    res = run_workers(_loader_worker, 2, tok_dir, data, cp, zigzag)
    for r, out in enumerate(res):
        assert out["ids"].tolist() == [5, 9, 61]
        dp_rank, cp_rank = r // cp, r % cp
        idx = cp_slice_indices(16, cp, cp_rank, zigzag)
        # DistributedSampler without shuffle: replica d gets samples d, d + dp, ...
        dp = 2 // cp
        rows = exp[[dp_rank, dp_rank + dp]]
        torch.testing.assert_close(out["inp"], rows[:, :-1][:, idx])
        torch.testing.assert_close(out["tgt"], rows[:, 1:][:, idx])
        assert out["pos"].tolist() == [idx.tolist()] * 2
    if cp == 2:  # the two CP ranks hold complementary token sets of the same samples
        both = torch.cat([res[0]["pos"][0], res[1]["pos"][0]]).sort().values
        assert both.tolist() == list(range(16))


def _train_worker(rank, world, tok_dir, data, kw):
    from scaletorch_amd.trainer.engine import Trainer

    tr = Trainer(_args(tok_dir, data, **kw))
    losses = [tr.reduced_loss(tr.train_step()) for _ in range(2)]
    return torch.tensor(losses)


@pytest.mark.slow
@pytest.mark.parametrize("kw", [dict(data_parallel_size=2), dict(context_parallel_size=2)], ids=["dp2", "cp2"])
def test_trainer_steps_on_tokenized_corpus(tmp_path, kw):
    tok_dir, data = _write_corpus(str(tmp_path))
    res = run_workers(_train_worker, 2, tok_dir, data, kw)
    for l in res:
        assert torch.isfinite(l).all() and l[0] > 0
    torch.testing.assert_close(res[0], res[1])  # the reduced loss is the same number on every rank

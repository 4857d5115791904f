"""Dataset processing: tokenizer + HF ``datasets`` (local only) + tokenize strategies.

Reference: DatasetProcessor / register_tokenize_strategy / concat_chunk
(scaletorch/data/dataset.py:28-489) and PretrainDataset
(scaletorch/data/pretrain_dataset.py).  No hub access exists here, so datasets
come from ``load_from_disk`` dirs, local json/jsonl/txt/parquet files, or a
local dataset script path; the tokenizer from a local directory.  The default
``concat_chunk`` strategy concatenates all token ids and cuts non-overlapping
chunks of ``seq_len + 1`` (targets are the shifted inputs).  The tokenizer is
built on rank 0 and broadcast (same as the reference), so only one process
touches the filesystem cache.
"""
from __future__ import annotations

import glob
import os
from typing import Callable

import numpy as np
import torch
from torch.utils.data import Dataset

from ..dist import collectives as C

_STRATEGIES: dict[str, Callable] = {}


def register_tokenize_strategy(name: str):
    def deco(fn):
        _STRATEGIES[name] = fn
        return fn
    return deco


def available_strategies() -> list[str]:
    return sorted(_STRATEGIES)


@register_tokenize_strategy("concat_chunk")
def _concat_chunk(token_lists: list[list[int]], seq_len: int, eos_id: int | None = None) -> np.ndarray:
    flat = []
    for t in token_lists:
        flat.extend(t)
        if eos_id is not None:
            flat.append(eos_id)
    n = len(flat) // (seq_len + 1)
    if n == 0:
        return np.zeros((0, seq_len + 1), dtype=np.int64)
    return np.asarray(flat[: n * (seq_len + 1)], dtype=np.int64).reshape(n, seq_len + 1)


@register_tokenize_strategy("pad_truncate")
def _pad_truncate(token_lists: list[list[int]], seq_len: int, eos_id: int | None = None, pad_id: int = 0):
    out = np.full((len(token_lists), seq_len + 1), pad_id, dtype=np.int64)
    for i, t in enumerate(token_lists):
        t = t[: seq_len + 1]
        out[i, : len(t)] = t
    return out


class TokenChunkDataset(Dataset):
    """In-memory [N, seq_len+1] int64 chunks (optionally memory-mapped .npy)."""

    def __init__(self, chunks: np.ndarray):
        self.chunks = chunks

    def __len__(self) -> int:
        return int(self.chunks.shape[0])

    def __getitem__(self, i: int) -> dict:
        # a copy: rows of a read-only memmap must not become (non-writable) tensor views
        return {"input_ids": torch.from_numpy(np.array(self.chunks[i], dtype=np.int64))}


def load_tokenizer(path: str):
    """Tokenizer built on rank 0, broadcast to the other ranks."""
    obj = [None]
    if C.get_rank() == 0:
        from transformers import AutoTokenizer

        obj[0] = AutoTokenizer.from_pretrained(path, local_files_only=True)
    C.broadcast_object_list(obj, src=0)
    return obj[0]


def _load_texts(data_path: str, dataset_name: str, subset: str | None, split: str, num_samples: int | None,
                text_field: str = "text") -> list[str]:
    import datasets

    if os.path.isdir(data_path) and os.path.exists(os.path.join(data_path, "dataset_info.json")):
        ds = datasets.load_from_disk(data_path)
        if isinstance(ds, datasets.DatasetDict):
            ds = ds[split]
    elif os.path.isdir(data_path) or os.path.isfile(data_path):
        files = [data_path] if os.path.isfile(data_path) else sorted(
            glob.glob(os.path.join(data_path, "*.json*")) + glob.glob(os.path.join(data_path, "*.txt"))
            + glob.glob(os.path.join(data_path, "*.parquet")))
        if not files:
            raise FileNotFoundError(f"no data files under {data_path}")
        ext = files[0].rsplit(".", 1)[-1]
        kind = {"jsonl": "json", "json": "json", "txt": "text", "parquet": "parquet"}[ext]
        ds = datasets.load_dataset(kind, data_files=files, split="train")
    else:
        raise FileNotFoundError(f"dataset {dataset_name!r} not found locally at {data_path} (no hub access)")
    if num_samples:
        ds = ds.select(range(min(num_samples, len(ds))))
    return [t for t in ds[text_field] if t]


class DatasetProcessor:
    def __init__(self, args, seq_len: int, strategy: str = "concat_chunk"):
        self.args, self.seq_len, self.strategy = args, seq_len, strategy
        self.tokenizer = load_tokenizer(args.tokenizer_name_or_path)

    def tokenize_dataset(self) -> TokenChunkDataset:
        a = self.args
        texts = _load_texts(a.data_path, a.dataset_name, a.subset_name, a.split, a.num_samples)
        ids = self.tokenizer(texts, add_special_tokens=False)["input_ids"]
        eos = getattr(self.tokenizer, "eos_token_id", None)
        return TokenChunkDataset(_STRATEGIES[self.strategy](ids, self.seq_len, eos))


def build_dataset(args, seq_len: int) -> Dataset:
    """Pre-tokenized ``.npy`` ([N, seq+1] int64, memory-mapped) or raw text + local tokenizer."""
    p = args.data_path
    if p.endswith(".npy") and os.path.isfile(p):
        return TokenChunkDataset(np.load(p, mmap_mode="r"))
    return DatasetProcessor(args, seq_len).tokenize_dataset()


class PretrainDataset(Dataset):
    """Local JSON/JSONL text -> tokenized, padded to ``max_length`` (reference pretrain_dataset.py:13-107)."""

    def __init__(self, path: str, tokenizer, max_length: int = 512, text_field: str = "text"):
        import json

        self.samples = []
        with open(path) as f:
            if path.endswith(".jsonl"):
                self.samples = [json.loads(line)[text_field] for line in f if line.strip()]
            else:
                data = json.load(f)
                self.samples = [d[text_field] for d in data]
        self.tok, self.max_length = tokenizer, max_length

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, i: int) -> dict:
        enc = self.tok(self.samples[i], max_length=self.max_length, truncation=True, padding="max_length",
                       return_tensors="pt")
        ids = enc["input_ids"][0]
        mask = enc["attention_mask"][0]
        labels = ids.clone()
        labels[mask == 0] = -100
        return {"input_ids": ids, "attention_mask": mask, "labels": labels}

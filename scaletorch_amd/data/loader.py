"""Micro-batch data loading with DP/EP sharding and context-parallel slicing.

Reference: MicroBatchDataLoader (scaletorch/data/dataloader.py:16-292).
Behaviour kept: a DistributedSampler over data-parallel replicas, targets
shifted by one, global ``position_ids``, a ``gradient_accumulation_steps``
attribute read by the pipeline schedules, epoch advance on exhaustion.
Changes: EP ranks are data-parallel replicas too (mesh.data_rank), and the
context-parallel slice is either contiguous (reference) or ZIG-ZAG -- the
sequence is cut into 2*cp chunks and rank r keeps chunks r and 2cp-1-r, which
balances causal-attention work across the CP ring.
"""
from __future__ import annotations

import math

import torch
from torch.utils.data import DataLoader, Dataset, DistributedSampler


class SyntheticTokenDataset(Dataset):
    """Deterministic random token sequences of length ``seq_len + 1`` (per-index seed)."""

    def __init__(self, vocab_size: int, seq_len: int, num_samples: int = 1 << 20, seed: int = 1234):
        self.vocab_size, self.seq_len = vocab_size, seq_len
        self.num_samples, self.seed = num_samples, seed

    def __len__(self) -> int:
        return self.num_samples

    def __getitem__(self, i: int) -> dict:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return {"input_ids": torch.randint(0, self.vocab_size, (self.seq_len + 1,), generator=g)}


def cp_slice_indices(seq_len: int, cp_size: int, cp_rank: int, zigzag: bool) -> torch.Tensor:
    """Token indices (into the length-``seq_len`` sequence) owned by one CP rank."""
    if cp_size == 1:
        return torch.arange(seq_len)
    if not zigzag:
        n = seq_len // cp_size
        return torch.arange(cp_rank * n, (cp_rank + 1) * n)
    if seq_len % (2 * cp_size):
        raise ValueError(f"zig-zag CP needs seq_len % (2*cp) == 0 (seq {seq_len}, cp {cp_size})")
    c = seq_len // (2 * cp_size)
    a = torch.arange(cp_rank * c, (cp_rank + 1) * c)
    b = torch.arange((2 * cp_size - 1 - cp_rank) * c, (2 * cp_size - cp_rank) * c)
    return torch.cat([a, b])


class Collator:
    def __init__(self, seq_len: int, cp_size: int = 1, cp_rank: int = 0, zigzag: bool = True):
        self.seq_len, self.cp_size, self.cp_rank, self.zigzag = seq_len, cp_size, cp_rank, zigzag
        self.idx = cp_slice_indices(seq_len, cp_size, cp_rank, zigzag)

    def __call__(self, batch: list[dict]) -> dict:
        ids = torch.stack([torch.as_tensor(b["input_ids"])[: self.seq_len + 1] for b in batch]).long()
        if ids.shape[1] < self.seq_len + 1:
            raise ValueError(f"sample length {ids.shape[1]} < seq_len+1 ({self.seq_len + 1})")
        inp, tgt = ids[:, :-1], ids[:, 1:]
        pos = self.idx.unsqueeze(0).expand(ids.shape[0], -1).contiguous()
        return {"input_ids": inp[:, self.idx].contiguous(), "target_ids": tgt[:, self.idx].contiguous(),
                "position_ids": pos, "hidden_states": None}


class _ResumableSampler(torch.utils.data.Sampler):
    """DistributedSampler whose next iteration starts ``skip`` samples into the epoch
    (resume from a checkpoint mid-epoch without replaying the consumed samples)."""

    def __init__(self, inner: DistributedSampler):
        self.inner, self.skip = inner, 0

    def __iter__(self):
        it = iter(self.inner)
        for _ in range(self.skip):
            next(it, None)
        self.skip = 0
        return it

    def __len__(self) -> int:
        return len(self.inner)

    def set_epoch(self, epoch: int) -> None:
        self.inner.set_epoch(epoch)


class MicroBatchDataLoader(DataLoader):
    def __init__(self, dataset: Dataset, micro_batch_size: int, seq_len: int, grad_acc_steps: int = 1,
                 data_rank: int = 0, data_world_size: int = 1, cp_rank: int = 0, cp_size: int = 1,
                 zigzag: bool = True, shuffle: bool = True, seed: int = 1, num_workers: int = 0,
                 pin_memory: bool = False, drop_last: bool = True):
        self.micro_batch_size, self.seq_len = micro_batch_size, seq_len
        self.gradient_accumulation_steps = grad_acc_steps
        self.global_batch_size = micro_batch_size * grad_acc_steps * data_world_size
        self.sampler_ = _ResumableSampler(DistributedSampler(dataset, num_replicas=data_world_size, rank=data_rank,
                                                             shuffle=shuffle, seed=seed, drop_last=drop_last))
        self.collator = Collator(seq_len, cp_size, cp_rank, zigzag)
        super().__init__(dataset, batch_size=micro_batch_size, sampler=self.sampler_, collate_fn=self.collator,
                         num_workers=num_workers, pin_memory=pin_memory, drop_last=drop_last,
                         persistent_workers=num_workers > 0)
        self.epoch = 0
        self._it = None

    def __next__(self) -> dict:
        if self._it is None:
            self._it = super().__iter__()
        try:
            return next(self._it)
        except StopIteration:
            self.epoch += 1
            self.sampler_.set_epoch(self.epoch)
            self._it = super().__iter__()
            return next(self._it)

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
        self.sampler_.set_epoch(epoch)
        self._it = None

    def skip_batches(self, n: int) -> None:
        """Position the loader after ``n`` consumed micro-batches (checkpoint resume)."""
        per_epoch = max(1, len(self.sampler_) // self.micro_batch_size)
        self.set_epoch(n // per_epoch)
        self.sampler_.skip = (n % per_epoch) * self.micro_batch_size


class DeviceSyntheticLoader:
    """Synthetic batches generated directly on the device (benchmarks): no host
    work or H2D copies inside the timed loop.  Same batch contract as
    MicroBatchDataLoader."""

    def __init__(self, vocab_size: int, micro_batch_size: int, seq_len: int, device, grad_acc_steps: int = 1,
                 cp_size: int = 1, cp_rank: int = 0, zigzag: bool = True, seed: int = 1234,
                 data_rank: int = 0):
        self.vocab_size, self.mbs, self.seq_len = vocab_size, micro_batch_size, seq_len
        self.gradient_accumulation_steps = grad_acc_steps
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device).manual_seed(seed + 7919 * data_rank)
        self.idx = cp_slice_indices(seq_len, cp_size, cp_rank, zigzag).to(self.device)
        self.pos = self.idx.unsqueeze(0).expand(micro_batch_size, -1).contiguous()

    def __iter__(self):
        return self

    def skip_batches(self, n: int) -> None:
        for _ in range(n):
            torch.randint(0, self.vocab_size, (self.mbs, self.seq_len + 1), device=self.device, generator=self.gen)

    def __next__(self) -> dict:
        ids = torch.randint(0, self.vocab_size, (self.mbs, self.seq_len + 1), device=self.device, generator=self.gen)
        return {"input_ids": ids[:, :-1][:, self.idx].contiguous(), "target_ids": ids[:, 1:][:, self.idx].contiguous(),
                "position_ids": self.pos, "hidden_states": None}

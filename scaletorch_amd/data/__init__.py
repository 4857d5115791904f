"""Data: synthetic / HF datasets, DP/EP sharded micro-batch loader with CP slicing."""
from .loader import (Collator, DeviceSyntheticLoader, MicroBatchDataLoader, SyntheticTokenDataset,
                     cp_slice_indices)

__all__ = ["Collator", "DeviceSyntheticLoader", "MicroBatchDataLoader", "SyntheticTokenDataset",
           "cp_slice_indices"]

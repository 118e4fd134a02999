"""Synthetic datasets, partitioners and packed (varlen) batching.

There is no network for HF datasets, so every dataset of the reference is replaced by a
synthetic token-id dataset of the same *shape* (row counts, class count, length distribution,
label order) with a planted, learnable label signal.
"""
from .registry import DATASETS, DatasetSpec, get_dataset, load_split
from .synthetic import TokenDataset, make_synthetic_split
from .partition import partition_clients, ClientSplit
from .batching import PackedBatch, PaddedBatch, ClientLoader, make_packed_batch, make_padded_batch

__all__ = [
    "DATASETS", "DatasetSpec", "get_dataset", "load_split", "TokenDataset", "make_synthetic_split",
    "partition_clients", "ClientSplit", "PackedBatch", "PaddedBatch", "ClientLoader",
    "make_packed_batch", "make_padded_batch",
]

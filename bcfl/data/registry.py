"""Dataset registry: synthetic stand-ins with the shapes of the reference's HF datasets.

Reference datasets: ``imdb`` (text->label, 2 classes, 25k/25k, label-sorted),
``bhargavi909/Medical_Transcriptions_upsampled`` (description->medical_specialty, 40 classes;
local CSV copy 12000/3000 rows, descriptions ≈17.6 words), ``bhargavi909/cancer_classification``
(input->label, 5408/1352 rows per ``serverless_cancer_classification_with_BioBERT.ipynb:424-431``),
``bhargavi909/covid_final`` (text->sentiment). Length medians are in *wordpiece tokens*.
"""
from __future__ import annotations

import functools
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

from .synthetic import TokenDataset, make_synthetic_split

__all__ = ["DatasetSpec", "DATASETS", "get_dataset", "load_split"]


@dataclass(frozen=True)
class DatasetSpec:
    name: str
    num_classes: int
    n_train: int
    n_test: int
    length_median: float
    length_sigma: float
    ref_train_stride: int       # reference contiguous-shard stride (load_data_clients)
    ref_train_len: int
    ref_test_from_train_stride: bool  # IMDB: test shard follows train shard inside the stride
    description: str


DATASETS: Dict[str, DatasetSpec] = {
    # IMDB reviews: ≈230 median wordpieces, long tail truncated at 512
    "imdb": DatasetSpec("imdb", 2, 25000, 25000, 230.0, 0.65, 300, 240, True,
                        "synthetic IMDB-shaped sentiment (2 classes, label-sorted)"),
    "medical": DatasetSpec("medical", 40, 12000, 3000, 28.0, 0.45, 500, 400, False,
                           "synthetic Medical-Transcriptions-shaped (40 specialties)"),
    "cancer": DatasetSpec("cancer", 3, 5408, 1352, 180.0, 0.6, 500, 400, False,
                          "synthetic cancer_classification-shaped (3 classes)"),
    "covid": DatasetSpec("covid", 3, 8000, 2000, 40.0, 0.5, 500, 400, False,
                         "synthetic covid_final-shaped sentiment (3 classes)"),
    # tiny split for unit tests
    "tiny": DatasetSpec("tiny", 2, 512, 256, 24.0, 0.4, 40, 32, True, "tiny test split"),
    # REAL text from the reference's local CSVs, WordPiece trained offline
    # (bcfl.data.text); shard strides follow the medical scripts (Serverless_NonIID_Medical:55-56)
    "medical_csv": DatasetSpec("medical_csv", 40, 12000, 3000, 28.0, 0.45, 500, 400, False,
                               "Medical Transcriptions CSV (reference Dataset/*_mt.csv), real text"),
    "selfdriving_csv": DatasetSpec("selfdriving_csv", 3, 400, 100, 12.0, 0.3, 40, 32, False,
                                   "self-driving sentiment CSV (reference Dataset/), real text"),
}

TEXT_DATASETS = ("medical_csv", "selfdriving_csv")


def get_dataset(name: str) -> DatasetSpec:
    if name not in DATASETS:
        raise KeyError(f"unknown dataset {name!r}; known {sorted(DATASETS)}")
    return DATASETS[name]


@functools.lru_cache(maxsize=16)
def load_split(name: str, split: str, vocab_size: int, max_len: int = 512, seed: int = 1234,
               cls_id: int = 101, sep_id: int = 102,
               signal: Optional[float] = None) -> TokenDataset:
    """``signal``: planted own-class tokens per 64 body tokens (None = generator default 3.0;
    other-class tokens stay at 1.0 per 64) — the difficulty knob of the synthetic task."""
    spec = get_dataset(name)
    if name in TEXT_DATASETS:
        from .text import load_csv_split
        return load_csv_split(name, split, vocab_size, max_len, cls_id, sep_id)
    n = spec.n_train if split == "train" else spec.n_test
    split_seed = seed * 7919 + (0 if split == "train" else 1)
    kw = {} if signal is None else {"own_signal_rate": float(signal)}
    return make_synthetic_split(n, spec.num_classes, vocab_size, seed=split_seed,
                                length_median=spec.length_median, length_sigma=spec.length_sigma,
                                max_len=max_len, cls_id=cls_id, sep_id=sep_id, class_seed=seed,
                                **kw)


def splits(name: str, vocab_size: int, max_len: int = 512, seed: int = 1234,
           cls_id: int = 101, sep_id: int = 102) -> Tuple[TokenDataset, TokenDataset]:
    return (load_split(name, "train", vocab_size, max_len, seed, cls_id, sep_id),
            load_split(name, "test", vocab_size, max_len, seed, cls_id, sep_id))

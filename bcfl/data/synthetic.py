"""Synthetic token-id datasets with a planted label signal.

Each class ``c`` owns a small set of "sentiment" token ids. A sample of class ``c`` is a
``[CLS] body [SEP]`` sequence whose body is Zipf-like background vocabulary with a few of its own
class tokens and fewer tokens of other classes mixed in, so the label is recoverable by counting
(a bag-of-words task a transformer learns quickly). Rows are stored label-sorted, like HF
``imdb`` (which is why the reference's contiguous Non-IID shards are single-class: SURVEY.md A.1).

Storage is packed: ``tokens`` (int32, all rows back to back) + ``offsets`` (N+1) + ``labels``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

__all__ = ["TokenDataset", "make_synthetic_split"]


@dataclass
class TokenDataset:
    tokens: np.ndarray    # int32 [sum(len)]
    offsets: np.ndarray   # int64 [N+1]
    labels: np.ndarray    # int64 [N]
    num_classes: int
    vocab_size: int

    def __len__(self) -> int:
        return int(self.labels.shape[0])

    @property
    def lengths(self) -> np.ndarray:
        return np.diff(self.offsets)

    def row(self, i: int) -> np.ndarray:
        return self.tokens[self.offsets[i]:self.offsets[i + 1]]

    def mean_length(self) -> float:
        return float(self.lengths.mean()) if len(self) else 0.0


def _lengths(rng: np.random.Generator, n: int, median: float, sigma: float,
             min_len: int, max_len: int) -> np.ndarray:
    raw = rng.lognormal(mean=np.log(median), sigma=sigma, size=n)
    return np.clip(np.round(raw), min_len, max_len).astype(np.int64)


def make_synthetic_split(n: int, num_classes: int, vocab_size: int, *, seed: int,
                         length_median: float, length_sigma: float, max_len: int = 512,
                         min_len: int = 8, cls_id: int = 101, sep_id: int = 102,
                         content_lo: int = 1000, signal_tokens_per_class: int = 24,
                         own_signal_rate: float = 3.0, other_signal_rate: float = 1.0,
                         class_seed: Optional[int] = None,
                         class_probs: Optional[Sequence[float]] = None) -> TokenDataset:
    """Generate one label-sorted split. ``class_seed`` fixes the per-class signal vocabulary so
    train and test splits share it (it defaults to ``seed``)."""
    rng = np.random.default_rng(seed)
    crng = np.random.default_rng(seed if class_seed is None else class_seed)
    content_lo = min(content_lo, max(4, vocab_size // 4))
    span = vocab_size - content_lo
    sig = crng.choice(span, size=(num_classes, signal_tokens_per_class), replace=False) + content_lo

    # label-sorted classes
    if class_probs is None:
        counts = np.full(num_classes, n // num_classes, dtype=np.int64)
        counts[: n - counts.sum()] += 1
    else:
        p = np.asarray(class_probs, dtype=np.float64)
        counts = np.floor(p / p.sum() * n).astype(np.int64)
        counts[: n - counts.sum()] += 1
    labels = np.repeat(np.arange(num_classes, dtype=np.int64), counts)

    lengths = _lengths(rng, n, length_median, length_sigma, min_len, max_len)
    offsets = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lengths, out=offsets[1:])
    total = int(offsets[-1])

    # Zipf-like background: u^3 concentrates mass on low content ids
    u = rng.random(total)
    tokens = (content_lo + np.floor((u ** 3) * span)).astype(np.int64)

    # plant class signal tokens at random body positions
    body = np.maximum(lengths - 2, 1)
    n_own = 1 + rng.poisson(own_signal_rate * np.minimum(body, 128) / 64.0)
    n_oth = rng.poisson(other_signal_rate * np.minimum(body, 128) / 64.0)
    for n_each, own in ((n_own, True), (n_oth, False)):
        rows = np.repeat(np.arange(n), n_each)
        if rows.size == 0:
            continue
        pos = offsets[rows] + 1 + np.floor(rng.random(rows.size) * body[rows]).astype(np.int64)
        if own:
            cls = labels[rows]
        else:
            shift = rng.integers(1, max(num_classes, 2), size=rows.size)
            cls = (labels[rows] + shift) % num_classes
        pick = rng.integers(0, signal_tokens_per_class, size=rows.size)
        tokens[pos] = sig[cls, pick]
    tokens[offsets[:-1]] = cls_id
    tokens[offsets[1:] - 1] = sep_id
    return TokenDataset(tokens=tokens.astype(np.int32), offsets=offsets, labels=labels,
                        num_classes=num_classes, vocab_size=vocab_size)

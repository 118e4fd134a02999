"""Client partitioners.

* ``iid_random``      — independent random draw per client (ref ``load_data()``,
                        ``src/Serverlesscase/serverless_IID_IMDB.py:46-82``; the reference draw is
                        unseeded ``random.sample``, here it is seeded by (seed, client, round)).
* ``shared_random``   — ONE random draw shared by every client (ref server case: ``client_fn``
                        returns the same loaders for every cid, ``src/Servercase/server_IID_IMDB.py:188-190``).
* ``ref_contiguous``  — the reference's contiguous shards of the *unshuffled* split
                        (``src/Serverlesscase/serverless_NonIID_IMDB.py:59-60``: train
                        ``[300k, 300k+240)``, test ``[300k+240, 300(k+1))``; medical
                        ``Serverless_NonIID_Medical_transcriptions.py:55-56``: train
                        ``[500k, 500k+400)``, test ``[0, 400)``). On label-sorted IMDB every
                        shard is single-class label 0 — reproduced on purpose.
* ``ref_shared_prefix`` — reference ``load_data_count(0)`` of ``server_NonIID_IMDB.py:65-101``:
                        the split is SHUFFLED once (``.shuffle(seed=42)``, :68) and EVERY client gets
                        the same rows — train ``[0, 240)``, test ``[240, 300)`` (:83-84, called once
                        at :224, ``client_fn`` returns the same loaders for every cid) — so the
                        script named "NonIID" is in fact IID with shared data. Reproduced on purpose.
* ``label_shards``    — pathological Non-IID spread over the whole label-sorted split: shard k is
                        the head of the k-th of ``num_clients`` equal contiguous blocks, so clients
                        see different single classes (what a Non-IID benchmark intends).
* ``dirichlet``       — per-class Dirichlet(alpha) proportions (standard FL Non-IID).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from .registry import DatasetSpec

__all__ = ["ClientSplit", "partition_clients", "global_test_indices", "majority_rate"]


@dataclass
class ClientSplit:
    train: np.ndarray
    test: np.ndarray


def _rng(seed: int, *salt: int) -> np.random.Generator:
    return np.random.default_rng([seed, *salt])


def _dirichlet(labels: np.ndarray, num_clients: int, per_client: int, alpha: float,
               rng: np.random.Generator) -> List[np.ndarray]:
    classes = np.unique(labels)
    by_cls = {c: rng.permutation(np.flatnonzero(labels == c)) for c in classes}
    ptr = {c: 0 for c in classes}
    out = []
    for _ in range(num_clients):
        p = rng.dirichlet(np.full(len(classes), alpha))
        counts = np.floor(p * per_client).astype(int)
        counts[: per_client - counts.sum()] += 1
        idx = []
        for c, k in zip(classes, counts):
            pool = by_cls[c]
            take = [pool[(ptr[c] + j) % len(pool)] for j in range(k)]
            ptr[c] = (ptr[c] + k) % len(pool)
            idx.extend(take)
        out.append(np.asarray(sorted(idx), dtype=np.int64))
    return out


def partition_clients(kind: str, spec: DatasetSpec, train_labels: np.ndarray,
                      test_labels: np.ndarray, num_clients: int, train_samples: int,
                      test_samples: int, seed: int = 42, round_idx: int = 0,
                      alpha: float = 0.5) -> List[ClientSplit]:
    n_tr, n_te = len(train_labels), len(test_labels)
    tr_k = min(train_samples, n_tr)
    te_k = min(test_samples, n_te)
    splits: List[ClientSplit] = []
    if kind == "iid_random":
        for k in range(num_clients):
            r = _rng(seed, k, round_idx)
            splits.append(ClientSplit(np.sort(r.choice(n_tr, tr_k, replace=False)),
                                      np.sort(r.choice(n_te, te_k, replace=False))))
    elif kind == "shared_random":
        r = _rng(seed, 0, round_idx)
        tr = np.sort(r.choice(n_tr, tr_k, replace=False))
        te = np.sort(r.choice(n_te, te_k, replace=False))
        splits = [ClientSplit(tr, te) for _ in range(num_clients)]
    elif kind == "ref_contiguous":
        stride, ln = spec.ref_train_stride, spec.ref_train_len
        for k in range(num_clients):
            lo = (stride * k) % max(n_tr - ln, 1)
            tr = np.arange(lo, lo + ln) % n_tr
            if spec.ref_test_from_train_stride:
                te = np.arange(lo + ln, lo + stride) % n_te
            else:
                te = np.arange(0, min(ln, n_te))
            splits.append(ClientSplit(tr.astype(np.int64), te.astype(np.int64)))
    elif kind == "ref_shared_prefix":
        r = _rng(seed, 4242)
        stride, ln = spec.ref_train_stride, spec.ref_train_len
        ptr, pte = r.permutation(n_tr), r.permutation(n_te)
        tr = np.sort(ptr[:min(ln, n_tr)]).astype(np.int64)
        te = np.sort(pte[ln:min(stride, n_te)]).astype(np.int64)
        splits = [ClientSplit(tr, te) for _ in range(num_clients)]
    elif kind == "label_shards":
        for k in range(num_clients):
            blk_tr = n_tr // num_clients
            blk_te = n_te // num_clients
            lo_tr, lo_te = k * blk_tr, k * blk_te
            tr = np.arange(lo_tr, lo_tr + min(tr_k, blk_tr))
            te = np.arange(lo_te, lo_te + min(te_k, blk_te))
            splits.append(ClientSplit(tr.astype(np.int64), te.astype(np.int64)))
    elif kind == "dirichlet":
        r = _rng(seed, 99, round_idx)
        trs = _dirichlet(train_labels, num_clients, tr_k, alpha, r)
        tes = _dirichlet(test_labels, num_clients, te_k, alpha, r)
        splits = [ClientSplit(a, b) for a, b in zip(trs, tes)]
    else:
        raise KeyError(f"unknown partition {kind!r}")
    return splits


def global_test_indices(n_test: int, k: int, seed: int, round_idx: Optional[int] = None,
                        labels: Optional[np.ndarray] = None) -> np.ndarray:
    """Global-eval draw (ref ``load_data()`` test sample, ``serverless_NonIID_IMDB.py:300-302``).

    The reference draws ``random.sample`` from the *shuffled* HF split, so its draw is balanced in
    expectation. Our splits are stored label-sorted, and a small uniform draw can be lopsided (a
    fixed 100-row draw is 61/39 on synthetic IMDB, so a constant predictor scores 0.61). With
    ``labels`` the draw is **stratified**: each class contributes ``k / num_classes`` rows (the
    remainder goes to the lowest class ids), so the majority-class rate is ``ceil(k/C)/k``."""
    r = _rng(seed, 7777, 0 if round_idx is None else round_idx + 1)
    k = min(k, n_test)
    if labels is None:
        return np.sort(r.choice(n_test, k, replace=False))
    labels = np.asarray(labels)
    classes = np.unique(labels)
    per = np.full(len(classes), k // len(classes), dtype=np.int64)
    per[: k - per.sum()] += 1
    out = []
    for c, m in zip(classes, per):
        pool = np.flatnonzero(labels == c)
        out.append(r.choice(pool, min(int(m), len(pool)), replace=False))
    return np.sort(np.concatenate(out)).astype(np.int64)


def majority_rate(labels: np.ndarray, idx: np.ndarray) -> float:
    """Accuracy of the best constant predictor on ``labels[idx]`` (what an untrained model
    that collapsed onto one class scores)."""
    if len(idx) == 0:
        return 0.0
    return float(np.bincount(np.asarray(labels)[idx]).max() / len(idx))

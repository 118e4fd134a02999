"""Anomaly filtering inside the training path ("mitigating node anomalies", reference README:10).

Two filters:

* :class:`UpdateAnomalyFilter` — per round, over the client UPDATES. Each client sketches its
  update (signed block sketch, GPU kernel, 8192 floats) and the sketches are all-gathered; a
  cosine-similarity graph of the sketches is ranked with PageRank (the reference's detector,
  ``All_graphs_IMDB_dataset.ipynb:168-180``) and clients below ``mu - k*sigma`` are rejected
  (sign-flipped / random updates have low similarity to everybody). Update norms go through the
  modified Z-score (``:362-366``) which catches scaled (boosted) updates that cosine cannot see.
* :func:`topology_filter` — at start-up, over the measured LINK graph (weight = 1/bandwidth, as
  N1): PageRank outliers are removed from the gossip neighbour sets.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Set

import numpy as np

from . import graph as G


@dataclass
class Verdicts:
    rejected: Set[int] = field(default_factory=set)
    pagerank: List[float] = field(default_factory=list)
    modz: List[float] = field(default_factory=list)
    reasons: Dict[int, str] = field(default_factory=dict)

    def verdict(self, c: int) -> str:
        return "reject:" + self.reasons[c] if c in self.rejected else "accept"


class UpdateAnomalyFilter:
    def __init__(self, method: str = "both", k: float = 2.0, modz_threshold: float = 3.5,
                 min_clients: int = 4, mad_floor: float = 0.5):
        self.method, self.k, self.thr, self.min_clients = method, k, modz_threshold, min_clients
        # honest updates of one round can have almost equal norms (MAD ~1-2 % of the median): the
        # modified Z of a plain 15 % difference then exceeds 3.5 and an honest client is rejected
        # (tiny-bert, 8 label-shard clients: client 0 rejected in 7 of 16 rounds, the federation
        # stalled at the majority rate); and label-shard clients' norms are bimodal by class (2x
        # apart), so with one client gone the median sits in one class and the other is flagged.
        # The MAD is floored at mad_floor x the median norm: with 0.5 only updates more than
        # ~2.6x the median norm's distance count (a 50x boost: z ~ 66; a 2x class gap: z ~ 1.3)
        self.mad_floor = float(mad_floor)

    def __call__(self, sketches: np.ndarray, norms: Sequence[float]) -> Verdicts:
        n = sketches.shape[0]
        v = Verdicts()
        if self.method == "none":
            return v
        norms = np.asarray(norms, dtype=np.float64)
        bad = ~np.isfinite(norms) | ~np.isfinite(sketches).all(axis=1)
        if bad.any():
            # a non-finite update can never be applied (one NaN poisons every model it enters):
            # always rejected, whatever the majority rule says; the rest are judged on their own
            ok = np.flatnonzero(~bad)
            sub = self(sketches[ok], norms[ok]) if len(ok) else Verdicts()
            v.rejected = {int(ok[i]) for i in sub.rejected}
            v.reasons = {int(ok[i]): r for i, r in sub.reasons.items()}
            for i in np.flatnonzero(bad):
                v.rejected.add(int(i))
                v.reasons[int(i)] = "non-finite"
            return v
        if n < self.min_clients:
            return v
        S = sketches.astype(np.float64)
        nrm = np.linalg.norm(S, axis=1, keepdims=True)
        S = S / np.maximum(nrm, 1e-30)
        C = S @ S.T
        A = np.clip(C, 0.0, None)
        np.fill_diagonal(A, 0.0)
        if self.method in ("pagerank", "both"):
            if A.sum() > 0:
                r = G.pagerank(A)
                v.pagerank = [float(x) for x in r]
                (lo, _), flags = G.sigma_flags(r, self.k, low_only=True)
                mu = float(np.mean(r))
                for i in flags:
                    if (mu - r[i]) / max(mu, 1e-30) > 0.05:
                        v.rejected.add(i)
                        v.reasons[i] = "pagerank"
            # a node with no positive similarity to anyone is isolated (dangling in A)
            for i in range(n):
                if A[i].sum() == 0 and A[:, i].sum() == 0:
                    v.rejected.add(i)
                    v.reasons.setdefault(i, "isolated")
        if self.method in ("modz", "both"):
            med = float(np.median(norms))
            mad = float(np.median(np.abs(norms - med)))
            floor = self.mad_floor * abs(med)
            z = (G.modified_z(list(norms)) if mad >= floor or floor == 0.0
                 else 0.6745 * (norms - med) / floor)
            v.modz = [float(x) for x in z]
            for i, s in enumerate(z):
                if not np.isnan(s) and abs(s) > self.thr:  # MAD = 0 -> ±inf for any deviation
                    v.rejected.add(i)
                    v.reasons.setdefault(i, "modz")
        # never reject a majority: keep the filter from isolating the honest set
        if len(v.rejected) * 2 >= n:
            v.rejected.clear()
            v.reasons.clear()
        return v


def topology_filter(bw: np.ndarray, k: float = 2.0, rel: float = 0.05) -> List[int]:
    """PageRank over a measured bandwidth matrix (weights 1/bw, reference N1/N2); returns the
    low-side outliers whose rank deviates by more than ``rel`` of the mean."""
    W = np.zeros_like(bw, dtype=np.float64)
    nz = bw > 0
    W[nz] = 1.0 / bw[nz]
    if W.sum() == 0:
        return []
    r = G.pagerank(W)
    (lo, hi), flags = G.sigma_flags(r, k, low_only=False)
    mu = float(np.mean(r))
    return [i for i in flags if abs(r[i] - mu) / max(mu, 1e-30) > rel]

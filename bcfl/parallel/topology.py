"""Client topologies and mixing matrices for serverless gossip.

The reference's serverless "P2P" is an all-to-all unweighted mean of every client's snapshot
(``avg_params = [sum(param)/len(param) ...]``, ``src/Serverlesscase/serverless_NonIID_IMDB.py:296``)
-> topology ``full`` with ``average`` mixing reproduces it exactly. ``ring`` and the
PageRank-filtered ``pagerank`` topology (nodes flagged by the trust layer removed from everybody's
neighbour set, N2 in SURVEY.md §2.3) are the decentralised variants the paper describes.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Set

import numpy as np


def neighbours(kind: str, n: int, excluded: Optional[Iterable[int]] = None) -> Dict[int, List[int]]:
    ex: Set[int] = set(excluded or ())
    live = [i for i in range(n) if i not in ex]
    out: Dict[int, List[int]] = {}
    for i in range(n):
        if kind in ("full", "pagerank"):
            out[i] = [j for j in live if j != i]
        elif kind == "ring":
            if len(live) <= 1:
                out[i] = []
                continue
            if i in ex:  # an excluded node still listens to its ring neighbours among live nodes
                pos = np.searchsorted(live, i) % len(live)
                out[i] = sorted({live[pos - 1], live[pos % len(live)]} - {i})
                continue
            k = live.index(i)
            out[i] = sorted({live[(k - 1) % len(live)], live[(k + 1) % len(live)]} - {i})
        else:
            raise KeyError(f"unknown topology {kind!r}")
    return out


def mixing_matrix(nbrs: Dict[int, List[int]], mode: str = "average",
                  rejected: Optional[Iterable[int]] = None) -> np.ndarray:
    """Row i = weights client i applies to [its own state, neighbour states].

    ``average``    uniform over the closed neighbourhood (row-stochastic; = reference mean on ``full``)
    ``metropolis`` Metropolis-Hastings weights (doubly stochastic -> consensus on the true mean)
    Rejected clients get zero weight in every OTHER row; their own row re-averages their honest
    neighbours (a rejected client is pulled back to consensus, not isolated).
    """
    n = len(nbrs)
    rej: Set[int] = set(rejected or ())
    W = np.zeros((n, n), dtype=np.float64)
    deg = {i: len(v) for i, v in nbrs.items()}
    for i in range(n):
        cand = [j for j in nbrs[i] if j not in rej]
        if mode == "average":
            members = ([i] if i not in rej else []) + cand
            if not members:
                members = [i]
            for j in members:
                W[i, j] = 1.0 / len(members)
        elif mode == "metropolis":
            for j in cand:
                W[i, j] = 1.0 / (1.0 + max(deg[i], deg[j]))
            if i in rej and cand:
                W[i] /= W[i].sum()
            else:
                W[i, i] = 1.0 - W[i].sum()
        else:
            raise KeyError(f"unknown mixing {mode!r}")
    return W


def client_rank(client: int, world: int) -> int:
    """Virtual client -> owning rank (round-robin, so 5/10/20 clients spread over 8 GPUs)."""
    return client % world


def clients_of_rank(rank: int, world: int, num_clients: int) -> List[int]:
    return [c for c in range(num_clients) if client_rank(c, world) == rank]

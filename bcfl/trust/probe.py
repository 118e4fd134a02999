"""Measured link-bandwidth probe -> topology anomaly filter.

The reference models the P2P network as a static 10-node digraph whose edge weights are
``1 / bandwidth_Mbps`` typed into the notebook (``All_graphs_IMDB_dataset.ipynb:73-167``, N1) and
flags nodes whose PageRank leaves ``[mu - sigma, mu + sigma]`` (``:168-180``, N2). Here the graph is
MEASURED on the running job: every ordered rank pair exchanges a buffer over RCCL (xGMI on one
MI355X node; gloo on CPU), the bandwidth matrix is all-gathered, and the same PageRank rule
(with a relative-deviation floor so that a uniform xGMI mesh's noise never evicts healthy peers)
selects ranks whose clients are dropped from the gossip neighbour sets.

Schedule: the circle method pairs the ranks into ``world - 1`` (even world) rounds of disjoint
pairs; each pair runs a bidirectional grouped send/recv, so every xGMI link is measured in both
directions while the other links of the round are busy too — the regime gossip runs in.
"""
from __future__ import annotations

import time
from typing import List, Sequence, Tuple

import numpy as np
import torch

from ..parallel import dist as D
from ..parallel.topology import clients_of_rank
from .anomaly import topology_filter


def round_robin_pairs(world: int) -> List[List[Tuple[int, int]]]:
    """Circle-method tournament: rounds of disjoint (a, b) pairs covering every unordered pair
    exactly once (a bye slot is added for odd ``world``)."""
    n = world + (world % 2)
    ids = list(range(n))
    rounds = []
    for _ in range(n - 1):
        pairs = []
        for i in range(n // 2):
            a, b = ids[i], ids[n - 1 - i]
            if a < world and b < world:
                pairs.append((min(a, b), max(a, b)))
        rounds.append(pairs)
        ids = [ids[0]] + [ids[-1]] + ids[1:-1]
    return rounds


def _timed_exchange(buf: torch.Tensor, rbuf: torch.Tensor, peer: int, iters: int) -> float:
    """Seconds per bidirectional exchange of ``buf`` with ``peer`` (median of ``iters``)."""
    ts = []
    for _ in range(iters):
        if buf.is_cuda:
            torch.cuda.synchronize(buf.device)
        t0 = time.perf_counter()
        D.p2p_exchange([(buf, peer)], [(rbuf, peer)]).wait()
        if buf.is_cuda:
            torch.cuda.synchronize(buf.device)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def measure_bandwidth(nbytes: int = 64 << 20, iters: int = 3, device=None) -> np.ndarray:
    """[world, world] matrix of measured one-direction bandwidth in MB/s (0 on the diagonal),
    identical on every rank. ``nbytes`` per message; one warm-up exchange per pair."""
    rt = D.runtime()
    w, me = rt.world, rt.rank
    dev = device if device is not None else rt.device
    n = max(nbytes // 4, 1)
    buf = torch.ones(n, dtype=torch.float32, device=dev)
    rbuf = torch.empty_like(buf)
    row = np.zeros(w, dtype=np.float64)
    for pairs in round_robin_pairs(w):
        peer = None
        for a, b in pairs:
            if me == a:
                peer = b
            elif me == b:
                peer = a
        if peer is not None:
            _timed_exchange(buf, rbuf, peer, 1)  # warm-up (communicator / link setup)
            t = _timed_exchange(buf, rbuf, peer, iters)
            row[peer] = (n * 4) / max(t, 1e-9) / 1e6
        D.barrier()
    rows = D.all_gather_object(row.tolist())
    return np.asarray(rows, dtype=np.float64)


def ranks_to_clients(ranks: Sequence[int], world: int, num_clients: int) -> List[int]:
    out: List[int] = []
    for r in ranks:
        out += clients_of_rank(r, world, num_clients)
    return sorted(out)


def probe_and_filter(ref: torch.Tensor, num_clients: int, nbytes: int = 64 << 20, iters: int = 3,
                     k: float = 1.0, rel: float = 0.05) -> List[int]:
    """Measure the rank bandwidth graph, flag anomalous ranks (PageRank +-k sigma with a ``rel``
    relative-deviation floor) and return the clients they host (excluded from gossip).
    ``ref`` only selects the device."""
    rt = D.runtime()
    if rt.world < 3:  # PageRank outliers need at least three nodes
        return []
    bw = measure_bandwidth(nbytes, iters, ref.device)
    bad = topology_filter(bw, k, rel)
    if len(bad) * 2 >= rt.world:  # never evict a majority on a noisy probe
        return []
    return ranks_to_clients(bad, rt.world, num_clients)

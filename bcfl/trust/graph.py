"""Graph analytics of the trust layer: PageRank, modified-Z, DBSCAN, greedy modularity,
shortest-path information-passing time and the latency objective (SURVEY.md N2–N7).

Each function runs the native C++ implementation (``bcfl._host``) when it is built and a
NumPy implementation of the same semantics otherwise (the CPU test-suite checks they agree and
that both reproduce the reference notebook's recorded outputs).
"""
from __future__ import annotations

import heapq
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

try:  # native host runtime
    from .. import _host as _H  # type: ignore
except Exception:  # pragma: no cover - exercised when the .so is absent
    _H = None


def native_available() -> bool:
    return _H is not None


# ------------------------------------- PageRank ---------------------------------------------

def pagerank(W: np.ndarray, alpha: float = 0.85, tol: float = 1e-6, max_iter: int = 100,
             use_native: Optional[bool] = None) -> np.ndarray:
    """networkx-3 ``pagerank(G, weight='weight')`` semantics on a dense weight matrix
    (W[i, j] = weight of edge i->j, 0 = no edge)."""
    W = np.ascontiguousarray(W, dtype=np.float64)
    if (use_native is None and _H is not None) or use_native:
        ranks, _, conv = _H.pagerank(W, alpha, tol, max_iter)
        if not conv:
            raise RuntimeError("pagerank failed to converge")
        return np.asarray(ranks)
    n = W.shape[0]
    S = W.sum(1)
    inv = np.zeros(n)
    inv[S != 0] = 1.0 / S[S != 0]
    Q = W * inv[:, None]
    dang = np.flatnonzero(S == 0)
    p = np.full(n, 1.0 / n)
    x = p.copy()
    for _ in range(max_iter):
        xl = x
        x = alpha * (xl @ Q + xl[dang].sum() * p) + (1 - alpha) * p
        if np.abs(x - xl).sum() < n * tol:
            return x
    raise RuntimeError("pagerank failed to converge")


def sigma_flags(values: Sequence[float], k: float = 1.0, low_only: bool = False
                ) -> Tuple[Tuple[float, float], List[int]]:
    """Flag values outside [mu - k sigma, mu + k sigma] (population sigma), as the reference's
    PageRank cell does with k = 1 (All_graphs_IMDB_dataset.ipynb:172-176)."""
    v = [float(x) for x in values]
    if _H is not None:
        lo, hi, flags = _H.sigma_flags(v, k, low_only)
        return (lo, hi), [i for i, f in enumerate(flags) if f]
    a = np.asarray(v)
    mu = a.mean() if a.size else 0.0
    sd = np.sqrt(((a - mu) ** 2).mean()) if a.size else 0.0
    lo, hi = mu - k * sd, mu + k * sd
    return (lo, hi), [i for i, x in enumerate(v) if x < lo or (not low_only and x > hi)]


def pagerank_anomalies(W: np.ndarray, k: float = 1.0, low_only: bool = False):
    r = pagerank(W)
    thr, flags = sigma_flags(r, k, low_only)
    return r, thr, flags


# ---------------------------------- modified Z / DBSCAN ---------------------------------------

def modified_z(values: Sequence[float]) -> np.ndarray:
    v = [float(x) for x in values]
    if _H is not None:
        return np.asarray(_H.modified_z(v))
    a = np.asarray(v)
    med = np.median(a)
    mad = np.median(np.abs(a - med))
    with np.errstate(divide="ignore", invalid="ignore"):
        return 0.6745 * (a - med) / mad


def modz_anomalies(values: Sequence[float], threshold: float = 1.0) -> List[int]:
    z = modified_z(values)
    return [i for i, s in enumerate(z) if abs(s) > threshold]


def dbscan(X: np.ndarray, eps: float, min_samples: int) -> np.ndarray:
    X = np.ascontiguousarray(np.asarray(X, dtype=np.float64).reshape(len(X), -1))
    if _H is not None:
        return np.asarray(_H.dbscan(X, eps, min_samples))
    n = X.shape[0]
    D = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    nb = [np.flatnonzero(D[i] <= eps) for i in range(n)]
    core = np.array([len(x) >= min_samples for x in nb])
    lab = np.full(n, -1)
    cid = 0
    for i in range(n):
        if not core[i] or lab[i] != -1:
            continue
        lab[i] = cid
        st = [i]
        while st:
            u = st.pop()
            if not core[u]:
                continue
            for v in nb[u]:
                if lab[v] == -1:
                    lab[v] = cid
                    if core[v]:
                        st.append(v)
        cid += 1
    return lab


def weighted_degree(W: np.ndarray) -> np.ndarray:
    return np.asarray(W, dtype=np.float64).sum(1)


def greedy_modularity(A: np.ndarray) -> List[int]:
    A = np.ascontiguousarray(A, dtype=np.float64)
    if _H is not None:
        return list(_H.greedy_modularity(A))
    n = A.shape[0]
    comm = list(range(n))
    m2 = A.sum()
    if m2 <= 0:
        return comm
    k = A.sum(1)
    while True:
        nc = max(comm) + 1
        E = np.zeros((nc, nc))
        a = np.zeros(nc)
        for i in range(n):
            a[comm[i]] += k[i] / m2
            for j in range(n):
                E[comm[i], comm[j]] += A[i, j] / m2
        best, bi, bj = 0.0, -1, -1
        for i in range(nc):
            for j in range(i + 1, nc):
                dq = 2 * (E[i, j] - a[i] * a[j])
                if dq > best + 1e-15:
                    best, bi, bj = dq, i, j
        if bi < 0:
            return comm
        comm = [bi if c == bj else (c - 1 if c > bj else c) for c in comm]


def community_anomalies(A: np.ndarray) -> List[int]:
    """Nodes in no community (reference Louvain cell, always empty by construction)."""
    comm = greedy_modularity(A)
    return [i for i, c in enumerate(comm) if c < 0]


# --------------------------- paths, passing time, latency objective ---------------------------

def latency_matrix(bw: np.ndarray, model_bytes_or_gb: float) -> np.ndarray:
    """L[i, j] = size / bandwidth (inf where no link)."""
    bw = np.asarray(bw, dtype=np.float64)
    L = np.full(bw.shape, np.inf)
    nz = bw > 0
    L[nz] = model_bytes_or_gb / bw[nz]
    np.fill_diagonal(L, 0.0)
    return L


def shortest_paths(L: np.ndarray, src: int, excluded: Sequence[int] = ()) -> np.ndarray:
    L = np.ascontiguousarray(L, dtype=np.float64)
    if _H is not None:
        return np.asarray(_H.shortest_paths(L, src, list(excluded)))
    n = L.shape[0]
    act = np.ones(n, bool)
    act[list(excluded)] = False
    dist = np.full(n, np.inf)
    if not act[src]:
        return dist
    dist[src] = 0.0
    done = np.zeros(n, bool)
    pq = [(0.0, src)]
    while pq:
        d, u = heapq.heappop(pq)
        if done[u]:
            continue
        done[u] = True
        for v in range(n):
            if v == u or not act[v] or not np.isfinite(L[u, v]):
                continue
            if d + L[u, v] < dist[v]:
                dist[v] = d + L[u, v]
                heapq.heappush(pq, (dist[v], v))
    return dist


@dataclass
class PassingTime:
    sync: float    # sequential sends: sum over destinations
    async_: float  # concurrent sends: max over destinations
    reached: int


def info_passing_time(L: np.ndarray, src: int = 0, excluded: Sequence[int] = ()) -> PassingTime:
    """Information-passing time from ``src`` to every live node along shortest paths (N6):
    sync = Σ_j t(src->j), async = max_j t(src->j) (Medical_Transcriptions_All_graphs.ipynb:974-999)."""
    if _H is not None:
        s, a, r = _H.info_passing_time(np.ascontiguousarray(L, dtype=np.float64), src, list(excluded))
        return PassingTime(s, a, r)
    d = shortest_paths(L, src, excluded)
    m = np.ones(len(d), bool)
    m[src] = False
    m[list(excluded)] = False
    m &= np.isfinite(d)
    return PassingTime(float(d[m].sum()), float(d[m].max()) if m.any() else 0.0, int(m.sum()))


def best_source(L: np.ndarray, excluded: Sequence[int] = (), d_g: float = 0.0) -> Tuple[int, float]:
    """Latency objective N7: argmin_s D_g + max_j t(s->j) (All_graphs_IMDB_dataset.ipynb:21)."""
    if _H is not None:
        return tuple(_H.best_source(np.ascontiguousarray(L, dtype=np.float64), list(excluded), d_g))
    best = (-1, np.inf)
    for s in range(L.shape[0]):
        if s in set(excluded):
            continue
        t = info_passing_time(L, s, excluded)
        if d_g + t.async_ < best[1]:
            best = (s, d_g + t.async_)
    return best


def anomaly_report(bw: np.ndarray) -> Dict[str, List[int]]:
    """All four reference detectors on a bandwidth graph (weights 1/bw)."""
    from .netdata import ref_undirected_weight_matrix  # noqa: F401
    W = np.zeros_like(bw, dtype=np.float64)
    nz = bw > 0
    W[nz] = 1.0 / bw[nz]
    U = np.zeros_like(W)
    n = W.shape[0]
    for u in range(n):
        for v in range(u + 1, n):
            U[u, v] = U[v, u] = W[v, u]
    _, _, pr = pagerank_anomalies(W, 1.0)
    deg = weighted_degree(U)
    return {
        "pagerank": pr,
        "modz": modz_anomalies(deg, 1.0),
        "dbscan": [i for i, l in enumerate(dbscan(deg[:, None], 300.0, 2)) if l == -1],
        "louvain": community_anomalies(U),
    }

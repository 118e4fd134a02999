"""Small helpers shared by the federation modules."""
from __future__ import annotations

import zlib

DATA_SEED = 1234


def _cseed(seed: int, c: int) -> int:
    return zlib.crc32(f"{seed}:{c}".encode()) & 0x7FFFFFFF

def weighted_average(metrics):
    """Reference metric aggregation (``server_IID_IMDB.py:199-203``): Σ n_k·m_k / Σ n_k."""
    ex = sum(n for n, _ in metrics)
    out = {}
    for key in ("accuracy", "loss"):
        vals = [n * m[key] for n, m in metrics if key in m]
        if vals:
            out[key] = sum(vals) / max(ex, 1)
    return out

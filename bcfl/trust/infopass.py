"""Information-passing time on the transport the federation actually uses: one-sided mailbox
posts (BASELINE.md "measure it for real over xGMI").

The reference's claim (``README.md:10``: async cuts information-passing time by 76 %) rests on a
hand computation: a node's model reaches its peers in sum_j t(src -> j) when sent one
destination after another (sync) and in max_j t(src -> j) when sent to all at once (async)
(``Medical_Transcriptions_All_graphs.ipynb:974-999``), repeated after removing the nodes that
DBSCAN / modified-Z / PageRank flag (``All_graphs_IMDB_dataset.ipynb:987-988``). Here both are
MEASURED with the gossip engine's own mailbox transport on the running job:

* sync  — the source posts its model to one destination, waits for the copy to land, then the
  next destination (each post on that destination's side stream, completion by event);
* async — the source posts to every destination at once (one side stream per destination, the
  copies run concurrently over their own xGMI links) and waits for all.

The per-destination single-post times give the measured bandwidth matrix row of the source;
the analytical model of the reference (``bcfl.trust.graph.info_passing_time``: size / bandwidth
along shortest paths) is evaluated on that matrix, and everything is repeated after the PageRank
topology filter (``bcfl.trust.anomaly.topology_filter``) removes its flagged ranks.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..parallel import dist as D
from ..parallel.mailbox import MailboxTransport, Snapshot
from . import graph as G
from .anomaly import topology_filter


def _sync_dev(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def measure(numel: int, sources: Optional[Sequence[int]] = None, iters: int = 3,
            dtype: torch.dtype = torch.bfloat16) -> Dict:
    """Collective: every rank calls it. Returns (identical on every rank) the measured sync /
    async information-passing times from each source, the measured bandwidth matrix, the
    analytical predictions, and the same after PageRank removal."""
    rt = D.runtime()
    w, me, dev = rt.world, rt.rank, rt.device
    if w < 2:
        return {}
    sources = list(range(w)) if sources is None else list(sources)
    peers_of = {s: [d for d in range(w) if d != s] for s in range(w)}
    tr = MailboxTransport(numel, dtype, dev, listen=[s for s in range(w) if s != me],
                          send_plan=[(me, d) for d in peers_of[me]], rank=me, world=w)
    payload = torch.full((numel,), 1.0 + me, dtype=dtype, device=dev)
    nbytes = numel * payload.element_size()
    version = [0]

    def post(dsts: Sequence[int]) -> None:
        version[0] += 1
        tr.post_to(me, payload, Snapshot(version[0], 0, 0, nbytes, b"\0" * 32), dsts)

    def timed(fn) -> float:
        ts = []
        for _ in range(iters):
            _sync_dev(dev)
            t0 = time.perf_counter()
            fn()
            tr.drain()
            _sync_dev(dev)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    bw = np.zeros((w, w))
    res = {"world": w, "model_bytes": nbytes, "transport": "mailbox", "sources": []}

    def run_from(src: int, peers: List[int]) -> Dict[str, float]:
        out = {"sync_s": 0.0, "async_s": 0.0, "per_dst_s": {}}
        if me == src:
            post(peers)          # warm-up: first touch of every peer mapping
            tr.drain()
            per = {}
            for d in peers:      # single-destination post times -> bandwidth row
                per[d] = timed(lambda d=d: post([d]))

            def sync():
                for d in peers:
                    post([d])
                    tr.drain()   # the next destination starts only when this copy has landed

            out = {"sync_s": timed(sync), "async_s": timed(lambda: post(peers)),
                   "per_dst_s": {int(d): t for d, t in per.items()}}
        allv = D.all_gather_object(out)
        return allv[src]

    for src in sources:
        o = run_from(src, peers_of[src])
        for d, t in o["per_dst_s"].items():
            bw[src, int(d)] = nbytes / max(t, 1e-12) / 1e6  # MB/s
        res["sources"].append({"source": src, "measured_sync_s": o["sync_s"],
                               "measured_async_s": o["async_s"],
                               "per_destination_s": o["per_dst_s"]})
        D.barrier()
    # analytical model on the measured matrix (rows of sources not measured: symmetric fill)
    full = bw.copy()
    for i in range(w):
        for j in range(w):
            if i != j and full[i, j] == 0.0 and full[j, i] > 0.0:
                full[i, j] = full[j, i]
    res["bw_MBps"] = full.tolist()
    L = G.latency_matrix(full * 1e6, float(nbytes)) if full.any() else None
    flagged = topology_filter(full) if full.any() else []
    res["pagerank_flagged"] = [int(x) for x in flagged]
    for rec in res["sources"]:
        s = rec["source"]
        if L is not None and np.isfinite(L[s]).sum() > 1:
            p = G.info_passing_time(L, s)
            rec.update(predicted_sync_s=p.sync, predicted_async_s=p.async_)
    # after removing the PageRank-flagged ranks: re-measure from the sources that remain
    res["after_pagerank_removal"] = []
    if flagged:
        for src in sources:
            if src in flagged:
                continue
            peers = [d for d in peers_of[src] if d not in flagged]
            if not peers:
                continue
            o = run_from(src, peers)
            rec = {"source": src, "excluded": res["pagerank_flagged"],
                   "measured_sync_s": o["sync_s"], "measured_async_s": o["async_s"]}
            if L is not None:
                p = G.info_passing_time(L, src, flagged)
                rec.update(predicted_sync_s=p.sync, predicted_async_s=p.async_)
            res["after_pagerank_removal"].append(rec)
            D.barrier()
    for rec in res["sources"] + res["after_pagerank_removal"]:
        if rec["measured_sync_s"] > 0:
            rec["async_reduction_pct"] = 100.0 * (1.0 - rec["measured_async_s"] / rec["measured_sync_s"])
    D.barrier()
    tr.close()
    return res

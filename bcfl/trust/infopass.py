"""Information-passing time on the transport the federation actually uses: one-sided mailbox
posts (BASELINE.md "measure it for real over xGMI").

The reference's claim (``README.md:10``: async cuts information-passing time by 76 %) rests on a
hand computation: a node's model reaches its peers in sum_j t(src -> j) when sent one
destination after another (sync) and in max_j t(src -> j) when sent to all at once (async)
(``Medical_Transcriptions_All_graphs.ipynb:974-999``), repeated after removing the nodes that
DBSCAN / modified-Z / PageRank flag (``All_graphs_IMDB_dataset.ipynb:987-988``), and once more
"through the BCFL algorithm" (``All_graphs_IMDB_dataset.ipynb:1048,1070-1071``;
``Medical_Transcriptions_All_graphs.ipynb:1091-1098``). Here every one of those numbers is
MEASURED with the gossip engine's own mailbox transport on the running job:

* **plain sync**  — the source posts its model to one destination; the next destination's copy
  is stream-ordered after the previous copy has landed (no host in between);
* **plain async** — the source posts to every destination at once (one side stream per
  destination: the copies run concurrently over their own xGMI links);
* **BC-FL** — the same with the ledger path: the source computes the payload's SHA-256 Merkle
  commitment on its GPU before posting (the root travels in the header), and every receiver
  copies the payload out of its inbox and re-hashes it to verify the commitment. BC-FL sync =
  commit + the sequential posts (measured) + the sum of the receivers' verification times
  (measured on each receiver); BC-FL async = commit + concurrent posts (measured) + the slowest
  receiver's verification;
* the measured per-destination post times give the source's bandwidth row; the reference's
  analytical model (``bcfl.trust.graph.info_passing_time``: size / bandwidth along shortest
  paths) is evaluated on that matrix;
* everything is repeated after removing the ranks each reference detector flags on the measured
  bandwidth graph (DBSCAN, modified-Z, PageRank: ``bcfl.trust.graph.anomaly_report``, the
  notebook's parameters).

GPU: every time is a HIP-event interval on the device (the host only enqueues), so several
processes sharing one GPU do not turn host scheduling into "transfer time". CPU (gloo + /dev/shm
rehearsal): host timing around the synchronous copies.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..parallel import dist as D
from ..parallel.mailbox import MailboxTransport, Snapshot
from . import graph as G

DETECTORS = ("dbscan", "modz", "pagerank")


class _Clock:
    """Device-event timing on GPU (median over iterations), host timing on CPU."""

    def __init__(self, dev: torch.device, iters: int):
        self.dev, self.iters = dev, max(1, int(iters))
        self.cuda = dev.type == "cuda"

    def __call__(self, enqueue: Callable[[], None]) -> float:
        ts = []
        for _ in range(self.iters):
            if self.cuda:
                s = torch.cuda.current_stream(self.dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                enqueue()            # must leave the current stream waiting on all its work
                e1.record(s)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) / 1e3)
            else:
                t0 = time.perf_counter()
                enqueue()
                ts.append(time.perf_counter() - t0)
        return float(np.median(ts))


def measure(numel: int, sources: Optional[Sequence[int]] = None, iters: int = 3,
            dtype: torch.dtype = torch.bfloat16,
            detectors: Sequence[str] = DETECTORS) -> Dict:
    """Collective: every rank calls it. Returns (identical on every rank) per source the measured
    plain and BC-FL sync / async information-passing times, the measured bandwidth matrix, the
    analytical predictions, and all of it again after each detector's removal."""
    rt = D.runtime()
    w, me, dev = rt.world, rt.rank, rt.device
    if w < 2:
        return {}
    sources = list(range(w)) if sources is None else list(sources)
    tr = MailboxTransport(numel, dtype, dev, listen=[s for s in range(w) if s != me],
                          send_plan=[(me, d) for d in range(w) if d != me], rank=me, world=w)
    payload = torch.full((numel,), 1.0 + me, dtype=dtype, device=dev)
    stage = torch.empty_like(payload)
    nbytes = numel * payload.element_size()
    clock = _Clock(dev, iters)
    version = [0]

    def post(dsts: Sequence[int], root=None) -> None:
        """Post to ``dsts`` and leave the current stream waiting until every copy has landed."""
        version[0] += 1
        v = version[0]
        tr.post_to(me, payload, Snapshot(v, 0, 0, nbytes, b"\0" * 32), dsts,
                   root if torch.is_tensor(root) else None)
        if tr.is_cuda:
            cur = torch.cuda.current_stream(dev)
            # pop: the current stream waits for these copies, so the slot needs no later wait
            # (and the events of past measurements do not pile up in the transport)
            for ev in tr.posted.pop((me, v % 2), []):
                cur.wait_event(ev)

    def commit():
        return ops.merkle_root_deferred(payload)

    def verify_time(src: int) -> float:
        """Receiver side of BC-FL: copy the newest complete payload of ``src`` out of the inbox
        and re-hash it (the comparison with the header's root is a 32-byte host compare)."""
        nw = tr.newest(tr.headers([src])[src])
        if nw is None:
            return 0.0
        slot = nw[0]

        def work():
            stage.copy_(tr.inbox[src].slots[slot], non_blocking=True)
            rt_ = ops.merkle_root_deferred(stage)
            if not torch.is_tensor(rt_):
                return
        return clock(work)

    def run_from(src: int, peers: List[int]) -> Dict:
        out: Dict = {}
        if me == src:
            post(peers)                               # warm-up: first touch of every mapping
            tr.drain()
            per = {int(d): clock(lambda d=d: post([d])) for d in peers}

            def sync_chain(with_commit: bool):
                r = commit() if with_commit else None
                for d in peers:
                    post([d], r)

            out = {"per_dst_s": per,
                   "sync_s": clock(lambda: sync_chain(False)),
                   "async_s": clock(lambda: post(peers)),
                   "commit_s": clock(lambda: commit()),
                   "bcfl_send_sync_s": clock(lambda: sync_chain(True)),
                   "bcfl_send_async_s": clock(lambda: post(peers, commit()))}
            tr.drain()
        D.barrier()                                   # the source's posts have landed
        ver = verify_time(src) if me in peers else None
        allv = D.all_gather_object({"out": out, "verify_s": ver})
        o = dict(allv[src]["out"])
        o["verify_s"] = {int(r): v["verify_s"] for r, v in enumerate(allv) if v["verify_s"] is not None}
        vs = list(o["verify_s"].values()) or [0.0]
        o["bcfl_sync_s"] = o["bcfl_send_sync_s"] + float(sum(vs))
        o["bcfl_async_s"] = o["bcfl_send_async_s"] + float(max(vs))
        return o

    def record(o: Dict, src: int, L, excluded: Sequence[int]) -> Dict:
        rec = {"source": src, "measured_sync_s": o["sync_s"], "measured_async_s": o["async_s"],
               "bcfl": {"sync_s": o["bcfl_sync_s"], "async_s": o["bcfl_async_s"],
                        "commit_s": o["commit_s"], "verify_s": o["verify_s"],
                        "send_sync_s": o["bcfl_send_sync_s"],
                        "send_async_s": o["bcfl_send_async_s"]}}
        if L is not None and np.isfinite(L[src]).sum() > 1:
            p = G.info_passing_time(L, src, list(excluded))
            rec.update(predicted_sync_s=p.sync, predicted_async_s=p.async_)
        for key, (s_, a_) in (("plain", (o["sync_s"], o["async_s"])),
                              ("bcfl", (o["bcfl_sync_s"], o["bcfl_async_s"]))):
            if s_ > 0:
                tgt = rec if key == "plain" else rec["bcfl"]
                tgt["async_reduction_pct"] = 100.0 * (1.0 - a_ / s_)
        return rec

    bw = np.zeros((w, w))
    res = {"world": w, "model_bytes": nbytes, "transport": "mailbox",
           "timing": "hip events (device)" if tr.is_cuda else "host (cpu rehearsal)",
           "sources": []}
    raw = {}
    for src in sources:
        o = run_from(src, [d for d in range(w) if d != src])
        raw[src] = o
        for d, t in o["per_dst_s"].items():
            bw[src, int(d)] = nbytes / max(t, 1e-12) / 1e6  # MB/s
        D.barrier()
    # analytical model on the measured matrix (rows of sources not measured: symmetric fill)
    full = bw.copy()
    for i in range(w):
        for j in range(w):
            if i != j and full[i, j] == 0.0 and full[j, i] > 0.0:
                full[i, j] = full[j, i]
    res["bw_MBps"] = full.tolist()
    L = G.latency_matrix(full * 1e6, float(nbytes)) if full.any() else None
    for src in sources:
        res["sources"].append(record(raw[src], src, L, []))
    # the reference detectors on the measured bandwidth graph, then re-measure without the flags
    flags = G.anomaly_report(full) if full.any() else {k: [] for k in DETECTORS}
    res["detectors"] = {}
    for det in detectors:
        fl = [int(x) for x in flags.get(det, [])]
        entry = {"flagged": fl, "sources": []}
        for src in sources:
            peers = [d for d in range(w) if d != src and d not in fl]
            if src in fl or not peers:
                entry["sources"].append({"source": src, "skipped": "source flagged" if src in fl
                                         else "no peers left"})
                continue
            entry["sources"].append(record(run_from(src, peers), src, L, fl))
            D.barrier()
        res["detectors"][det] = entry
    # round-3 key kept for readers of older records
    pr = res["detectors"].get("pagerank", {"flagged": [], "sources": []})
    res["pagerank_flagged"] = pr["flagged"]
    res["after_pagerank_removal"] = [dict(s, excluded=pr["flagged"]) for s in pr["sources"]
                                     if "skipped" not in s] if pr["flagged"] else []
    D.barrier()
    tr.close()
    return res


def summary(res: Dict) -> List[str]:
    """One line per (source, detector) with the eight measured numbers and the prediction."""
    lines = []
    for s in res.get("sources", []):
        lines.append(_line("all ranks", s))
    for det, e in res.get("detectors", {}).items():
        for s in e["sources"]:
            if "skipped" in s:
                lines.append(f"source {s['source']} after {det} {e['flagged']}: {s['skipped']}")
            else:
                lines.append(_line(f"after {det} {e['flagged']}", s))
    return lines


def _line(tag: str, s: Dict) -> str:
    b = s["bcfl"]
    return (f"source {s['source']} {tag}: plain sync {s['measured_sync_s'] * 1e3:.3f} ms async "
            f"{s['measured_async_s'] * 1e3:.3f} ms | BC-FL sync {b['sync_s'] * 1e3:.3f} ms async "
            f"{b['async_s'] * 1e3:.3f} ms | predicted sync "
            f"{s.get('predicted_sync_s', float('nan')) * 1e3:.3f} ms async "
            f"{s.get('predicted_async_s', float('nan')) * 1e3:.3f} ms")

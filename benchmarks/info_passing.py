#!/usr/bin/env python
"""Information-passing time, MEASURED: how long one client's model takes to reach
every peer when it is sent synchronously (one destination after another: Σ) versus
asynchronously (all destinations at once over their own xGMI links: max), next to the
prediction of the reference's analytical model (size / bandwidth along shortest paths) evaluated
on the bandwidth matrix measured by :mod:`bcfl.trust.probe` on the same job.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        benchmarks/info_passing.py --model bert-base [--json out.json]
    python benchmarks/info_passing.py --cpu-world 4          # gloo rehearsal on the CPU

The reference hand-computed 44.8 s (sync) / 9.38 s (async) for the 0.4036 GB BioBERT on its
10-node 88-496 Mbps graph (``Medical_Transcriptions_All_graphs.ipynb:974-999``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _timed(fn, dev, iters=3):
    ts = []
    for _ in range(iters):
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def run(numel: int, iters: int = 3, probe_bytes: int = 64 << 20) -> dict:
    from bcfl.parallel import dist as D
    from bcfl.trust import graph as G
    from bcfl.trust.probe import measure_bandwidth
    rt = D.runtime()
    dev, w, me = rt.device, rt.world, rt.rank
    buf = torch.ones(numel, dtype=torch.bfloat16, device=dev)
    rbuf = torch.empty_like(buf)
    nbytes = numel * 2
    bw = measure_bandwidth(probe_bytes, iters, dev)  # MB/s
    res = {"world": w, "model_bytes": nbytes, "bw_MBps": bw.tolist(), "sources": []}
    for src in range(w):
        peers = [j for j in range(w) if j != src]

        def sync_send():
            for j in peers:
                if me == src:
                    D.p2p_exchange([(buf, j)], []).wait()
                elif me == j:
                    D.p2p_exchange([], [(rbuf, src)]).wait()

        def async_send():
            if me == src:
                D.p2p_exchange([(buf, j) for j in peers], []).wait()
            else:
                D.p2p_exchange([], [(rbuf, src)]).wait()

        sync_send()  # warm-up
        D.barrier()
        ts = _timed(sync_send, dev, iters)
        D.barrier()
        ta = _timed(async_send, dev, iters)
        D.barrier()
        ts, ta = D.max_over_ranks(ts), D.max_over_ranks(ta)
        L = G.latency_matrix(bw * 1e6, float(nbytes))  # seconds
        pred = G.info_passing_time(L, src)
        res["sources"].append({"source": src, "measured_sync_s": ts, "measured_async_s": ta,
                               "predicted_sync_s": pred.sync, "predicted_async_s": pred.async_})
    return res


def _cpu_worker(rank, world, numel, out, transport="rccl"):
    from bcfl.parallel import dist as D
    D.init_runtime("cpu", "gloo")
    if transport == "mailbox":
        from bcfl.trust.infopass import measure
        r = measure(numel, iters=2)
    else:
        r = run(numel, 2, 1 << 18)
    if rank == 0:
        with open(out, "w") as fh:
            json.dump(r, fh)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--numel", type=int, default=0, help="override: elements (bf16) per model")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--json", default=None)
    ap.add_argument("--cpu-world", type=int, default=0, help="gloo rehearsal with this many CPU ranks")
    ap.add_argument("--transport", default="mailbox", choices=("mailbox", "rccl"),
                    help="mailbox: one-sided posts (what the gossip engine uses); rccl: send/recv")
    a = ap.parse_args(argv)
    numel = a.numel
    if not numel:
        from bcfl.models import build_model
        m = build_model(a.model, 2, device="meta")
        numel = sum(p.numel() for p in m.parameters())
    if a.cpu_world:
        import tempfile

        import torch.multiprocessing as mp
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
        from dist_utils import run_world
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "r.json")
            run_world(_cpu_worker, a.cpu_world, td, min(numel, 1 << 20), out, a.transport)
            res = json.load(open(out))
        del mp
    else:
        from bcfl.parallel import dist as D
        D.init_runtime("auto", "auto")
        if a.transport == "mailbox":
            from bcfl.trust.infopass import measure
            res = measure(numel, iters=a.iters)
        else:
            res = run(numel, a.iters)
        if not D.runtime().is_main:
            return 0
    for s in res["sources"] + res.get("after_pagerank_removal", []):
        tag = f" (without {s['excluded']})" if "excluded" in s else ""
        print(f"source {s['source']}{tag}: measured sync {s['measured_sync_s'] * 1e3:.2f} ms async "
              f"{s['measured_async_s'] * 1e3:.2f} ms | predicted sync "
              f"{s.get('predicted_sync_s', float('nan')) * 1e3:.2f} ms async "
              f"{s.get('predicted_async_s', float('nan')) * 1e3:.2f} ms")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

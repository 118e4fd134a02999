#!/usr/bin/env python
"""Asynchronous-gossip protocol sweep on ONE GPU: the multi-rank delta protocol in one process.

Every hosted client is its own virtual rank (``gossip_transport="loopback"``,
:mod:`bcfl.parallel.loopback`): a client's post reaches the others ``loopback_lag_steps`` local
steps after it was made, so the 8-client federation runs the asynchronous protocol of the 8-GPU
layout (late, mid-round application of every neighbour update; exchanged SCAFFOLD control
variates) at the speed of one GPU — 25 rounds of BERT-base in ~20 s instead of ~100 s for 8
processes on CU slices. Each variant is one line of JSON (curve, final accuracy, s/round).

    python benchmarks/async_protocol.py --out profiles/async_protocol.jsonl \\
        --variant 'sync:gossip_transport="mailbox"' \\
        --variant 'arrival:gossip_transport="loopback",gossip_apply="arrival"' \\
        --variant 'complete:gossip_transport="loopback",gossip_apply="complete"'

Reference claim being tested: async P2P learns as well as the synchronous scheme
(``/root/reference/README.md:10``; serverless Non-IID curve, ``All_graphs_IMDB_dataset.ipynb:1142``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_variant(tag: str, overrides: dict, a) -> dict:
    import torch
    from bcfl.config import get_preset
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    kw = dict(model=a.model, num_clients=a.clients, num_rounds=a.rounds, ledger=False,
              save_every=0, reference_prints=False, out_dir=os.path.join("runs", "async_protocol", tag),
              client_lanes=a.lanes, device=a.device)
    kw.update(overrides)
    cfg = get_preset(a.preset, **kw)
    fed = Federation(cfg, verbose=False)
    t0 = time.perf_counter()
    fed.run()
    dt = time.perf_counter() - t0
    fa = fed.federation_accuracy()
    h = fed.history
    g = fed.gossip
    rec = {"tag": tag, "overrides": overrides, "rounds": a.rounds,
           "s_per_round": dt / a.rounds,
           "final_accuracy": fa.get("accuracy"),
           "curve": [round(float(x), 4) for x in fed.global_accuracies],
           "train_loss": [round(float(x["train_loss"]), 4) if x.get("train_loss") is not None else None
                          for x in h],
           "stale_rounds": [x.get("stale_rounds") for x in h],
           "exchange": getattr(g, "exchange", "state"),
           "apply": getattr(g, "apply_mode", None),
           "transport": fed.transport,
           "lag": (g.transport.stats() if hasattr(getattr(g, "transport", None), "stats") else None),
           "drift": fed.drift.mode, "drift_exchange": fed.drift.exchange,
           "keep_opt": bool(fed.keep_opt)}
    del fed
    D.set_runtime_for_tests(None)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", default=[],
                    help="TAG:key=value,key=value (FLConfig overrides, Python literals)")
    ap.add_argument("--preset", default="baseline3_learnable")
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=25)
    ap.add_argument("--lanes", type=int, default=8)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    for v in a.variant:
        tag, _, spec = v.partition(":")
        ov = eval(f"dict({spec})") if spec.strip() else {}
        rec = run_variant(tag, ov, a)
        line = json.dumps(rec)
        print(f"{tag}: final {rec['final_accuracy']} s/round {rec['s_per_round']:.3f} "
              f"curve {rec['curve']}", flush=True)
        if a.out:
            os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
            with open(a.out, "a") as fh:
                fh.write(line + "\n")


if __name__ == "__main__":
    main()

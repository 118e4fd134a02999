#!/usr/bin/env python
"""The reference's worker grid on MI355X: server (FedAvg) vs serverless (P2P gossip) at 5 / 10 /
20 clients, 20 rounds each — the experiment behind the latency and accuracy bar charts of
``All_graphs_IMDB_dataset.ipynb:747-748`` (latency) and ``:830-831`` (accuracy).

Setup (both modes identical except the protocol): IMDB-shaped synthetic data, IID, 100 train /
100 test rows per client (``server_IID_IMDB.py:79-84`` / ``serverless_IID_IMDB.py:258``),
BERT-base (the BioBERT architecture of the server script), random init with the learnable
protocol of ``baseline3_learnable``, class-balanced 1000-row global draw, all clients on one GPU
(client lanes), per-round checkpoints and the ledger on.

    python benchmarks/worker_grid.py [--clients 5 10 20] [--rounds 20] [--out profiles/x.json]
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(mode: str, clients: int, rounds: int, out_dir: str, model: str, keep_opt: bool,
        **extra) -> dict:
    import torch
    from bcfl.config import get_preset
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    D.set_runtime_for_tests(None)
    t_proc = time.time()
    part = "shared_random" if mode == "server" else "iid_random"
    if mode == "serverless":
        # the reference's serverless global model: the mean of the client models, scored on the
        # whole draw (serverless_IID_IMDB.py:269-279 avg_params -> global_model), as the server scores its
        # FedAvg model: one model per round in both modes
        extra.setdefault("global_eval_models", "average")
    cfg = get_preset("baseline3_learnable", mode=mode, model=model, num_clients=clients,
                     num_rounds=rounds, partition=part, train_samples=100, test_samples=100,
                     resample_each_round=(mode == "serverless"), out_dir=out_dir,
                     reference_prints=False, save_every=1, keep_optimizer_state=keep_opt,
                     **extra)
    fed = Federation(cfg, verbose=False)
    # steady-state time as bench.py measures it: the rounds after the first 3 as ONE block,
    # synchronised only at its two ends (a per-round device sync would serialise every round's
    # host-side start with the GPU and penalise the protocol that defers its host reads)
    warm = 3 if rounds > 4 else 0
    times = []
    t_block = None
    for r in range(rounds):
        if r == warm:
            if fed.is_cuda:
                torch.cuda.synchronize()
            t_block = time.perf_counter()
        t0 = time.perf_counter()
        fed.run_round(r)
        times.append(time.perf_counter() - t0)
    fed.drain()
    if fed.ckpt is not None:
        fed.ckpt.wait()
    if fed.is_cuda:
        torch.cuda.synchronize()
    steady_s = (time.perf_counter() - t_block) / max(rounds - warm, 1)
    fed.timer.resolve(block=True)
    steady_h = fed.history[3:] if len(fed.history) > 4 else fed.history
    phases = {}
    for h in steady_h:
        for k, v in h.items():
            if (k.startswith("t_") or k.startswith("dev_t_")) and isinstance(v, (int, float)):
                phases[k] = phases.get(k, 0.0) + float(v) / len(steady_h)
    fa = fed.federation_accuracy()
    fed.finish()
    rec = {"mode": mode, "clients": clients, "rounds": rounds, "model": model,
           "keep_optimizer_state": keep_opt, "overrides": extra,
           "train_loss_curve": [h.get("train_loss") for h in fed.history],
           "s_per_round_steady": steady_s, "host_issue_s_per_round": times,
           "total_rounds_s": sum(times),
           "process_latency_min": (time.time() - t_proc) / 60.0,
           "final_accuracy": fa.get("accuracy"), "global_eval_rows": fa.get("rows"),
           "final_majority_rate": fed.history[-1].get("global_majority_rate"),
           "accuracy_curve": list(fed.global_accuracies), "lanes": len(fed.lanes) or 1,
           "hbm_peak_gb": fed.history[-1].get("hbm_peak_gb"),
           "steady_phase_means_s": phases}
    del fed
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
    return rec


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, nargs="+", default=[5, 10, 20])
    ap.add_argument("--modes", nargs="+", default=["server", "serverless"])
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--out", default="gpurun_out/worker_grid.json")
    ap.add_argument("--fresh-adamw", action="store_true",
                    help="the reference's fresh AdamW per round (oscillates on IID from random "
                         "init, profiles/accuracy_server_stability.json); default keeps moments")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="extra FLConfig override (JSON value), e.g. --set max_grad_norm=1.0")
    ap.add_argument("--protocol", choices=["iid", "none"], default="iid",
                    help="iid: the IID learning protocol (bcfl.config.IID_PROTOCOL) under the "
                         "--set overrides; none: baseline3_learnable's label-shard settings")
    a = ap.parse_args(argv)
    from bcfl.config import IID_PROTOCOL
    extra = dict(IID_PROTOCOL) if a.protocol == "iid" else {}
    extra.pop("keep_optimizer_state", None)   # governed by --fresh-adamw
    for it in a.set:
        k, _, v = it.partition("=")
        try:
            extra[k.strip()] = json.loads(v)
        except json.JSONDecodeError:
            extra[k.strip()] = v
    res = {"reference": {"latency_min_server": [38, 41.8, 45.4], "latency_min_serverless": [27.8, 40, 41.5],
                         "acc_server": [68, 74, 80], "acc_serverless": [76, 83, 88],
                         "source": "All_graphs_IMDB_dataset.ipynb:747-748,830-831 (5/10/20 workers, 20 rounds, hardware unspecified, pretrained models)"},
           "runs": []}
    for k in a.clients:
        for mode in a.modes:
            rec = one(mode, k, a.rounds, os.path.join("runs", "grid", f"{mode}{k}"), a.model,
                      not a.fresh_adamw, **extra)
            print(json.dumps({x: rec[x] for x in rec if x != "accuracy_curve"}), flush=True)
            res["runs"].append(rec)
            os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
            with open(a.out, "w") as fh:
                json.dump(res, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

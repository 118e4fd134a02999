#!/usr/bin/env python
"""Per-round global-accuracy curves (the reference's 20-round charts,
``All_graphs_IMDB_dataset.ipynb:1141-1144``: serverless-IID / serverless-NonIID / server-IID /
server-NonIID) on MI355X, plus learning-rate sweeps for the "learnable from random init" protocol.

Each run is a full federation (default BERT-base, 8 clients, synthetic IMDB-shaped data,
random-init weights) evaluated every round on a class-balanced global draw; the majority-class
rate of that draw is recorded beside the accuracy.

    python benchmarks/accuracy_curves.py --out gpurun_out/curves.json               # 4 reference curves
    python benchmarks/accuracy_curves.py --runs '[{"lr": 5e-4}, {"lr": 2e-4}]'     # sweep
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bcfl  # noqa: E402,F401
from bcfl.config import get_preset  # noqa: E402

# the four reference curves: (label, mode, partition)
CURVES = [
    ("serverless-IID", "serverless", "iid_random"),
    ("serverless-NonIID", "serverless", "label_shards"),
    ("server-IID", "server", "iid_random"),
    ("server-NonIID", "server", "label_shards"),
]


def run_one(preset: str, overrides: dict, rounds: int, label: str) -> dict:
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    kw = {"save_every": 0, "reference_prints": False, "overlap_global_eval": False,
          "out_dir": os.path.join("runs", "curves", str(abs(hash(label)))), **overrides,
          "num_rounds": rounds}
    cfg = get_preset(preset, **kw)
    fed = Federation(cfg, verbose=False)
    t0 = time.perf_counter()
    curve, losses = [], []
    for r in range(rounds):
        rec = fed.run_round(r)
        curve.append(rec["global_acc"])
        losses.append(rec["train_loss"])
        if fed.rt.is_main:
            print(f"[{label}] round {r}: acc={rec['global_acc']:.4f} "
                  f"(majority {rec['global_majority_rate']:.3f}) train_loss={rec['train_loss']:.4f} "
                  f"t={rec['t_round']:.3f}s", flush=True)
    fed.finish()
    D.shutdown()
    return {"label": label, "overrides": overrides, "global_acc": curve, "train_loss": losses,
            "majority_rate": fed.history[-1]["global_majority_rate"],
            "global_eval_rows": fed.history[-1]["global_eval_rows"],
            "wall_s": time.perf_counter() - t0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="baseline3_bert_serverless_noniid")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--runs", default=None, help="JSON list of override dicts (sweep)")
    ap.add_argument("--common", default="{}", help="JSON overrides applied to every run")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    common = json.loads(a.common)
    if a.runs:
        plan = [(json.dumps(o, sort_keys=True), {**common, **o}) for o in json.loads(a.runs)]
    else:
        plan = [(lab, {**common, "mode": m, "partition": p}) for lab, m, p in CURVES]
    res = []
    for label, ov in plan:
        res.append(run_one(a.preset, ov, a.rounds, label))
        if a.out:
            os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
            with open(a.out, "w") as fh:
                json.dump(res, fh, indent=1)
    for x in res:
        print(json.dumps({"label": x["label"], "final_acc": x["global_acc"][-1],
                          "majority_rate": x["majority_rate"], "wall_s": round(x["wall_s"], 1)}))


if __name__ == "__main__":
    main()

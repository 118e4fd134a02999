"""Result charts (reference N9: ``All_graphs_IMDB_dataset.ipynb:733-1150``, bar charts of latency /
accuracy / memory / information-passing time and 20-round accuracy curves, ``savefig(dpi=600)``),
generated from this framework's own outputs instead of hard-coded arrays:

* :func:`accuracy_curves`  — global accuracy per round for one or more ``metrics.jsonl`` runs;
* :func:`round_time_bars`  — mean round time / HBM peak per run;
* :func:`info_passing_bars` — sync vs async passing time per source (``bcfl.trust.report`` JSON or
  ``benchmarks/info_passing.py`` JSON).

    python -m bcfl.utils.plots --metrics runs/a/metrics.jsonl runs/b/metrics.jsonl --out figs/ \\
        [--report report.json] [--dpi 600]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import Dict, List, Optional, Sequence


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def read_metrics(path: str) -> Dict[str, list]:
    rounds, acc, t = [], [], []
    hbm = None
    for line in open(path):
        r = json.loads(line)
        if "round" in r and "client" not in r and "t_round" in r:
            rounds.append(r["round"])
            acc.append(r.get("global_acc"))
            t.append(r["t_round"])
            hbm = r.get("hbm_peak_gb", hbm)
    return {"round": rounds, "global_acc": acc, "t_round": t, "hbm_peak_gb": hbm}


def accuracy_curves(paths: Sequence[str], labels: Optional[Sequence[str]], out: str, dpi: int = 150) -> str:
    plt = _plt()
    fig, ax = plt.subplots(figsize=(6, 4))
    for i, p in enumerate(paths):
        m = read_metrics(p)
        ys = [a * 100 if a is not None else float("nan") for a in m["global_acc"]]
        ax.plot([r + 1 for r in m["round"]], ys, marker="o", ms=3,
                label=(labels[i] if labels else os.path.basename(os.path.dirname(p)) or p))
    ax.set_xlabel("round")
    ax.set_ylabel("global accuracy (%)")
    ax.grid(alpha=0.3)
    ax.legend(fontsize=8)
    fig.tight_layout()
    fig.savefig(out, dpi=dpi)
    plt.close(fig)
    return out


def round_time_bars(paths: Sequence[str], labels: Optional[Sequence[str]], out: str, dpi: int = 150) -> str:
    plt = _plt()
    names, ts = [], []
    for i, p in enumerate(paths):
        m = read_metrics(p)
        names.append(labels[i] if labels else os.path.basename(os.path.dirname(p)) or p)
        ts.append(sum(m["t_round"]) / max(len(m["t_round"]), 1))
    fig, ax = plt.subplots(figsize=(6, 4))
    ax.bar(names, ts, color="tab:blue")
    ax.set_ylabel("mean round time (s)")
    for x, v in enumerate(ts):
        ax.text(x, v, f"{v:.3g}", ha="center", va="bottom", fontsize=8)
    fig.tight_layout()
    fig.savefig(out, dpi=dpi)
    plt.close(fig)
    return out


def info_passing_bars(report: Dict, out: str, dpi: int = 150) -> str:
    plt = _plt()
    rows = report.get("info_passing") or report.get("sources")
    keys = ("sync_s", "async_s") if "sync_s" in rows[0] else ("measured_sync_s", "measured_async_s")
    xs = [r["source"] for r in rows]
    fig, ax = plt.subplots(figsize=(7, 4))
    wdt = 0.4
    ax.bar([x - wdt / 2 for x in xs], [r[keys[0]] for r in rows], wdt, label="synchronous (sum)")
    ax.bar([x + wdt / 2 for x in xs], [r[keys[1]] for r in rows], wdt, label="asynchronous (max)")
    ax.set_xlabel("source node")
    ax.set_ylabel("information passing time (s)")
    ax.set_xticks(xs)
    ax.legend(fontsize=8)
    fig.tight_layout()
    fig.savefig(out, dpi=dpi)
    plt.close(fig)
    return out


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--metrics", nargs="*", default=[])
    ap.add_argument("--labels", nargs="*", default=None)
    ap.add_argument("--report", default=None, help="bcfl.trust.report / info_passing JSON")
    ap.add_argument("--out", default="figs")
    ap.add_argument("--dpi", type=int, default=150)
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    made = []
    if a.metrics:
        made.append(accuracy_curves(a.metrics, a.labels, os.path.join(a.out, "global_accuracy.png"), a.dpi))
        made.append(round_time_bars(a.metrics, a.labels, os.path.join(a.out, "round_time.png"), a.dpi))
    if a.report:
        with open(a.report) as fh:
            made.append(info_passing_bars(json.load(fh), os.path.join(a.out, "info_passing.png"), a.dpi))
    for m in made:
        print(m)
    return 0


if __name__ == "__main__":
    sys.exit(main())

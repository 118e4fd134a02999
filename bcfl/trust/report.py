"""Trust / network analysis report: the reference notebooks' analyses as one command.

Re-runs, on the reference fixture graph (N1, ``All_graphs_IMDB_dataset.ipynb:73-167``) or on a
measured bandwidth matrix (``bcfl.trust.probe`` / ``benchmarks/info_passing.py`` JSON):

* PageRank ±σ anomalies with thresholds (N2, ``:168-180``), DBSCAN (N3, ``:300-314``), modified-Z
  (N4, ``:463-472``), greedy-modularity communities (N5, ``:544-650``);
* information-passing time from every source, sync (Σ) vs async (max) along shortest paths, for a
  model size in GB (N6, ``Medical_Transcriptions_All_graphs.ipynb:974-999``), with and without the
  PageRank-flagged nodes;
* the latency objective: best source minimising D_g + max-path latency (N7, ``:21``).

    python -m bcfl.trust.report [--bw measured.json] [--model-gb 0.4036] [--dg 0] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import Dict, Optional

import numpy as np

from . import graph as G
from .netdata import BIOBERT_GB, REF_BW_MBPS


def analyse(bw: np.ndarray, model_gb: float = BIOBERT_GB, d_g: float = 0.0) -> Dict:
    bw = np.asarray(bw, dtype=np.float64)
    W = np.zeros_like(bw)
    nz = bw > 0
    W[nz] = 1.0 / bw[nz]
    ranks = G.pagerank(W)
    (lo, hi), flags = G.sigma_flags(ranks, 1.0)
    det = G.anomaly_report(bw)
    # bandwidth in Mbps -> GB/s for the passing-time model (size in GB / GB/s = seconds)
    L = G.latency_matrix(bw / 8.0 / 1000.0, model_gb)
    per_src = []
    for s in range(bw.shape[0]):
        t = G.info_passing_time(L, s)
        tf = G.info_passing_time(L, s, [i for i in flags if i != s])
        per_src.append({"source": s, "sync_s": t.sync, "async_s": t.async_,
                        "sync_filtered_s": tf.sync, "async_filtered_s": tf.async_})
    best, obj = G.best_source(L, [], d_g)
    best_f, obj_f = G.best_source(L, flags, d_g)
    return {"n": int(bw.shape[0]), "model_gb": model_gb,
            "pagerank": [float(x) for x in ranks], "pagerank_thresholds": [float(lo), float(hi)],
            "anomalies": det, "info_passing": per_src,
            "best_source": {"node": int(best), "objective_s": float(obj)},
            "best_source_filtered": {"node": int(best_f), "objective_s": float(obj_f)}}


def format_report(rep: Dict) -> str:
    out = [f"PageRank thresholds: ({rep['pagerank_thresholds'][0]}, {rep['pagerank_thresholds'][1]})"]
    for k in ("pagerank", "dbscan", "modz", "louvain"):
        out.append(f"Anomalies ({k}): {[str(i) for i in rep['anomalies'][k]]}")
    out.append(f"Information passing time, model {rep['model_gb']:.4f} GB (sync = sum, async = max):")
    for r in rep["info_passing"]:
        out.append(f"  node {r['source']}: sync {r['sync_s']:.2f} s  async {r['async_s']:.2f} s"
                   f"  | anomalies removed: sync {r['sync_filtered_s']:.2f} s async {r['async_filtered_s']:.2f} s")
    b, bf = rep["best_source"], rep["best_source_filtered"]
    out.append(f"Latency objective: best source {b['node']} ({b['objective_s']:.2f} s); "
               f"with anomalous nodes excluded {bf['node']} ({bf['objective_s']:.2f} s)")
    return "\n".join(out)


def main(argv: Optional[list] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--bw", default=None, help="JSON file with a bandwidth matrix in Mbps (key 'bw_mbps' or a list)")
    ap.add_argument("--model-gb", type=float, default=BIOBERT_GB)
    ap.add_argument("--dg", type=float, default=0.0, help="fixed global-model compute delay D_g (s)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    bw = REF_BW_MBPS
    if a.bw:
        with open(a.bw) as fh:
            d = json.load(fh)
        bw = np.asarray(d["bw_mbps"] if isinstance(d, dict) else d, dtype=np.float64)
    rep = analyse(bw, a.model_gb, a.dg)
    print(format_report(rep))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rep, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

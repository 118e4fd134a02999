#!/usr/bin/env python
"""Condense bench.py JSON lines (multi-rank rehearsals, config records) into one tracked record:
    python scripts/collect_runs.py OUT.json TAG=path/to/bench.json [TAG=...] [--note TEXT]
Keeps the headline numbers, the accuracy curve, the async-gossip semantics and the per-rank
staleness / wait statistics; drops the bulky per-phase spreads."""
import json
import sys

KEEP = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "final_accuracy",
        "final_majority_rate", "accuracy_curve", "global_eval_rows", "final_train_loss",
        "tokens_per_s", "exchange", "p2p_post_measured", "timed_rounds_device_phases_mean_s",
        "timed_rounds_host_phases_mean_s", "hbm_peak_gb", "accuracy_protocol")


def condense(d):
    out = {k: d[k] for k in KEEP if k in d}
    out["config"] = d.get("config", {})
    mr = d.get("multi_rank", {}).get("per_rank")
    if mr:
        out["per_rank"] = [{"stale_rounds_mean": (sum(x for x in p["stale_rounds"] if x is not None)
                                                  / max(1, len(p["stale_rounds"]))),
                            "stale_max": p.get("stale_max"), "wait_s_total": p.get("wait_s_total"),
                            "lead_wait_s_total": p.get("lead_wait_s_total"),
                            "torn": p.get("torn")} for p in mr]
    return out


def main(argv):
    out, note, runs = argv[0], "", {}
    it = iter(argv[1:])
    for a in it:
        if a == "--note":
            note = next(it)
            continue
        tag, _, path = a.partition("=")
        lines = [l for l in open(path) if l.startswith("{")]
        runs[tag] = condense(json.loads(lines[-1]))
    json.dump({"note": note, "runs": runs}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])

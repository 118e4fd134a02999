#!/usr/bin/env python
"""Which host calls of a one-client round take long on the host (and so leave the training stream
without queued work)? Wraps the round's host-side steps with perf_counter timers and runs the
bench unchanged; prints per-call host time (median / max over the timed rounds).

    python scripts/host_block_probe.py --clients 1 --global-test-samples 125 --steps 6 --warmup 2"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

T = collections.defaultdict(list)


def wrap(cls, name, label=None):
    f = getattr(cls, name)

    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T[label or f"{cls.__name__}.{name}"].append(time.perf_counter() - t)
    setattr(cls, name, g)


def main():
    import bench
    from bcfl.fl import evaluation, serverless, trainer
    from bcfl.fl.federation import Federation
    from bcfl.ops import flat as F
    for n in ("_launch_eval_local", "_launch_eval_global", "_resolve_eval", "_resolve_eval_local",
              "test_batches", "_activate", "_deactivate", "_train_client", "_run_deferred"):
        for cls in (Federation, evaluation.EvalMixin,
                    serverless.ServerlessRoundMixin):
            if cls is not None and n in cls.__dict__:
                wrap(cls, n)
    wrap(trainer.LocalTrainer, "evaluate_device")
    F_merkle = F.merkle_root_deferred

    def md(*a, **k):
        t = time.perf_counter()
        try:
            return F_merkle(*a, **k)
        finally:
            T["merkle_root_deferred"].append(time.perf_counter() - t)
    import bcfl.ops as O
    O.merkle_root_deferred = md
    rc = bench.main()
    for k, v in sorted(T.items()):
        v = sorted(v)
        print(f"{k:48s} n={len(v):4d} median {1e3 * v[len(v) // 2]:8.2f} ms  max {1e3 * v[-1]:8.2f} ms",
              file=sys.stderr, flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main() or 0)

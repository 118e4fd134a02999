"""Command-line entry points.

The four canonical reference entry points (reference ``README.md:2-5``) are console scripts with
the same names; each is ``bcfl.cli.main`` with the matching preset, and every FLConfig field can be
overridden (``--num-clients 8 --model bert-base ...``). Multi-GPU::

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m bcfl.cli --preset serverless_NonIID --model bert-base --num-clients 8
"""
from __future__ import annotations

import sys
from typing import List, Optional

from .config import parse_cli


def run_sweep(cfg) -> List[dict]:
    """Client-count scaling sweep (reference C19: ``for NUM_CLIENTS in [5,10,20]`` wrapping a whole
    experiment, ``serverless_cancer_biobert_allclients.py:41-46``): one fresh federation per count,
    each in ``<out_dir>/clients_<n>``, telemetry reset in between. Returns the final records."""
    import os

    from .fl import Federation
    out = []
    for n in cfg.sweep_clients:
        sub = cfg.replace(num_clients=int(n), sweep_clients=[],
                          out_dir=os.path.join(cfg.out_dir, f"clients_{int(n)}"))
        fed = Federation(sub)
        if fed.verbose:
            print(f"NUM_CLIENTS = {int(n)}", flush=True)
        hist = fed.run()
        out.append({"num_clients": int(n), "rounds": len(hist),
                    "global_accuracies": list(fed.global_accuracies),
                    "global_accuracy_rounds": list(fed.global_accuracy_rounds),
                    "mean_round_s": sum(h["t_round"] for h in hist) / max(len(hist), 1)})
    return out


def main(argv: Optional[List[str]] = None, default_preset: Optional[str] = None) -> int:
    import os
    if os.environ.get("BCFL_STACKDUMP"):  # periodic all-thread stack dumps (diagnose stalls)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["BCFL_STACKDUMP"]), repeat=True)
    cfg = parse_cli(argv, default_preset=default_preset)
    from .fl import Federation
    from .parallel import dist as D
    if cfg.sweep_clients:
        run_sweep(cfg)
    else:
        fed = Federation(cfg)
        fed.run()
    D.shutdown()
    return 0


def server_IID(argv=None):
    return main(argv, "server_IID")


def server_NonIID(argv=None):
    return main(argv, "server_NonIID")


def serverless_IID(argv=None):
    return main(argv, "serverless_IID")


def serverless_NonIID(argv=None):
    return main(argv, "serverless_NonIID")


if __name__ == "__main__":
    sys.exit(main())

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


def main(argv: Optional[List[str]] = None, default_preset: Optional[str] = None) -> int:
    cfg = parse_cli(argv, default_preset=default_preset)
    from .fl import Federation
    from .parallel import dist as D
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

"""Bitwise reproducibility of short lane runs with / without the batch prefetcher (GPU
diagnostic): N alternating inline / prefetched 3-round runs, each compared with the first."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_federation import _run  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
ref = None
with tempfile.TemporaryDirectory() as d:
    for i in range(n):
        for pf in (False, True):
            o = _run(os.path.join(d, f"{i}{pf}"), 3, False, num_rounds=3, prefetch_batches=pf)
            if ref is None:
                ref = o
                continue
            dm = float((o[0] - ref[0]).abs().max())
            rows = [c for c in range(o[0].shape[0]) if not torch.equal(o[0][c], ref[0][c])]
            print(i, "prefetch" if pf else "inline", "max|d|", dm, "clients differing", rows,
                  "loss eq", o[1] == ref[1], "roots eq", o[2] == ref[2], flush=True)

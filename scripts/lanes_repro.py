"""Cross-run reproducibility of short 3-lane GPU runs (ROADMAP #8): N runs of the bitwise lanes
test configuration (4 clients on 3 lanes, 3 rounds), each compared with the first — masters,
loss curve and ledger update roots must be bit-identical. Run with BCFL_DEBUG_STREAMS=1 to put the
happens-before checker on every run as well. Prints one JSON line per run and a summary."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_federation import _run  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
import tempfile  # noqa: E402
ref, bad = None, 0
with tempfile.TemporaryDirectory() as d:
    for i in range(n):
        o = _run(os.path.join(d, str(i)), 3, False, num_rounds=3)
        if ref is None:
            ref = o
            print(json.dumps({"run": i, "ref": True}), flush=True)
            continue
        same = torch.equal(o[0], ref[0]) and o[1] == ref[1] and o[2] == ref[2]
        bad += int(not same)
        print(json.dumps({"run": i, "bitwise_equal": same,
                          "max_abs_diff": float((o[0] - ref[0]).abs().max()),
                          "loss_equal": o[1] == ref[1], "roots_equal": o[2] == ref[2]}), flush=True)
print(json.dumps({"runs": n, "differing": bad}), flush=True)

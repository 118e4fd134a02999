"""Cross-run reproducibility of short 3-lane GPU runs (ROADMAP #8): N runs of the bitwise lanes
test configuration (4 clients on 3 lanes, 3 rounds), each compared with the first — masters,
loss curve and ledger update roots must be bit-identical. For a differing run the first differing
ledger block (round, client) and the clients whose masters differ are printed. With
BCFL_DEBUG_STREAMS=1 the happens-before checker runs on every run as well (races printed to
stderr). One JSON line per run and a summary."""
import json
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl.config import FLConfig  # noqa: E402
from bcfl.fl import Federation  # noqa: E402
from bcfl.parallel import dist as D  # noqa: E402


def run(tmp, lanes=3, rounds=3, **kw):
    D.set_runtime_for_tests(None)
    cfg = FLConfig(mode="serverless", model="bert-base-2l", dataset="imdb", num_clients=4,
                   train_samples=64, test_samples=32, global_test_samples=64, num_rounds=rounds,
                   out_dir=tmp, reference_prints=False, client_lanes=lanes, overlap_wgrad=False,
                   async_gossip=False, gossip_transport="rccl", ledger=True, save_every=0,
                   dropout=0.1, drift_correction="scaffold", **kw)
    fed = Federation(cfg, verbose=False)
    fed.run()
    torch.cuda.synchronize()
    blocks = [(b["round"], b["client"], b["kind"], b["update_root"]) for b in fed.ledger.blocks()]
    out = (torch.stack([fed.client_master[c] for c in range(4)]).cpu(),
           [h["train_loss"] for h in fed.history], blocks, fed.stream_races)
    D.set_runtime_for_tests(None)
    return out


n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ref, bad = None, 0
with tempfile.TemporaryDirectory() as d:
    for i in range(n):
        o = run(os.path.join(d, str(i)), lanes)
        races = len(o[3]) if o[3] is not None else None
        if ref is None:
            ref = o
            print(json.dumps({"run": i, "ref": True, "races": races}), flush=True)
            continue
        same = torch.equal(o[0], ref[0]) and o[1] == ref[1] and o[2] == ref[2]
        bad += int(not same)
        rec = {"run": i, "bitwise_equal": same, "races": races}
        if not same:
            first = next((ref[2][k][:3] for k in range(min(len(o[2]), len(ref[2])))
                          if o[2][k] != ref[2][k]), None)
            rec.update(max_abs_diff=float((o[0] - ref[0]).abs().max()),
                       clients_differing=[c for c in range(4) if not torch.equal(o[0][c], ref[0][c])],
                       loss_equal=o[1] == ref[1],
                       first_loss_diff=next((k for k in range(len(o[1])) if o[1][k] != ref[1][k]), None),
                       first_block_diff=first)
        print(json.dumps(rec), flush=True)
print(json.dumps({"runs": n, "lanes": lanes, "differing": bad}), flush=True)

"""Determinism stress test of the training step's kernels under concurrency (ROADMAP #8): L
client replicas of a small BERT train the SAME fixed batch (per replica) with the SAME dropout
keys on L concurrent HIP streams, iteration after iteration, without any optimizer step, so
every iteration must reproduce every gradient bit for bit. An intra-kernel race, an order-
dependent reduction or a buffer shared across streams shows up as an iteration whose gradients
differ from the replica's first; the report names the parameters that differ, in backward order
(the first one listed is closest to the kernel that diverged).

    python scripts/kernel_determinism.py [iters=100] [lanes=3] [--overlap-wgrad]

DET_MODEL (default bert-base-2l) picks the model, DET_SERIAL=1 synchronises after every lane's
step (the no-concurrency control), DET_SAVED=1 checks every saved activation between forward and
backward; BCFL_TORCH_OPS / BCFL_G8_PERSIST bisect the kernels.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402
from bcfl.data.batching import make_packed_batch, pad_packed  # noqa: E402
from bcfl.data.registry import load_split  # noqa: E402
from bcfl.fl.trainer import backward  # noqa: E402
from bcfl.models import build_model  # noqa: E402
from bcfl.parallel.flat import FlatParams  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    iters = int(args[0]) if args else 100
    L = int(args[1]) if len(args) > 1 else 3
    model_name = os.environ.get("DET_MODEL", "bert-base-2l")
    ops.set_wgrad_overlap("--overlap-wgrad" in sys.argv)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    ds = load_split("imdb", "train", 30522, 512)
    lanes = []
    for i in range(L):
        m = build_model(model_name, 2, device=dev, dtype=torch.bfloat16)
        flat = FlatParams.from_model(m, dev, torch.bfloat16)
        rows = np.random.default_rng(100 + i).choice(len(ds), 32, replace=False)
        b = pad_packed(make_packed_batch(ds, rows), 256).to(dev)
        lanes.append({"m": m, "flat": flat, "b": b, "s": torch.cuda.Stream(dev),
                      "rng": (1234 + 7 * i, 99 + i), "ref": None, "bad": 0})
    names = lanes[0]["flat"].names
    order = list(reversed(range(len(names))))   # backward order: head first
    rng = ops.rng.global_rng()
    first_bad = []
    check_saved = os.environ.get("DET_SAVED") == "1"
    for it in range(iters):
        for ln in lanes:
            with torch.cuda.stream(ln["s"]):
                rng.load_state({"seed": ln["rng"][0], "counter": ln["rng"][1]})
                ln["m"].train()
                if check_saved:
                    # every tensor autograd saves is cloned when saved (on the saving stream) and
                    # compared with its clone when backward unpacks it (on the unpacking
                    # stream): a saved activation changed in between is counted, by save order
                    seq, marks = [0], []

                    def pack(t, seq=seq):
                        seq[0] += 1
                        if t.is_cuda and t.numel() > 1:
                            return (t, t.clone(), seq[0])
                        return (t, None, seq[0])

                    def unpack(pk, marks=marks):
                        t, c, i = pk
                        if c is not None:
                            marks.append((i, tuple(t.shape), str(t.dtype), (t != c).sum()))
                        return t
                    with torch.autograd.graph.saved_tensors_hooks(pack, unpack):
                        loss = ops.cross_entropy(ln["m"](ln["b"]), ln["b"].labels)
                    ln["marks"] = marks
                else:
                    loss = ops.cross_entropy(ln["m"](ln["b"]), ln["b"].labels)
                backward(loss)
                ops.join_wgrad(dev)
                g = torch.cat([p.grad.reshape(-1).float() for p in ln["flat"].params])
                ln["out"] = (loss.detach().float().clone(), g)
                ln["flat"].zero_grad()
            if os.environ.get("DET_SERIAL") == "1":   # no cross-lane concurrency (control)
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        for k, ln in enumerate(lanes):
            for i, shp, dt, n in ln.get("marks", []):
                if int(n):
                    print(json.dumps({"iter": it, "lane": k, "saved_tensor_changed": i,
                                      "shape": shp, "dtype": dt, "elements": int(n)}), flush=True)
            loss, g = ln["out"]
            if ln["ref"] is None:
                ln["ref"] = (loss, g)
                continue
            if torch.equal(loss, ln["ref"][0]) and torch.equal(g, ln["ref"][1]):
                continue
            ln["bad"] += 1
            diff = []
            off = 0
            spans = []
            for p in ln["flat"].params:
                spans.append((off, off + p.numel()))
                off += p.numel()
            for j in order:
                a, e = spans[j]
                d = (g[a:e] - ln["ref"][1][a:e]).abs().max().item()
                if d > 0:
                    diff.append((names[j], d))
            rec = {"iter": it, "lane": k, "loss_equal": bool(torch.equal(loss, ln["ref"][0])),
                   "params_differing": len(diff), "first_in_backward_order": diff[:6]}
            first_bad.append(rec)
            print(json.dumps(rec), flush=True)
    print(json.dumps({"iters": iters, "lanes": L, "model": model_name,
                      "overlap_wgrad": "--overlap-wgrad" in sys.argv,
                      "differing_iterations": [ln["bad"] for ln in lanes]}), flush=True)


if __name__ == "__main__":
    main()

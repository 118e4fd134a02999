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
backward, DET_TRACE=1 compares the gradients of the tensors around every LayerNorm, attention and
FFN-down op, DET_PROBE=1 compares every LayerNorm backward's inputs and outputs at kernel time;
BCFL_TORCH_OPS / BCFL_G8_PERSIST bisect the kernels.
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
        same = os.environ.get("DET_SAME_BATCH") == "1"   # same shapes in every lane
        rows = np.random.default_rng(100 + (0 if same else i)).choice(len(ds), 32, replace=False)
        b = pad_packed(make_packed_batch(ds, rows), 256).to(dev)
        lanes.append({"m": m, "flat": flat, "b": b, "s": torch.cuda.Stream(dev),
                      "rng": (1234 + 7 * i, 99 + i), "ref": None, "bad": 0})
    names = lanes[0]["flat"].names
    order = list(reversed(range(len(names))))   # backward order: head first
    rng = ops.rng.global_rng()
    first_bad = []
    check_saved = os.environ.get("DET_SAVED") == "1"
    # DET_PROBE=1: every LayerNorm backward's inputs and outputs, cloned right before / after the
    # kernel on its stream, compared with the replica's first iteration
    probe = os.environ.get("DET_PROBE") == "1"
    from bcfl.ops import functional as F
    trace = None
    if os.environ.get("DET_TRACE") == "1":
        # gradients of the intermediate tensors around every LayerNorm / attention / FFN-down op,
        # cloned when autograd produces them: the first one (in backward order) that differs from
        # the replica's first iteration names the op whose backward diverged
        trace = {"cur": None}

        def hooked(name, fn, argi):
            def wrap(*a, **k):
                out = fn(*a, **k)
                rec = trace["cur"]
                if rec is not None and torch.is_grad_enabled():
                    o = out[0] if isinstance(out, tuple) else out
                    tag = f"{name}#{rec['n']}"
                    rec["n"] += 1
                    if getattr(o, "requires_grad", False):
                        o.register_hook(lambda g, tag=tag: rec["g"].append((tag + ".out", g.detach().clone())))
                    for i in argi:
                        t = a[i]
                        if getattr(t, "requires_grad", False) and t.grad_fn is not None:
                            t.register_hook(lambda g, tag=tag, i=i: rec["g"].append((f"{tag}.in{i}", g.detach().clone())))
                return out
            return wrap
        ops.bias_dropout_add_layernorm = hooked("bdaln", ops.bias_dropout_add_layernorm, (0,))
        ops.varlen_attention = hooked("attn", ops.varlen_attention, (0,))
        ops.linear_after_act = hooked("ffn_down", ops.linear_after_act, (1,))
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
                    if trace is not None:
                        trace["cur"] = ln["tr"] = {"n": 0, "g": []}
                    loss = ops.cross_entropy(ln["m"](ln["b"]), ln["b"].labels)
                    if trace is not None:
                        trace["cur"] = None
                if probe:
                    F._PROBE["bdaln"] = ln["probe"] = []
                backward(loss)
                F._PROBE.pop("bdaln", None)
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
            if probe:
                if ln["ref"] is None:
                    ln["ref_probe"] = ln["probe"]
                else:
                    for j, (a, b) in enumerate(zip(ln["probe"], ln["ref_probe"])):
                        din = [int((x != y).sum()) for x, y in zip(a["in"], b["in"])]
                        din_after = [int((x != y).sum()) for x, y in zip(a["in_after"], a["in"])]
                        dout_ = [int((x != y).sum()) for x, y in zip(a["out"], b["out"])]
                        if any(din) or any(dout_) or a["keys"] != b["keys"]:
                            rows = torch.nonzero((a["out"][0] != b["out"][0]).any(1)).flatten()
                            # the same kernel re-run now, on the inputs cloned right before the
                            # original launch: does it reproduce the reference outputs?
                            x = a["in"]
                            rr = F.native().bdaln_bwd(x[0], x[1], x[2], x[3], x[4], *a["keys"], a["has_b"])
                            torch.cuda.synchronize()
                            rerun_vs_ref = [int((rr[0] != b["out"][0]).sum()), int((rr[2] != b["out"][1]).sum())]
                            rerun_vs_orig = [int((rr[0] != a["out"][0]).sum()), int((rr[2] != a["out"][1]).sum())]
                            # the 16-element groups that differ: (row, first column)
                            dif = (a["out"][0] != b["out"][0])
                            cols = [(int(r_), int(torch.nonzero(dif[r_]).flatten()[0]), int(torch.nonzero(dif[r_]).flatten()[-1]))
                                    for r_ in rows[:4].tolist()]
                            # sample values: this run, the reference, and the other lanes' outputs
                            # of the same call at the same position (cross-lane contamination?)
                            r0 = int(rows[0])
                            c0 = torch.nonzero(dif[r0]).flatten()[:4].tolist()
                            samp = {"got": [float(a["out"][1][r0, c]) for c in c0],
                                    "ref": [float(b["out"][1][r0, c]) for c in c0],
                                    "dout": [float(a["in"][0][r0, c]) for c in c0]}
                            for k2, ln2 in enumerate(lanes):
                                pr2 = ln2.get("probe") if k2 != k else None
                                if pr2 and j < len(pr2) and pr2[j]["out"][1].shape == a["out"][1].shape:
                                    samp[f"lane{k2}"] = [float(pr2[j]["out"][1][r0, c]) for c in c0]
                            print(json.dumps({"iter": it, "lane": k, "ln_bwd_call": j,
                                              "inputs_differing": din, "outputs_differing": dout_,
                                              "inputs_changed_during_kernel": din_after,
                                              "keys_equal": a["keys"] == b["keys"],
                                              "dy_rows": rows[:8].tolist(),
                                              "rerun_vs_ref": rerun_vs_ref, "rerun_vs_orig": rerun_vs_orig,
                                              "row_first_last_col": cols, "samples": samp}), flush=True)
                            break
            if trace is not None:
                if ln["ref"] is None:
                    ln["ref_tr"] = ln["tr"]["g"]
                else:
                    for (tag, a), (_, b) in zip(ln["tr"]["g"], ln["ref_tr"]):
                        if not torch.equal(a, b):
                            nd = int((a != b).sum())
                            rows = torch.nonzero((a != b).reshape(a.shape[0], -1).any(1)).flatten()
                            print(json.dumps({"iter": it, "lane": k, "first_grad_diff": tag,
                                              "shape": list(a.shape), "elements": nd,
                                              "rows": rows[:12].tolist(), "nrows": int(rows.numel()),
                                              "max_abs": float((a.float() - b.float()).abs().max())}),
                                  flush=True)
                            break
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

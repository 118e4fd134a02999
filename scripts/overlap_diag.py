"""Diagnose overlapped-wgrad vs inline gradient differences on one step (bert-base-2l)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bcfl  # noqa: F401,E402
import bcfl.ops as ops
from bcfl.data.batching import make_packed_batch
from bcfl.data.registry import load_split
from bcfl.models import build_model, special_tokens

dev = torch.device("cuda", 0)
name = "bert-base-2l"
cls_id, sep_id, vocab = special_tokens(name)
ds = load_split("imdb", "train", vocab, 512, 1234, cls_id, sep_id)
b = make_packed_batch(ds, np.arange(0, 25000, 781)[:32]).to(dev)


def grads(overlap, on_stream):
    ops.set_wgrad_overlap(overlap)
    m = build_model(name, 2, device=dev, dtype=torch.bfloat16, seed=0, dropout=0.0)
    s = torch.cuda.Stream(dev) if on_stream else torch.cuda.current_stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        m.train()
        loss = ops.cross_entropy(m(b), b.labels)
        loss.backward()
        ops.join_wgrad(dev)
        out = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    return out


ref = grads(False, False)
for ov, st in [(False, True), (True, False), (True, True)]:
    for rep in range(3):
        g = grads(ov, st)
        bad = [(n, (g[n].float() - ref[n].float()).abs().max().item()) for n in ref if not torch.equal(g[n], ref[n])]
        print(f"overlap={ov} stream={st} rep={rep}: {len(bad)} params differ", bad[:6], flush=True)

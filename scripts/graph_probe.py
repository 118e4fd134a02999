"""Upper bound for hipGraph-captured client steps: L lanes of BERT-base (bf16, fp32 master, fused
AdamW), each on its own stream with a fixed packed batch; per-step time of (a) eager issue,
interleaved lane by lane on one host thread (what the federation does), and (b) one captured
graph per lane replayed on the lane's stream. Dropout off and a fixed lr (graph-static)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bcfl  # noqa: E402,F401
from bcfl import ops  # noqa: E402
from bcfl.data.batching import make_packed_batch, pad_packed  # noqa: E402
from bcfl.data.registry import load_split  # noqa: E402
from bcfl.models import build_model  # noqa: E402
from bcfl.parallel.flat import FlatAdamW, FlatParams  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 8
STEPS = 16
dev = torch.device("cuda")
ds = load_split("imdb", "train", 30522, 512)
rs = np.random.default_rng(0)
lanes = []
for i in range(L):
    m = build_model("bert-base", 2, device=dev, dtype=torch.bfloat16, seed=i, dropout=0.0)
    flat = FlatParams.from_model(m, dev, torch.bfloat16)
    opt = FlatAdamW(flat, 2e-5, (0.9, 0.999), 1e-6, 0.0, "hf")
    b = pad_packed(make_packed_batch(ds, rs.choice(len(ds), 32, replace=False)), 256).to(dev)
    m.train()
    lanes.append(dict(m=m, flat=flat, opt=opt, b=b, s=torch.cuda.Stream(), acc=torch.zeros((), device=dev)))


def step(ln):
    loss = ops.cross_entropy(ln["m"](ln["b"]), ln["b"].labels)
    loss.backward()
    ln["opt"].step()
    ln["flat"].zero_grad()
    ln["acc"] += loss.detach()


res = {"lanes": L, "T": [int(ln["b"].num_tokens) for ln in lanes]}
for ln in lanes:  # warm-up (allocator, kernels)
    with torch.cuda.stream(ln["s"]):
        for _ in range(3):
            step(ln)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(STEPS):
    for ln in lanes:
        with torch.cuda.stream(ln["s"]):
            step(ln)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
res["eager_ms_per_client_step"] = 1e3 * (t2 - t0) / (STEPS * L)
res["eager_host_ms_per_client_step"] = 1e3 * (t1 - t0) / (STEPS * L)
print(json.dumps(res), flush=True)

for ln in lanes:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(ln["s"]):
        step(ln)  # one more eager step on the capture stream
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=ln["s"]):
        step(ln)
    ln["g"] = g
torch.cuda.synchronize()
for ln in lanes:
    with torch.cuda.stream(ln["s"]):
        ln["g"].replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(STEPS):
    for ln in lanes:
        with torch.cuda.stream(ln["s"]):
            ln["g"].replay()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
res["graph_ms_per_client_step"] = 1e3 * (t2 - t0) / (STEPS * L)
res["graph_host_ms_per_client_step"] = 1e3 * (t1 - t0) / (STEPS * L)
res["finite"] = bool(all(torch.isfinite(ln["flat"].master).all() for ln in lanes))
print(json.dumps(res), flush=True)

"""Host issue time vs device time of one BERT-base local training step (is the step launch-bound?)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402
from bcfl.data.batching import make_packed_batch, pad_packed  # noqa: E402
from bcfl.data.registry import load_split  # noqa: E402
from bcfl.models import build_model  # noqa: E402
from bcfl.parallel.flat import FlatAdamW, FlatParams  # noqa: E402

dev = torch.device("cuda")
m = build_model("bert-base", 2, device=dev, dtype=torch.bfloat16)
flat = FlatParams.from_model(m, dev, torch.bfloat16)
opt = FlatAdamW(flat, 5e-5, (0.9, 0.999), 1e-6, 0.0, "hf")
ds = load_split("imdb", "train", 30522, 512)
rs = np.random.default_rng(0)
batches = [pad_packed(make_packed_batch(ds, rs.choice(len(ds), 32, replace=False)), 256).to(dev) for _ in range(8)]
m.train()


def step(b):
    loss = ops.cross_entropy(m(b), b.labels)
    loss.backward()
    opt.step()
    flat.zero_grad()


for b in batches:
    step(b)
torch.cuda.synchronize()
res = {}
for phase in ("fwd", "fwd_bwd", "full"):
    ts_cpu, ts_gpu = [], []
    for b in batches * 2:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if phase == "fwd":
            with torch.no_grad():
                ops.cross_entropy(m(b), b.labels)
        elif phase == "fwd_bwd":
            ops.cross_entropy(m(b), b.labels).backward()
            flat.zero_grad()
        else:
            step(b)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ts_cpu.append(t1 - t0)
        ts_gpu.append(t2 - t0)
    res[phase] = (1e3 * float(np.median(ts_cpu)), 1e3 * float(np.median(ts_gpu)))
    print(f"{phase}: host issue {res[phase][0]:.2f} ms, wall {res[phase][1]:.2f} ms", flush=True)
# host-side cost of the optimizer call alone
ops.cross_entropy(m(batches[0]), batches[0].labels).backward()
torch.cuda.synchronize()
t0 = time.perf_counter()
opt.step()
t1 = time.perf_counter()
print(f"opt.step host {1e3 * (t1 - t0):.3f} ms", flush=True)

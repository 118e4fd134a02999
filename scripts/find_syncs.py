"""Report host<->device synchronizing calls inside one training step (torch sync debug mode)."""
import os
import sys
import warnings

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
b = pad_packed(make_packed_batch(ds, np.random.default_rng(0).choice(len(ds), 32, replace=False)), 256).to(dev)
m.train()
for _ in range(2):
    ops.cross_entropy(m(b), b.labels).backward()
    opt.step()
    flat.zero_grad()
torch.cuda.synchronize()
torch.cuda.set_sync_debug_mode("warn")
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    loss = ops.cross_entropy(m(b), b.labels)
    print("---- forward done", flush=True)
    loss.backward()
    print("---- backward done", flush=True)
    opt.step()
    flat.zero_grad()
torch.cuda.set_sync_debug_mode(0)
for x in w:
    print("SYNC:", str(x.message)[:200], "@", x.filename, x.lineno)
import traceback  # noqa: E402,F401

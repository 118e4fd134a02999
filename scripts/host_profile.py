"""Host-side cost of one BERT-base client step (cProfile over 20 steps, GPU): which Python /
dispatch layers dominate the ~7 ms of launch work per step."""
import cProfile
import os
import pstats
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402
from bcfl.data.batching import make_packed_batch, pad_packed  # noqa: E402
from bcfl.data.registry import load_split  # noqa: E402
from bcfl.fl.trainer import LocalTrainer  # noqa: E402
from bcfl.models import build_model  # noqa: E402
from bcfl.parallel.flat import FlatAdamW, FlatParams  # noqa: E402

dev = torch.device("cuda")
m = build_model("bert-base", 2, device=dev, dtype=torch.bfloat16)
flat = FlatParams.from_model(m, dev, torch.bfloat16)
opt = FlatAdamW(flat, 5e-5)
tr = LocalTrainer(m, flat, opt)
ds = load_split("imdb", "train", 30522, 512)
rs = np.random.default_rng(0)
batches = [pad_packed(make_packed_batch(ds, rs.choice(len(ds), 16, replace=False)), 256).to(dev)
           for _ in range(4)]
acc = torch.zeros((), device=dev)
for b in batches:
    tr.step(b, acc)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for i in range(20):
    tr.step(batches[i % 4], acc)
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)

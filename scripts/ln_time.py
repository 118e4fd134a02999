"""Isolated LayerNorm-family kernel bandwidth at the bench shape (T = 11264, H = 768, bf16):
bdaln fwd / bwd (+ its colsum3 reduction), bias_act. Bytes = HBM traffic the kernel must move."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402

dev = torch.device("cuda")
T, H = 11264, 768
C = ops.native()
bf = torch.bfloat16
y = torch.randn(T, H, device=dev, dtype=bf)
r = torch.randn(T, H, device=dev, dtype=bf)
g = torch.ones(H, device=dev, dtype=bf)
b = torch.zeros(H, device=dev, dtype=bf)
bias = torch.zeros(H, device=dev, dtype=bf)


def med(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return float(np.median(ts))


res = {}
for p8 in (0, 26):
    out, z, mean, rstd = C.bdaln_fwd(y, bias, r, g, b, 1e-12, p8, 1, 2)
    tf = med(lambda: C.bdaln_fwd(y, bias, r, g, b, 1e-12, p8, 1, 2))
    dout = torch.randn_like(out)
    tb = med(lambda: C.bdaln_bwd(dout, z, mean, rstd, g, p8, 1, 2, True))
    nb = T * H * 2
    # fwd: read y, r; write out, z.  bwd: read dout, z; write dz (+ dy when dropout)
    res[f"p8={p8}"] = {"fwd_us": tf, "fwd_TBps": 4 * nb / tf / 1e6, "bwd_us": tb,
                       "bwd_TBps": (4 if p8 else 3) * nb / tb / 1e6}
print(json.dumps(res))

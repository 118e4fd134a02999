"""Attention fwd / bwd kernel time at the bench batch shape (dropout 0.1), median of 30 launches.
BCFL_ATTN_WPE=f,q,k selects the occupancy variant (read once per process)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402
from bcfl.data.batching import make_packed_batch, pad_packed  # noqa: E402
from bcfl.data.registry import load_split  # noqa: E402

dev = torch.device("cuda")
ds = load_split("imdb", "train", 30522, 512)
b = pad_packed(make_packed_batch(ds, np.random.default_rng(0).choice(len(ds), 32, replace=False)), 256).to(dev)
qkv = (0.5 * torch.randn(b.num_tokens, 3 * 768, device=dev)).bfloat16()
C = ops.native()
sl2 = float((b.seq_lens.astype(np.float64) ** 2).sum())
fl = 4.0 * sl2 * 12 * 64


def med(fn, n=30):
    for _ in range(3):
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


p8, ka, kb = int(os.environ.get("P8", "26")), 12345, 678
for sc in (None, b.attn_sched):
    out, lse, mask = C.attn_fwd(qkv, b.cu_seqlens, b.max_seqlen, 12, 12, 64, 0.125, False, p8, ka, kb, sc)
    g = torch.randn_like(out)
    tf_ = med(lambda: C.attn_fwd(qkv, b.cu_seqlens, b.max_seqlen, 12, 12, 64, 0.125, False, p8, ka, kb, sc))
    tb = med(lambda: C.attn_bwd(g, qkv, out, lse, b.cu_seqlens, b.max_seqlen, 12, 12, 64, 0.125, False,
                                p8, ka, kb, mask, sc))
    dq = C.attn_bwd(g, qkv, out, lse, b.cu_seqlens, b.max_seqlen, 12, 12, 64, 0.125, False, p8, ka, kb, mask, sc)
    print(json.dumps({"wpe": os.environ.get("BCFL_ATTN_WPE", "3,1,1"), "sched": sc is not None,
                      "p8": p8, "T": int(b.num_tokens),
                      "fwd_us": tf_, "bwd_us": tb, "fwd_tflops": fl / tf_ / 1e6,
                      "bwd_tflops": 2.5 * fl / tb / 1e6,
                      "out_sum": float(out.float().sum()), "dqkv_sum": float(dq.float().abs().sum())}),
          flush=True)

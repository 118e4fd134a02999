"""Isolated attention kernel runs for profiling (fwd + bwd at the bench batch shape)."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops
from bcfl.data.batching import make_packed_batch, pad_packed
from bcfl.data.registry import load_split
dev = torch.device("cuda")
ds = load_split("imdb", "train", 30522, 512)
b = pad_packed(make_packed_batch(ds, np.random.default_rng(0).choice(len(ds), 32, replace=False)), 256).to(dev)
qkv = (0.5 * torch.randn(b.num_tokens, 3 * 768, device=dev)).bfloat16().requires_grad_(True)
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    o = ops.varlen_attention(qkv, b.cu_seqlens, b.cu_host, b.max_seqlen, 12, 12, 64, 0.1, True,
                             sched=b.attn_sched)
    o.backward(torch.ones_like(o))
torch.cuda.synchronize()
print("T", b.num_tokens, "sum L^2", float((b.seq_lens.astype(float) ** 2).sum()))

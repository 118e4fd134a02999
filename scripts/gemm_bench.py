"""Isolated K9 weight-gradient runs at the BERT-base bench shapes (for rocprofv3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402

dev = torch.device("cuda")
M = 11264
shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]
ts = [(torch.randn(M, n, device=dev).bfloat16(), torch.randn(M, k, device=dev).bfloat16()) for n, k in shapes]
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    for g, x in ts:
        ops.wgrad(g, x)
torch.cuda.synchronize()
print("ok")

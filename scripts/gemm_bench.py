"""Isolated 8-phase GEMM runs at the BERT-base bench shapes (for rocprofv3 kernel stats / PMC):
the weight gradients dW = G^T X (COL x COL operands) and, with ``fwd`` as the second argument,
the forward projections y = x W^T (ROW x ROW) of the same layer.

    python scripts/gemm_bench.py [ITERS] [fwd]       (M = BCFL_BENCH_M tokens, default 7680)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402

dev = torch.device("cuda")
M = int(os.environ.get("BCFL_BENCH_M", "7680"))
shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]   # (out features, in features)
ts = [(torch.randn(M, n, device=dev).bfloat16(), torch.randn(M, k, device=dev).bfloat16()) for n, k in shapes]
ws = [torch.randn(n, k, device=dev).bfloat16() for n, k in shapes]
fwd = len(sys.argv) > 2 and sys.argv[2] == "fwd"
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    for (g, x), w in zip(ts, ws):
        ops.wgrad(g, x)
        if fwd:
            ops.native().linear_fwd(x, w, None, -1)
torch.cuda.synchronize()
print("ok")

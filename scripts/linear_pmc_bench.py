"""One linear.hip shape (fwd, bias+GELU epilogue) for PMC collection: python scripts/linear_pmc_bench.py [iters]"""
import sys
import torch
import bcfl  # noqa: F401
from bcfl import ops
dev = torch.device("cuda", 0)
M, N, K = 11264, 3072, 768
x = torch.randn(M, K, device=dev).bfloat16()
w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
b = torch.randn(N, device=dev).bfloat16()
g = torch.randn(M, N, device=dev).bfloat16()
C = ops.native()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    C.linear_fwd(x, w, b, 0)
    C.linear_fwd(x, w, b, -1)
    C.linear_dgrad(g, w, None, -1)
torch.cuda.synchronize()

"""Compare formulations of the weight-gradient GEMM dW[N,K] = G[M,N]^T X[M,K] (M = tokens)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.microbench import timeit  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
M = 11264
res = {}
for name, (N, K) in {"qkv": (2304, 768), "attn_out": (768, 768), "ffn_up": (3072, 768),
                     "ffn_down": (768, 3072)}.items():
    G = torch.randn(M, N, device=dev, dtype=bf)
    X = torch.randn(M, K, device=dev, dtype=bf)
    fl = 2.0 * M * N * K
    Gt = G.t().contiguous()
    Xt = X.t().contiguous()
    out32 = torch.empty(N, K, device=dev, dtype=torch.float32)
    v = {
        "Gt@X": lambda: G.t() @ X,
        "(Xt@G)t": lambda: (X.t() @ G).t(),
        "Gt_contig@X": lambda: Gt @ X,
        "Gt_contig@Xt_contig.t": lambda: Gt @ Xt.t(),
        "transpose+mm": lambda: G.t().contiguous() @ X,
        "fp32_out": lambda: torch.mm(G.t(), X, out_dtype=torch.float32) if hasattr(torch.mm, "__call__") else None,
    }
    r = {}
    for k, f in v.items():
        try:
            t = timeit(f)
            r[k] = {"us": round(t * 1e6, 1), "tflops": round(fl / t / 1e12)}
        except Exception as e:  # noqa: BLE001
            r[k] = str(e)[:80]
    res[name] = r
    print(name, r, flush=True)
json.dump(res, open(sys.argv[1] if len(sys.argv) > 1 else "wgrad.json", "w"), indent=1)

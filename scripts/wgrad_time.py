"""K9 weight-gradient kernel time on the bench shapes (BCFL_WGRAD_PF selects the variant)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402

dev = torch.device("cuda")
C = ops.native()
res = {"pf": os.environ.get("BCFL_WGRAD_PF", "2")}
for (M, N, K, bias) in [(9216, 2304, 768, True), (9216, 768, 768, False), (9216, 3072, 768, True),
                        (9216, 768, 3072, False), (16384, 1024, 1024, False)]:
    g = torch.randn(M, N, device=dev).bfloat16()
    x = torch.randn(M, K, device=dev).bfloat16()
    fn = (lambda: C.wgrad_bias(g, x)) if bias else (lambda: C.wgrad(g, x))
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    res[f"{M}x{N}x{K}{'+b' if bias else ''}"] = {"us": round(us, 1), "tflops": round(2 * M * N * K / us / 1e6, 1)}
    ref = (g.float().t() @ x.float())
    out = C.wgrad(g, x)
    res[f"{M}x{N}x{K}{'+b' if bias else ''}"]["relerr"] = float((out.float() - ref).norm() / ref.norm())
print(json.dumps(res))

"""Diagnostic: the 8-phase GEMM's tail-segment kernel vs the base kernel at a Llama shape
(run with BCFL_G8_TAIL_FORCE=0 / 1: plain STORE GEMMs on the base / tail kernel)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402

C = ops.native()
M, N, K = 8192, 6144, 4096
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
xa = torch.zeros(M, 128, device="cuda", dtype=torch.bfloat16)
bb = torch.zeros(N, 128, device="cuda", dtype=torch.bfloat16)


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)


print("force", os.environ.get("BCFL_G8_TAIL_FORCE"), "linear_fwd_us", t(lambda: C.linear_fwd(x, w, None, -1)),
      "lora_fwd_us", t(lambda: C.lora_fwd(x, w, xa, bb)), flush=True)

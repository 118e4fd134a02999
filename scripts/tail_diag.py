"""Diagnostic: the 8-phase GEMM's tail-segment kernel vs the base kernel at Llama shapes, with
zero and random tail operands, interleaved in one process (BCFL_G8_TAIL_FORCE=1 runs the plain
STORE GEMMs on the tail kernel too)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402

C = ops.native()


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


M = 8192
for name, N, K, nr in (("qkv", 6144, 4096, 48), ("gate_up", 28672, 4096, 32)):
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
    xz = torch.zeros(M, 128, device="cuda", dtype=torch.bfloat16)
    bz = torch.zeros(N, 128, device="cuda", dtype=torch.bfloat16)
    xr, br = xz.clone(), bz.clone()
    xr[:, :nr] = torch.randn(M, nr, device="cuda").bfloat16()
    br[:, :nr] = (torch.randn(N, nr, device="cuda") * 0.02).bfloat16()
    g = torch.randn(M, N, device="cuda").bfloat16()
    a = (torch.randn(nr, K, device="cuda") * 0.02).bfloat16()
    gz = torch.zeros(M, 128, device="cuda", dtype=torch.bfloat16)
    gr = gz.clone()
    gr[:, :nr] = torch.randn(M, nr, device="cuda").bfloat16()
    for rep in range(2):
        print(name, "rep", rep, "force", os.environ.get("BCFL_G8_TAIL_FORCE"),
              "fwd", t(lambda: C.linear_fwd(x, w, None, -1)),
              "lora_fwd0", t(lambda: C.lora_fwd(x, w, xz, bz)),
              "lora_fwdR", t(lambda: C.lora_fwd(x, w, xr, br)),
              "dgrad", t(lambda: C.linear_dgrad(g, w, None, -1)),
              "lora_dgrad0", t(lambda: C.lora_dgrad(g, w, gz, a)),
              "lora_dgradR", t(lambda: C.lora_dgrad(g, w, gr, a)), flush=True)

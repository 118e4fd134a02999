"""Llama-3-8B LoRA MLP / skinny-product kernels at the config-5 shapes: the SwiGLU GEMM epilogues
vs plain tail GEMM (+ the separate SwiGLU pass), and skinny.hip's tall-skinny products vs the
library, with effective HBM bandwidth. One JSON line per measurement.

    python scripts/lora_mlp_bench.py [M]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402

DEV = "cuda"
M = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 8192
H, I = 4096, 14336
C = ops.native()


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def emit(**kw):
    print(json.dumps(kw), flush=True)


SKINNY_ONLY = "--skinny-only" in sys.argv
torch.manual_seed(0)
x = torch.randn(M, H, device=DEV).bfloat16()
wgu = (torch.randn(2 * I, H, device=DEV) * 0.02).bfloat16() if not SKINNY_ONLY else None
if not SKINNY_ONLY:
    xa = torch.zeros(M, 128, device=DEV, dtype=torch.bfloat16)
    xa[:, :32] = torch.randn(M, 32, device=DEV).bfloat16()
    bb = torch.zeros(2 * I, 128, device=DEV, dtype=torch.bfloat16)
    bb[:, :32] = (torch.randn(2 * I, 32, device=DEV) * 0.02).bfloat16()
    fl = 2.0 * M * 2 * I * H
    t_plain = timeit(lambda: C.lora_fwd(x, wgu, xa, bb))
    gu = C.lora_fwd(x, wgu, xa, bb)
    t_sw = timeit(lambda: C.swiglu_fwd(gu))
    t_fused = timeit(lambda: C.lora_fwd_swiglu(x, wgu, xa, bb))
    emit(op="gate_up_fwd", M=M, plain_us=t_plain, swiglu_pass_us=t_sw, fused_us=t_fused,
         plain_tflops=fl / t_plain / 1e6, fused_tflops=fl / t_fused / 1e6)
    wd = (torch.randn(H, I, device=DEV) * 0.02).bfloat16()
    g = torch.randn(M, H, device=DEV).bfloat16()
    gb = torch.zeros(M, 128, device=DEV, dtype=torch.bfloat16)
    gb[:, :16] = torch.randn(M, 16, device=DEV).bfloat16()
    ad = (torch.randn(16, I, device=DEV) * 0.02).bfloat16()
    fl = 2.0 * M * I * H
    t_plain = timeit(lambda: C.lora_dgrad(g, wd, gb, ad))
    dA = C.lora_dgrad(g, wd, gb, ad)
    t_sw = timeit(lambda: C.swiglu_bwd(dA, gu))
    t_fused = timeit(lambda: C.lora_dgrad_swiglu(g, wd, gb, ad, gu))
    emit(op="down_dgrad", M=M, plain_us=t_plain, swiglu_pass_us=t_sw, fused_us=t_fused,
         plain_tflops=fl / t_plain / 1e6, fused_tflops=fl / t_fused / 1e6)
    del gu, dA
for K, R in ((H, 48), (H, 32), (I, 16), (2 * I, 32)):
    X = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(R, K, device=DEV) * 0.02).bfloat16()
    t = timeit(lambda: C.skinny_xwt(X, W, 128, 1.0))
    tl = timeit(lambda: torch.mm(X, W.t()))
    emit(op="skinny_xwt", M=M, K=K, R=R, us=t, lib_us=tl, TBps=M * K * 2 / t / 1e6)
    P = torch.randn(M, R, device=DEV).bfloat16()
    t = timeit(lambda: C.skinny_ptx(P, X, 1.0))
    tl = timeit(lambda: torch.mm(P.t(), X))
    emit(op="skinny_ptx", M=M, N=K, R=R, us=t, lib_us=tl, TBps=M * K * 2 / t / 1e6)
    del X, W, P
    torch.cuda.empty_cache()

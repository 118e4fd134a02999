"""Llama-3-8B projection shapes: fused LoRA tail-segment GEMMs (lora_fwd / lora_dgrad) vs the
two-GEMM path (low-rank product written, base GEMM accumulating), numerics vs fp32 and timings.
Prints one line per shape as it goes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402

DEV = "cuda"
M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
H, I, r = 4096, 14336, 16
SHAPES = [("qkv", 6144, H, 3 * r), ("o", H, H, r), ("gate_up", 2 * I, H, 2 * r), ("down", H, I, r)]
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


out = []
for name, N, K, nr in SHAPES:
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    a = (torch.randn(nr, K, device=DEV) * 0.02).bfloat16()
    bbd = (torch.randn(N, nr, device=DEV) * 0.02).bfloat16()
    xa_p = torch.zeros(M, 128, device=DEV, dtype=torch.bfloat16)
    xa_p[:, :nr] = x @ a.t()
    bb_p = torch.zeros(N, 128, device=DEV, dtype=torch.bfloat16)
    bb_p[:, :nr] = bbd
    rec = {"shape": name, "M": M, "N": N, "K": K, "nr": nr}
    y = C.lora_fwd(x, w, xa_p, bb_p)
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t() + xa_p.float() @ bb_p.float().t()
    rec["fwd_rel"] = float((y.float() - ref).norm() / ref.norm())
    del ref

    def two_fwd():
        yy = torch.mm(xa_p[:, :nr], bb_p[:, :nr].t())
        C.linear_fwd_acc(x, w, yy)
    rec["fwd_tail_us"] = timeit(lambda: C.lora_fwd(x, w, xa_p, bb_p))
    rec["fwd_two_gemm_us"] = timeit(two_fwd)
    g = torch.randn(M, N, device=DEV).bfloat16()
    gb_p = torch.zeros(M, 128, device=DEV, dtype=torch.bfloat16)
    gb_p[:, :nr] = g @ bbd
    dx = C.lora_dgrad(g, w, gb_p, a)
    torch.cuda.synchronize()
    ref = g.float() @ w.float() + gb_p[:, :nr].float() @ a.float()
    rec["dgrad_rel"] = float((dx.float() - ref).norm() / ref.norm())
    del ref

    def two_dgrad():
        d = C.linear_dgrad(g, w, None, -1)
        d.addmm_(gb_p[:, :nr], a)
    rec["dgrad_tail_us"] = timeit(lambda: C.lora_dgrad(g, w, gb_p, a))
    rec["dgrad_two_gemm_us"] = timeit(two_dgrad)
    fl = 2.0 * M * N * K
    rec["fwd_tail_tflops"] = fl / rec["fwd_tail_us"] / 1e6
    rec["dgrad_tail_tflops"] = fl / rec["dgrad_tail_us"] / 1e6
    print(json.dumps(rec), flush=True)
    out.append(rec)
    del x, w, g, y, dx
    torch.cuda.empty_cache()

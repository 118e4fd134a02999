"""linear.hip vs the library GEMM (hipBLASLt through torch) on the bench's shapes (TF/s)."""
import os

import torch
import bcfl  # noqa: F401
from bcfl import ops

dev = torch.device("cuda", 0)


def tf(fn, flop, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    return flop / ms / 1e9, ms * 1e3


C = ops.native()
for M, N, K in [(11264, 2304, 768), (11264, 768, 768), (11264, 3072, 768), (11264, 768, 3072),
                (4096, 4096, 4096), (2048, 14336, 4096)]:
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    g = torch.randn(M, N, device=dev).bfloat16()
    pre = torch.randn(M, K, device=dev).bfloat16()
    f = 2.0 * M * N * K
    r = {"fwd_lib": tf(lambda: torch.nn.functional.linear(x, w, b), f),
         "fwd_gelu_lib": tf(lambda: ops.bias_act(torch.nn.functional.linear(x, w), b, "gelu"), f),
         "dgrad_lib": tf(lambda: g.mm(w), f)}
    for tile in ("0", "1"):
        os.environ["BCFL_LINEAR_TILE"] = tile
        if tile == "1" and (N % 256 or K % 256):
            continue
        r[f"fwd_t{tile}"] = tf(lambda: C.linear_fwd(x, w, b, -1), f)
        r[f"fwd_gelu_t{tile}"] = tf(lambda: C.linear_fwd(x, w, b, 0), f)
        r[f"dgrad_t{tile}"] = tf(lambda: C.linear_dgrad(g, w, None, -1), f)
        r[f"dgrad_dact_t{tile}"] = tf(lambda: C.linear_dgrad(g, w, pre, 0), f)
    os.environ["BCFL_LINEAR_TILE"] = ""
    print(f"M={M} N={N} K={K}: " + "  ".join(f"{k}={v[0]:.0f}" for k, v in r.items()), flush=True)

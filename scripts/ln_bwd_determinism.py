"""Is the LayerNorm backward kernel (bdaln_bwd) bitwise reproducible on FIXED inputs while other
streams keep the GPU busy? (ROADMAP #8 bisection.) Each iteration runs bdaln_bwd on stream A with
the same dout / z / stats / gamma and compares dy, dz, dgamma, dbeta, dbias with the first
iteration; streams B and C run BERT-sized GEMMs and attention concurrently. MODE=acc produces dout
each iteration with the accumulate-into-C dgrad GEMM first (the producer of every LayerNorm
backward's input in the training step).

    python scripts/ln_bwd_determinism.py [iters=300]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bcfl import ops  # noqa: E402
from bcfl.ops._native import native  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    mode = os.environ.get("MODE", "fixed")
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    T, H, I = 9728, 768, 3072
    bf = torch.bfloat16
    dout0 = (torch.randn(T, H, device=dev, generator=g) * 1e-3).to(bf)
    z = torch.randn(T, H, device=dev, generator=g).to(bf)
    mean = z.float().mean(1)
    rstd = torch.rsqrt(z.float().var(1, unbiased=False) + 1e-12)
    gamma = (1 + 0.1 * torch.randn(H, device=dev, generator=g)).to(bf)
    g2 = (torch.randn(T, I, device=dev, generator=g) * 1e-3).to(bf)
    w = (torch.randn(I, H, device=dev, generator=g) * 0.02).to(bf)
    # background load
    xa = torch.randn(T, H, device=dev, generator=g).to(bf)
    wa = (torch.randn(I, H, device=dev, generator=g) * 0.02).to(bf)
    sa, sb, sc = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    C = native()
    ref, bad = None, 0
    torch.cuda.synchronize()
    for it in range(iters):
        with torch.cuda.stream(sb):
            for _ in range(3):
                ops.linear(xa, wa)
        with torch.cuda.stream(sc):
            for _ in range(3):
                C.linear_dgrad(g2, w, None, -1)
        with torch.cuda.stream(sa):
            if mode == "acc":
                dout = dout0.clone()
                C.linear_dgrad_acc(g2, w, dout)
            else:
                dout = dout0
            outs = C.bdaln_bwd(dout, z, mean, rstd, gamma, 26, 12345, 678, True)
            outs = [o.clone() for o in outs if o is not None]
        torch.cuda.synchronize()
        if ref is None:
            ref = outs
            continue
        diff = [int((a != b).sum()) for a, b in zip(outs, ref)]
        if any(diff):
            bad += 1
            rows = torch.nonzero((outs[0] != ref[0]).any(1)).flatten()[:8].tolist()
            print(json.dumps({"iter": it, "elements_differing": diff, "dy_rows": rows}), flush=True)
    print(json.dumps({"iters": iters, "mode": mode, "differing": bad}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Per-op micro-benchmarks on the GPU: achieved TFLOP/s (MFMA ops) and GB/s (memory-bound ops)
for the BERT-base hot path at the bench's batch shape (32 packed IMDB-length rows, T ~ 8.3k).

    python benchmarks/microbench.py [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bcfl import ops  # noqa: E402
from bcfl.data.batching import make_packed_batch, pad_packed  # noqa: E402
from bcfl.data.registry import load_split  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda")
    ds = load_split("imdb", "train", 30522, 512)
    rs = np.random.default_rng(0)
    b = pad_packed(make_packed_batch(ds, rs.choice(len(ds), a.batch, replace=False)), 256).to(dev)
    T = b.num_tokens
    lens = b.seq_lens
    H, I, nh, d = 768, 3072, 12, 64
    res = {"T": T, "batch": a.batch, "mean_len": float(lens.mean())}
    bf = torch.bfloat16
    x = torch.randn(T, H, device=dev, dtype=bf)
    # ---------------- GEMMs (hipBLASLt via torch) ------------------------------------------
    gemms = {}
    for name, (M, N, K) in {"qkv": (T, 3 * H, H), "attn_out": (T, H, H), "ffn_up": (T, I, H),
                            "ffn_down": (T, H, I)}.items():
        A = torch.randn(M, K, device=dev, dtype=bf)
        W = torch.randn(N, K, device=dev, dtype=bf)
        G = torch.randn(M, N, device=dev, dtype=bf)
        fl = 2.0 * M * N * K
        t_f = timeit(lambda: torch.nn.functional.linear(A, W))
        t_dx = timeit(lambda: G @ W)
        t_dw = timeit(lambda: G.t() @ A)
        t_k9 = timeit(lambda: ops.wgrad(G, A))
        t_k9b = timeit(lambda: ops.native().wgrad_bias(G, A))
        t_k9s = timeit(lambda: (ops.wgrad(G, A), G.sum(0)))
        gemms[name] = {"MNK": [M, N, K], "fwd_tflops": fl / t_f / 1e12,
                       "dgrad_tflops": fl / t_dx / 1e12, "wgrad_tflops": fl / t_dw / 1e12,
                       "wgrad_k9_tflops": fl / t_k9 / 1e12,
                       "fwd_us": t_f * 1e6, "dgrad_us": t_dx * 1e6, "wgrad_us": t_dw * 1e6,
                       "wgrad_k9_us": t_k9 * 1e6, "wgrad_k9_fused_bias_us": t_k9b * 1e6,
                       "wgrad_k9_plus_torch_bias_us": t_k9s * 1e6}
    res["gemm"] = gemms
    # ---------------- attention ------------------------------------------------------------------
    qkv = (0.5 * torch.randn(T, 3 * H, device=dev)).to(bf).requires_grad_(True)
    sum_l2 = float((lens.astype(np.float64) ** 2).sum())
    fl_f = 4.0 * sum_l2 * nh * d
    for p in (0.0, 0.1):
        def fwd():
            return ops.varlen_attention(qkv, b.cu_seqlens, b.cu_host, b.max_seqlen, nh, nh, d, p, True)
        t_f = timeit(lambda: fwd())
        out = fwd()
        g = torch.randn_like(out)
        t_fb = timeit(lambda: torch.autograd.grad(fwd(), qkv, g))
        res[f"attn_p{p}"] = {"fwd_us": t_f * 1e6, "fwd_tflops": fl_f / t_f / 1e12,
                             "bwd_us": (t_fb - t_f) * 1e6,
                             "bwd_tflops": 2.5 * fl_f / max(t_fb - t_f, 1e-9) / 1e12}
    # ---------------- LayerNorm / bias-act --------------------------------------------------------
    y = torch.randn(T, H, device=dev, dtype=bf, requires_grad=True)
    r = torch.randn(T, H, device=dev, dtype=bf)
    gm = torch.ones(H, device=dev, dtype=bf, requires_grad=True)
    bt = torch.zeros(H, device=dev, dtype=bf, requires_grad=True)
    bias = torch.zeros(H, device=dev, dtype=bf, requires_grad=True)
    t = timeit(lambda: ops.bias_dropout_add_layernorm(y, bias, r, gm, bt, 1e-12, 0.1, True))
    res["ln_fwd"] = {"us": t * 1e6, "GBps": 4 * T * H * 2 / t / 1e9}
    o = ops.bias_dropout_add_layernorm(y, bias, r, gm, bt, 1e-12, 0.1, True)
    go = torch.randn_like(o)
    t2 = timeit(lambda: torch.autograd.grad(ops.bias_dropout_add_layernorm(y, bias, r, gm, bt, 1e-12, 0.1, True), [y, gm], go))
    res["ln_bwd"] = {"us": (t2 - t) * 1e6, "GBps": 4 * T * H * 2 / (t2 - t) / 1e9}
    h = torch.randn(T, I, device=dev, dtype=bf, requires_grad=True)
    hb = torch.zeros(I, device=dev, dtype=bf, requires_grad=True)
    t = timeit(lambda: ops.bias_act(h, hb, "gelu"))
    res["bias_gelu_fwd"] = {"us": t * 1e6, "GBps": 2 * T * I * 2 / t / 1e9}
    go = torch.randn(T, I, device=dev, dtype=bf)
    t2 = timeit(lambda: torch.autograd.grad(ops.bias_act(h, hb, "gelu"), [h, hb], go))
    res["bias_gelu_bwd"] = {"us": (t2 - t) * 1e6, "GBps": 3 * T * I * 2 / (t2 - t) / 1e9}
    # ---------------- flat-buffer ops (BERT-base 110M params) -------------------------------------
    n = 110_000_000 // 64 * 64
    master = torch.randn(n, device=dev)
    m_, v_ = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    pout = torch.empty(n, device=dev, dtype=bf)
    grads = [torch.randn(n, device=dev, dtype=bf)]
    t = timeit(lambda: ops.adamw_multi_(master, grads, [0], m_, v_, 1, 1e-4, 0.9, 0.999, 1e-6, 0.0, "hf", pout), iters=10)
    res["adamw"] = {"us": t * 1e6, "GBps": n * 28 / t / 1e9}
    nb = [torch.randn(n, device=dev) for _ in range(3)]
    t = timeit(lambda: ops.gossip_mix_(master, nb, 0.25, [0.25] * 3, pout), iters=10)
    res["mix3"] = {"us": t * 1e6, "GBps": n * (8 + 12 + 2) / t / 1e9}
    t = timeit(lambda: ops.merkle_root_sha256(master), iters=5)
    res["sha256_merkle"] = {"us": t * 1e6, "GBps": n * 4 / t / 1e9}
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""gemm8.hip (8-phase LDS-DMA MFMA GEMM): numerics vs an fp32 reference, then interleaved timing
against hipBLASLt (torch.mm) and linear.hip on the BERT-base bench shapes (+ 4096^3 / Llama).

    python scripts/g8_bench.py [--check-only] [--reps 20] [--out gpurun_out/g8.json]
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bcfl  # noqa: E402,F401
from bcfl.ops._native import native  # noqa: E402


def ref_mm(A, B, a_col, b_col):
    a = A.float().t() if a_col else A.float()
    b = B.float() if b_col else B.float().t()
    return a @ b


def mk(M, N, K, a_col, b_col, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    A = (torch.rand((K, M) if a_col else (M, K), generator=g, device=dev) * 2 - 1).bfloat16()
    B = (torch.rand((K, N) if b_col else (N, K), generator=g, device=dev) * 2 - 1).bfloat16()
    return A, B


def check(dev):
    C = native()
    res = []
    cases = [  # M, N, K, a_col, b_col, bm  (the last three: > 256 tiles, persistent grids)
        (512, 256, 128, 0, 0, 256), (1000, 768, 768, 0, 0, 256), (2304, 2304, 768, 0, 0, 256),
        (777, 512, 3072, 0, 0, 256), (512, 768, 256, 0, 1, 256), (1000, 768, 2304, 0, 1, 256),
        (640, 3072, 768, 0, 1, 256), (384, 768, 768, 0, 0, 128), (300, 512, 384, 0, 1, 128),
        (7680, 2304, 768, 0, 0, 128), (7777, 3072, 768, 0, 1, 128), (9000, 1024, 512, 0, 0, 128),
    ]
    for M, N, K, ac, bc, bm in cases:
        A, B = mk(M, N, K, ac, bc, dev, seed=M + N + K)
        ref = ref_mm(A, B, ac, bc)
        out = C.gemm8(A, B, bool(ac), bool(bc), 0, 0, None, None, None, bm, 1, 0)[0]
        torch.cuda.synchronize()
        err = (out.float() - ref).abs().max().item()
        rel = ((out.float() - ref).norm() / ref.norm()).item()
        ok = rel < 1e-2 and err < 0.05 * ref.abs().max().item()
        res.append({"case": [M, N, K, ac, bc, bm], "max_abs": err, "rel": rel, "ok": ok})
        # epilogues on the same operands
        bias = (torch.rand(N, device=dev) - 0.5).bfloat16()
        o1 = C.gemm8(A, B, bool(ac), bool(bc), 1, 0, bias, None, None, bm, 1, 0)[0]
        e1 = ((o1.float() - (ref + bias.float())).norm() / ref.norm()).item()
        h, pre = C.gemm8(A, B, bool(ac), bool(bc), 2, 0, bias, None, None, bm, 1, 0)
        pref = ref + bias.float()
        e2 = ((pre.float() - pref).norm() / pref.norm()).item()
        e2h = ((h.float() - torch.nn.functional.gelu(pre.float())).norm() /
               torch.nn.functional.gelu(pre.float()).norm()).item()
        aux = (torch.rand(M, N, device=dev) * 4 - 2).bfloat16()
        o3 = C.gemm8(A, B, bool(ac), bool(bc), 3, 0, None, aux, None, bm, 1, 0)[0]
        x = aux.float()
        gd = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * 3.141592653589793) ** 0.5
        e3 = ((o3.float() - ref * gd).norm() / (ref * gd).norm()).item()
        base = (torch.rand(M, N, device=dev) - 0.5).bfloat16()
        o4 = base.clone()
        C.gemm8(A, B, bool(ac), bool(bc), 4, 0, None, None, o4, bm, 1, 0)
        e4 = ((o4.float() - (ref + base.float())).norm() / ref.norm()).item()
        epi_ok = max(e1, e2, e2h, e3, e4) < 1e-2
        res[-1].update({"bias": e1, "bias_act_pre": e2, "bias_act_h": e2h, "dact": e3, "accum": e4,
                        "epi_ok": epi_ok})
        # split-K partials
        if K % 256 == 0 and K >= 256:
            kc = (K // 2 + 127) // 128 * 128
            S = -(-K // kc)
            part = C.gemm8(A, B, bool(ac), bool(bc), 5, 0, None, None, None, bm, S, kc)[0]
            e5 = ((part.sum(0) - ref).norm() / ref.norm()).item()
            res[-1]["splitk"] = e5
            res[-1]["epi_ok"] = res[-1]["epi_ok"] and e5 < 1e-2
        print(json.dumps(res[-1]), flush=True)
    return res


def check_wgrad(dev):
    import os
    C = native()
    res = []
    for M, N, K in [(7680, 768, 768), (7777, 2304, 768), (1500, 768, 3072), (11264, 3072, 768)]:
        g = torch.Generator(device=dev).manual_seed(M + N)
        G = (torch.rand(M, N, generator=g, device=dev) * 2 - 1).bfloat16()
        X = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).bfloat16()
        ref = G.float().t() @ X.float()
        rb = G.float().sum(0)
        os.environ["BCFL_WGRAD_G8"] = "1"
        dw, db = C.wgrad_bias(G, X)
        torch.cuda.synchronize()
        e = ((dw.float() - ref).norm() / ref.norm()).item()
        eb = ((db.float() - rb).norm() / rb.norm()).item()
        r = {"wgrad": [M, N, K], "rel": e, "bias_rel": eb, "ok": e < 1e-2 and eb < 1e-2}
        print(json.dumps(r), flush=True)
        res.append(r)
    return res


TR = False


def bench_wgrad(dev, reps):
    import os
    C = native()
    out = []
    for name, M, N, K in [("qkv_wgrad", 7680, 2304, 768), ("attn_out_wgrad", 7680, 768, 768),
                          ("ffn_up_wgrad", 7680, 3072, 768), ("ffn_down_wgrad", 7680, 768, 3072),
                          ("ffn_up_wgrad_11k", 11264, 3072, 768)]:
        g = torch.Generator(device=dev).manual_seed(2)
        G = (torch.rand(M, N, generator=g, device=dev) * 2 - 1).bfloat16()
        X = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).bfloat16()

        def k9():
            os.environ["BCFL_WGRAD_G8"] = "0"
            return C.wgrad_bias(G, X)

        def g8():
            os.environ["BCFL_WGRAD_G8"] = "1"
            return C.wgrad_bias(G, X)
        arms = {"hipblaslt": lambda: (G.t() @ X, G.sum(0)), "k9": k9, "g8": g8}
        if TR:   # the weight gradient as a forward-layout GEMM over transposed operands
            GT, XT = G.t().contiguous(), X.t().contiguous()

            def tr_gemm(gt, xt, bm, S):
                if S == 1:
                    return C.gemm8(gt, xt, False, False, 0, 0, None, None, None, bm, 1, 0)[0]
                kc = (M // S + 63) // 64 * 64
                return C.gemm8(gt, xt, False, False, 5, 0, None, None, None, bm,
                               -(-M // kc), kc)[0].sum(0)
            arms = {"g8_nobias": lambda: C.wgrad(G, X, 0),
                    "transpose_only": lambda: (G.t().contiguous(), X.t().contiguous()),
                    **{f"pre_tr_bm{bm}_s{S}": (lambda bm=bm, S=S: tr_gemm(GT, XT, bm, S))
                       for bm in (128, 256) for S in (1, 2, 4)},
                    "tr_bm128_s2": lambda: tr_gemm(G.t().contiguous(), X.t().contiguous(), 128, 2)}
            ref = G.float().t() @ X.float()
            for k, f in arms.items():
                if k.startswith(("pre_tr", "tr_")):
                    o = f().float()
                    rel = ((o - ref).norm() / ref.norm()).item()
                    assert rel < 1e-2, (k, rel)
        for f in arms.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in arms}
        for _ in range(reps):
            for k, f in arms.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    f()
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / 5)
        fl = 2.0 * M * N * K
        rec = {"shape": name, "M": M, "N": N, "K": K}
        for k, ts in times.items():
            ts.sort()
            rec[k + "_us"] = round(ts[len(ts) // 2] * 1000, 1)
            rec[k + "_tflops"] = round(fl / (ts[len(ts) // 2] * 1e-3) / 1e12, 1)
        print(json.dumps(rec), flush=True)
        out.append(rec)
    os.environ["BCFL_WGRAD_G8"] = "1"
    return out


def bench(dev, reps):
    C = native()
    shapes = [  # name, M, N, K, kind ('fwd' = x W^T, 'dgrad' = g W)
        ("qkv_fwd", 7680, 2304, 768, "fwd"), ("attn_out_fwd", 7680, 768, 768, "fwd"),
        ("ffn_up_fwd", 7680, 3072, 768, "fwd"), ("ffn_down_fwd", 7680, 768, 3072, "fwd"),
        ("qkv_dgrad", 7680, 768, 2304, "dgrad"), ("attn_out_dgrad", 7680, 768, 768, "dgrad"),
        ("ffn_up_dgrad", 7680, 768, 3072, "dgrad"), ("ffn_down_dgrad", 7680, 3072, 768, "dgrad"),
        ("qkv_fwd_11k", 11264, 2304, 768, "fwd"), ("ffn_up_fwd_11k", 11264, 3072, 768, "fwd"),
        ("ffn_down_fwd_11k", 11264, 768, 3072, "fwd"), ("ffn_down_dgrad_11k", 11264, 3072, 768, "dgrad"),
        ("sq4096", 4096, 4096, 4096, "fwd"), ("sq4096_dgrad", 4096, 4096, 4096, "dgrad"),
        ("llama_ffn", 2048, 14336, 4096, "fwd"),
    ]
    out = []
    for name, M, N, K, kind in shapes:
        g = torch.Generator(device=dev).manual_seed(1)
        x = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).bfloat16()
        if kind == "fwd":   # W [N, K]
            W = (torch.rand(N, K, generator=g, device=dev) * 2 - 1).bfloat16()
            arms = {
                "hipblaslt": lambda: torch.mm(x, W.t()),
                "linear_hip": lambda: C.linear_fwd(x, W, None, -1),
                "g8_256": lambda: C.gemm8(x, W, False, False, 0, 0, None, None, None, 256, 1, 0),
                "g8_128": lambda: C.gemm8(x, W, False, False, 0, 0, None, None, None, 128, 1, 0),
            }
        else:               # W [K_out, N_in], x plays g [M, K_out]
            W = (torch.rand(K, N, generator=g, device=dev) * 2 - 1).bfloat16()
            arms = {
                "hipblaslt": lambda: torch.mm(x, W),
                "linear_hip": lambda: C.linear_dgrad(x, W, None, -1),
                "g8_256": lambda: C.gemm8(x, W, False, True, 0, 0, None, None, None, 256, 1, 0),
                "g8_128": lambda: C.gemm8(x, W, False, True, 0, 0, None, None, None, 128, 1, 0),
            }
        for f in arms.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in arms}
        for _ in range(reps):  # interleaved rounds (one process, one device)
            for k, f in arms.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    f()
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / 5)
        fl = 2.0 * M * N * K
        rec = {"shape": name, "M": M, "N": N, "K": K}
        for k, ts in times.items():
            ts.sort()
            rec[k + "_us"] = round(ts[len(ts) // 2] * 1000, 1)
            rec[k + "_tflops"] = round(fl / (ts[len(ts) // 2] * 1e-3) / 1e12, 1)
        print(json.dumps(rec), flush=True)
        out.append(rec)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--wgrad-only", action="store_true")
    ap.add_argument("--wgrad-transposed", action="store_true",
                    help="time the weight gradient as a forward-layout GEMM on transposed operands")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/g8.json")
    a = ap.parse_args()
    dev = torch.device("cuda")
    global TR
    TR = a.wgrad_transposed
    t0 = time.time()
    res = {"check": check(dev), "check_wgrad": check_wgrad(dev)}
    ok = all(r["ok"] and r["epi_ok"] for r in res["check"]) and all(r["ok"] for r in res["check_wgrad"])
    print("CHECK", "PASS" if ok else "FAIL", flush=True)
    if ok and not a.check_only:
        res["bench_wgrad"] = bench_wgrad(dev, a.reps)
        if not a.wgrad_only:
            res["bench"] = bench(dev, a.reps)
    res["wall_s"] = time.time() - t0
    import os
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

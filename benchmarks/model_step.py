#!/usr/bin/env python
"""One client's training step, timed per step with a progress line each: model build time, step
time, achieved model TFLOP/s and HBM peak for any registered model (BERT-base ... Llama-3-8B LoRA).

    python benchmarks/model_step.py --model llama3-8b-lora --batch 8 --steps 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bcfl import ops  # noqa: E402
from bcfl.data.batching import make_packed_batch, pad_packed  # noqa: E402
from bcfl.data.registry import load_split  # noqa: E402
from bcfl.models import build_model, special_tokens  # noqa: E402
from bcfl.parallel.flat import FlatAdamW, FlatParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--lr", type=float, default=2e-4)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    cls_id, sep_id, vocab = special_tokens(a.model)
    model = build_model(a.model, 2, device=dev, dtype=torch.bfloat16, seed=0)
    flat = FlatParams.from_model(model, dev, torch.bfloat16)
    opt = FlatAdamW(flat, lr=a.lr)
    torch.cuda.synchronize()
    n_all = sum(p.numel() for p in model.parameters())
    n_tr = flat.num_params
    print(f"built {a.model}: {n_all / 1e9:.3f} B params ({n_tr / 1e6:.2f} M trainable) in "
          f"{time.perf_counter() - t0:.1f} s, HBM {torch.cuda.memory_allocated() / 2**30:.1f} GiB",
          flush=True)
    ds = load_split("imdb", "train", vocab, a.seq, 1234, cls_id, sep_id)
    rng = np.random.default_rng(0)
    res = []
    for s in range(a.steps + 1):
        idx = rng.choice(len(ds), a.batch, replace=False)
        b = pad_packed(make_packed_batch(ds, idx), 256).to(dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        model.train()
        loss = ops.cross_entropy(model(b), b.labels)
        loss.backward()
        ops.join_wgrad()
        opt.step()
        flat.zero_grad()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t1
        T = b.real_tokens
        # matmul FLOPs: frozen base = fwd + dgrad (4N), fully trained = fwd + dgrad + wgrad (6N)
        f_per_tok = (4 if n_tr < 0.5 * n_all else 6) * n_all
        tf = f_per_tok * T / dt / 1e12
        print(f"step {s}: {dt * 1e3:.1f} ms  T={T}  loss={loss.item():.4f}  ~{tf:.0f} TFLOP/s (linear)  "
              f"HBM peak {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB", flush=True)
        if s > 0:
            res.append({"ms": dt * 1e3, "tokens": T, "tflops": tf})
    out = {"model": a.model, "batch": a.batch, "params_b": n_all / 1e9, "trainable_m": n_tr / 1e6,
           "median_ms": float(np.median([r["ms"] for r in res])),
           "median_tflops": float(np.median([r["tflops"] for r in res])),
           "hbm_peak_gib": torch.cuda.max_memory_allocated() / 2**30}
    print(json.dumps(out), flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Probe: library GEMMs (hipBLASLt via torch) issued concurrently from two HIP streams, at the
Llama-3-8B LoRA layer shapes. Prints per-group progress so a hang is attributed to a shape group."""
import sys
import time

import torch

dev = torch.device("cuda", 0)
T = int(sys.argv[1]) if len(sys.argv) > 1 else 2304
H, I, r = 4096, 14336, 16
groups = {
    "qkv": (T, 6144, H), "o": (T, H, H), "gate_up": (T, 2 * I, H), "down": (T, H, I),
    "lora_A": (T, 3 * r, H), "lora_B": (T, H, r), "dgrad_qkv": (T, H, 6144), "dgrad_down": (T, I, H),
    "lora_wgrad_A": (3 * r, H, T), "lora_wgrad_B": (H, r, T),
}
streams = [torch.cuda.Stream() for _ in range(2)]
for name, (M, N, K) in groups.items():
    a = [torch.randn(M, K, device=dev, dtype=torch.bfloat16) for _ in streams]
    b = [torch.randn(K, N, device=dev, dtype=torch.bfloat16) for _ in streams]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        for s, x, y in zip(streams, a, b):
            with torch.cuda.stream(s):
                x @ y
    torch.cuda.synchronize()
    print(f"{name:14s} M={M} N={N} K={K}: ok {1e3 * (time.perf_counter() - t0) / 20:.2f} ms/iter", flush=True)
print("all ok", flush=True)

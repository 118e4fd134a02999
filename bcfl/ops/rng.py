"""Counter-based dropout RNG shared bit-for-bit by the HIP kernels and the torch reference.

One 32-bit hash yields four 8-bit dropout decisions (element ``e`` uses byte ``e & 3`` of
``hash(e >> 2)``), as flash-attention implementations do: the per-element cost must stay far
below the MFMA work it rides on. Dropout probability is quantised to ``p8 / 256``.

hash(x) = lowbias32 with two key injections::

    x ^= ka; x ^= x >> 16; x *= 0x7feb352d; x ^= kb; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16

Keys come from a per-process generator state (seed, counter); every dropout call consumes one
counter value so forward and backward of the same call regenerate the same mask.
"""
from __future__ import annotations

import threading
from typing import Tuple

import torch

M32 = 0xFFFFFFFF


def _lowbias32_int(x: int) -> int:
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def derive_keys(seed: int, counter: int) -> Tuple[int, int]:
    a = _lowbias32_int(seed ^ _lowbias32_int(counter * 2 + 1))
    b = _lowbias32_int(a ^ 0x9E3779B9 ^ _lowbias32_int(counter * 2 + 2))
    return a, b


def quantize_p(p: float) -> int:
    return max(0, min(255, int(round(p * 256.0))))


def keep_scale(p8: int) -> float:
    return 0.0 if p8 >= 256 else 256.0 / (256.0 - p8)


class DropoutRNG:
    """Per-process (seed, counter) stream."""

    def __init__(self, seed: int = 0):
        self.seed = seed & M32
        self.counter = 0
        self._lock = threading.Lock()

    def next(self) -> Tuple[int, int]:
        with self._lock:
            c = self.counter
            self.counter += 1
        return derive_keys(self.seed, c)

    def state(self):
        return {"seed": self.seed, "counter": self.counter}

    def load_state(self, st):
        self.seed, self.counter = int(st["seed"]), int(st["counter"])


_GLOBAL = DropoutRNG(0)


def global_rng() -> DropoutRNG:
    return _GLOBAL


def manual_seed(seed: int) -> None:
    _GLOBAL.seed = seed & M32
    _GLOBAL.counter = 0


# ----------------------------- torch reference of the hash -----------------------------------

def _mulmod32(x: torch.Tensor, c: int) -> torch.Tensor:
    lo, hi = c & 0xFFFF, c >> 16
    return (x * lo + (((x * hi) & 0xFFFF) << 16)) & M32


def hash32(x: torch.Tensor, ka: int, kb: int) -> torch.Tensor:
    """x: int64 tensor of values in [0, 2^32)."""
    x = (x ^ ka) & M32
    x = x ^ (x >> 16)
    x = _mulmod32(x, 0x7FEB352D)
    x = x ^ kb
    x = x ^ (x >> 15)
    x = _mulmod32(x, 0x846CA68B)
    x = x ^ (x >> 16)
    return x


def keep_mask_from_index(idx: torch.Tensor, p8: int, ka: int, kb: int) -> torch.Tensor:
    """Boolean keep-mask for int64 element indices ``idx`` (uint32 wrap)."""
    idx = idx & M32
    h = hash32(idx >> 2, ka, kb)
    byte = (h >> ((idx & 3) * 8)) & 0xFF
    return byte >= p8


def keep_mask(numel: int, p8: int, ka: int, kb: int, device="cpu") -> torch.Tensor:
    return keep_mask_from_index(torch.arange(numel, dtype=torch.int64, device=device), p8, ka, kb)

"""Flat-buffer ops: fused AdamW (K10), FedAvg/gossip mixing (K11), sketches and SHA-256 Merkle.

Every federated exchange in bcfl works on ONE contiguous buffer per client (parameters are views
into it), so each op here is a single kernel launch over the whole model instead
of the reference's per-tensor Python loops (HF AdamW over 201 tensors; ``sum(param)/len(param)``
over ``zip(*aggregated_params)`` at ``src/Serverlesscase/serverless_IID_IMDB.py:269``).
"""
from __future__ import annotations

import hashlib
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import ref
from ._native import native, use_native

LEAF_BYTES_DEFAULT = 1 << 12  # 4 KiB Merkle leaves (~100k leaves for BERT-base: fills the GPU)


def adamw_(master, grad, m, v, step: int, lr: float, beta1: float, beta2: float, eps: float,
           weight_decay: float, mode: str = "hf", param_out: Optional[torch.Tensor] = None,
           grad_scale: float = 1.0):
    if use_native(master):
        native().adamw(master, grad, m, v, param_out, float(lr), float(beta1), float(beta2),
                       float(eps), float(weight_decay), int(step), 0 if mode == "hf" else 1,
                       float(grad_scale))
        return
    ref.adamw_(master, grad, m, v, step, lr, beta1, beta2, eps, weight_decay, mode, param_out,
               grad_scale)


def adamw_multi_(master, grads: Sequence[torch.Tensor], offsets: Sequence[int], m, v, step: int,
                 lr: float, beta1: float, beta2: float, eps: float, weight_decay: float,
                 mode: str = "hf", param_out: Optional[torch.Tensor] = None,
                 grad_scale: float = 1.0, corr: Optional[torch.Tensor] = None,
                 corr_lr: float = 0.0, grads2: Optional[Sequence[torch.Tensor]] = None,
                 gscale: Optional[torch.Tensor] = None):
    """AdamW where each gradient is its own tensor (as autograd produced it) and master / m / v /
    param live in flat buffers at ``offsets``: one multi-tensor launch per <=40 tensors.

    ``corr`` (flat fp32, optional): drift correction in update space, applied in the same pass as
    ``p -= corr_lr * corr`` on every element that received a gradient (bcfl.fl.drift).
    ``grads2`` (optional, aligned with ``grads``): a second gradient of each tensor — the
    micro-batch replica's — summed in the same pass (no separate accumulation kernel).
    ``gscale`` (optional, device fp32 ``[coef, ...]``): a gradient multiplier read on the device
    (the global-norm clip coefficient of :func:`grad_clip_coef`)."""
    if not grads:
        return
    if grads2 is not None and len(grads2) != len(grads):
        raise ValueError("grads2 must align with grads")
    if use_native(master, "adamw"):
        native().adamw_mt(master, m, v, param_out, list(grads), [int(o) for o in offsets],
                          float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
                          int(step), 0 if mode == "hf" else 1, float(grad_scale), corr,
                          float(corr_lr), list(grads2) if grads2 is not None else [], gscale)
        return
    if grads2 is not None:
        grads = [g + g2 for g, g2 in zip(grads, grads2)]
    if gscale is not None:
        grad_scale = grad_scale * float(gscale[0])
    for g, o in zip(grads, offsets):
        n = g.numel()
        po = None if param_out is None or param_out.data_ptr() == master.data_ptr() else param_out[o:o + n]
        ref.adamw_(master[o:o + n], g.reshape(-1), m[o:o + n], v[o:o + n], step, lr, beta1, beta2,
                   eps, weight_decay, mode, None if corr is not None else po, grad_scale)
        if corr is not None:
            master[o:o + n].sub_(corr[o:o + n], alpha=corr_lr)
            if po is not None:
                po.copy_(master[o:o + n])


def grad_clip_coef(grads: Sequence[torch.Tensor], max_norm: float,
                   grads2: Optional[Sequence[torch.Tensor]] = None) -> torch.Tensor:
    """``[min(1, max_norm / (||g||_2 + 1e-6)), ||g||_2]`` over all gradients (``g + g2`` per
    tensor with a micro-batch replica) as a 2-element fp32 tensor on the gradients' device —
    ``torch.nn.utils.clip_grad_norm_`` semantics, consumed by :func:`adamw_multi_` (``gscale``)
    without a host sync. GPU: a multi-tensor partial-sum kernel + one deterministic finisher."""
    if grads2 is not None and len(grads2) != len(grads):
        raise ValueError("grads2 must align with grads")
    if grads and use_native(grads[0], "adamw"):
        return native().grad_clip_coef(list(grads), list(grads2) if grads2 is not None else [],
                                       float(max_norm))
    tot = torch.zeros((), dtype=torch.float64, device=grads[0].device if grads else "cpu")
    for i, g in enumerate(grads):
        x = g.float() if grads2 is None else g.float() + grads2[i].float()
        tot += (x.double() ** 2).sum()
    norm = tot.sqrt().float()
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    return torch.stack([coef, norm])


def gossip_mix_(master: torch.Tensor, neighbours: Sequence[torch.Tensor], self_w: float,
                weights: Sequence[float], param_out: Optional[torch.Tensor] = None):
    """master <- self_w * master + sum_j w_j * neighbour_j (fp32 accumulate; neighbours any dtype)."""
    if use_native(master):
        native().mix(master, list(neighbours), float(self_w), [float(w) for w in weights], param_out)
        return
    ref.gossip_mix_(master, neighbours, self_w, weights, param_out)


def weighted_accumulate_(acc: torch.Tensor, x: torch.Tensor, w: float):
    if use_native(acc):
        native().axpby(acc, x, float(w), 1.0)
        return
    ref.weighted_accumulate_(acc, x, w)


def axpby_(y: torch.Tensor, x: torch.Tensor, a: float, b: float):
    """y <- a*x + b*y."""
    if use_native(y):
        native().axpby(y, x, float(a), float(b))
        return
    y.mul_(b).add_(x.to(y.dtype), alpha=a)


def delta_round_end_(y: torch.Tensor, x: torch.Tensor, cum: torch.Tensor, wire: torch.Tensor,
                     param_out: Optional[torch.Tensor] = None, d: Optional[torch.Tensor] = None,
                     cv: Optional[torch.Tensor] = None, inv_l: float = 0.0, scale: float = 0.0):
    """Round end of one client under round-complete delta gossip, one pass (elementwise.hip):
    ``u = y - x; cum += u; wire[:n] = cum; [cv = (x - y) inv_l - scale d; wire[n:] = cv];
    y = x; param_out = x``."""
    if use_native(y):
        native().delta_round_end(y, x, cum, wire, param_out, d, cv, float(inv_l), float(scale))
        return
    ref.delta_round_end_(y, x, cum, wire, param_out, d, cv, inv_l, scale)


def scale_(x: torch.Tensor, a: float):
    if use_native(x):
        native().axpby(x, x, 0.0, float(a))
        return
    x.mul_(a)


def cast_copy_(dst: torch.Tensor, src: torch.Tensor):
    if use_native(dst) and dst.dtype != src.dtype:
        native().cast_copy(dst, src)
        return
    dst.copy_(src)


def block_sketch(x: torch.Tensor, dim: int, seed: int = 0x5EED) -> torch.Tensor:
    if use_native(x):
        from .rng import derive_keys
        ka, kb = derive_keys(seed, 0)
        return native().block_sketch(x.contiguous(), int(dim), int(ka), int(kb))
    return ref.block_sketch(x, dim, seed)


def update_stats(a: torch.Tensor, b: torch.Tensor, dim: int, seed: int = 0x5EED):
    """Anomaly-filter statistics of the update ``a - b`` without materialising it: its signed
    block sketch (as :func:`block_sketch`) and its L2 norm, both device fp32 (one fused pass over
    the two operands on GPU; no host sync)."""
    if use_native(a):
        from .rng import derive_keys
        ka, kb = derive_keys(seed, 0)
        out = native().update_stats(a.contiguous(), b.contiguous(), int(dim), int(ka), int(kb))
        return out[:dim], out[dim:].sum().sqrt()
    d = a.reshape(-1).float() - b.reshape(-1).float()
    return ref.block_sketch(d, dim, seed), d.norm()


# ------------------------------- SHA-256 Merkle ----------------------------------------------

def _np_bytes(buf: torch.Tensor) -> np.ndarray:
    t = buf.detach().reshape(-1)
    if t.is_cuda:
        t = t.cpu()
    return t.contiguous().view(torch.uint8).numpy()


def _leaf_digests_host(b: np.ndarray, leaf: int) -> List[bytes]:
    n = max(1, (b.size + leaf - 1) // leaf)
    mv = memoryview(b)
    return [hashlib.sha256(b"\x00" + mv[i * leaf:(i + 1) * leaf].tobytes()).digest()
            for i in range(n)]


def merkle_from_leaves(leaves: Sequence[bytes]) -> bytes:
    level = list(leaves)
    if not level:
        return hashlib.sha256(b"").digest()
    while len(level) > 1:
        nxt = []
        for i in range(0, len(level) - 1, 2):
            nxt.append(hashlib.sha256(b"\x01" + level[i] + level[i + 1]).digest())
        if len(level) % 2:
            nxt.append(level[-1])
        level = nxt
    return level[0]


def leaf_digests_sha256(buf: torch.Tensor, leaf_bytes: int = LEAF_BYTES_DEFAULT) -> torch.Tensor:
    """[n_leaves, 32] uint8 SHA-256(0x00 || leaf) digests (GPU kernel on device buffers)."""
    if use_native(buf):
        return native().sha256_leaves(buf, int(leaf_bytes))
    ds = _leaf_digests_host(_np_bytes(buf), leaf_bytes)
    return torch.from_numpy(np.frombuffer(b"".join(ds), dtype=np.uint8).reshape(-1, 32).copy())


def merkle_root_sha256(buf: torch.Tensor, leaf_bytes: int = LEAF_BYTES_DEFAULT) -> bytes:
    """RFC-6962-style Merkle root over the raw bytes of ``buf``.

    GPU: leaves AND inner levels hashed on device (``sha256_leaves`` + ``sha256_merkle``), only
    the 32-byte root crosses to the host (a 433 MB host SHA-256 would
    dominate a ms-scale round)."""
    if use_native(buf):
        C = native()
        leaves = C.sha256_leaves(buf, int(leaf_bytes))
        root = C.sha256_merkle(leaves)
        return bytes(root.cpu().numpy().tobytes())
    return merkle_from_leaves(_leaf_digests_host(_np_bytes(buf), leaf_bytes))


def merkle_root_deferred(buf: torch.Tensor, leaf_bytes: int = LEAF_BYTES_DEFAULT):
    """Like :func:`merkle_root_sha256` but without the host sync: on GPU the 32-byte root stays a
    device tensor (stream-ordered after the hashing kernels) until :func:`root_bytes` reads it,
    so concurrent client lanes are never stalled by a per-client readback."""
    if use_native(buf):
        C = native()
        return C.sha256_merkle(C.sha256_leaves(buf, int(leaf_bytes)))
    return merkle_root_sha256(buf, leaf_bytes)


def root_bytes(root) -> bytes:
    if isinstance(root, (bytes, bytearray)):
        return bytes(root)
    return bytes(root.cpu().numpy().tobytes())

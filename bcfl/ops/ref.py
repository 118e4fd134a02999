"""PyTorch reference implementations of every bcfl op.

These define the exact math of the HIP kernels (including the dropout masks, which share the
counter-based hash of :mod:`bcfl.ops.rng`). They run the CPU path and are the numerics oracles
for the GPU kernel tests (compute in fp32, cast to the input dtype at the end).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from . import rng as _rng

ATTN_DROP_STRIDE = 8192  # dropout element index = (tq * nh + h) * ATTN_DROP_STRIDE + key_pos


def _dropout(x: torch.Tensor, p8: int, ka: int, kb: int) -> torch.Tensor:
    if p8 <= 0:
        return x
    keep = _rng.keep_mask(x.numel(), p8, ka, kb, device=x.device).view_as(x)
    return x * keep.to(x.dtype) * _rng.keep_scale(p8)


def bias_dropout_add_layernorm(y, bias, residual, gamma, beta, eps: float, p8: int = 0,
                               ka: int = 0, kb: int = 0):
    z = y.float()
    if bias is not None:
        z = z + bias.float()
    z = _dropout(z, p8, ka, kb)
    if residual is not None:
        z = z + residual.float()
    out = F.layer_norm(z, (z.shape[-1],), gamma.float() if gamma is not None else None,
                       beta.float() if beta is not None else None, eps)
    return out.to(y.dtype)


def layernorm(x, gamma, beta, eps: float):
    return F.layer_norm(x.float(), (x.shape[-1],), gamma.float(), beta.float(), eps).to(x.dtype)


def bias_gelu(y, bias, approximate: str = "none"):
    z = y.float() + (bias.float() if bias is not None else 0.0)
    return F.gelu(z, approximate=approximate).to(y.dtype)


def bias_act(y, bias, act: str):
    z = y.float() + (bias.float() if bias is not None else 0.0)
    if act == "gelu":
        r = F.gelu(z)
    elif act == "gelu_new" or act == "gelu_tanh":
        r = F.gelu(z, approximate="tanh")
    elif act == "relu":
        r = F.relu(z)
    elif act == "tanh":
        r = torch.tanh(z)
    elif act == "silu":
        r = F.silu(z)
    else:
        raise KeyError(act)
    return r.to(y.dtype)


def varlen_attention(qkv: torch.Tensor, nh: int, nkv: int, d: int, cu: Sequence[int],
                     scale: float, causal: bool = False, p8: int = 0, ka: int = 0, kb: int = 0,
                     return_lse: bool = False):
    """qkv: [T, (nh + 2*nkv) * d] packed rows; cu: host row boundaries. Returns [T, nh*d]."""
    T = qkv.shape[0]
    q_all = qkv[:, : nh * d].reshape(T, nh, d).float()
    k_all = qkv[:, nh * d: (nh + nkv) * d].reshape(T, nkv, d).float()
    v_all = qkv[:, (nh + nkv) * d:].reshape(T, nkv, d).float()
    rep = nh // nkv
    outs, lses = [], []
    cu = [int(c) for c in cu]
    for b in range(len(cu) - 1):
        s, e = cu[b], cu[b + 1]
        L = e - s
        q = q_all[s:e].transpose(0, 1)  # [nh, L, d]
        k = k_all[s:e].transpose(0, 1).repeat_interleave(rep, dim=0)
        v = v_all[s:e].transpose(0, 1).repeat_interleave(rep, dim=0)
        sc = torch.matmul(q, k.transpose(1, 2)) * scale  # [nh, L, L]
        if causal:
            m = torch.ones(L, L, dtype=torch.bool, device=qkv.device).triu(1)
            sc = sc.masked_fill(m, float("-inf"))
        lse = torch.logsumexp(sc, dim=-1)  # [nh, L]
        p = torch.softmax(sc, dim=-1)
        if p8 > 0:
            tq = torch.arange(s, e, dtype=torch.int64, device=qkv.device)
            hh = torch.arange(nh, dtype=torch.int64, device=qkv.device)
            jj = torch.arange(L, dtype=torch.int64, device=qkv.device)
            idx = ((tq[None, :, None] * nh + hh[:, None, None]) * ATTN_DROP_STRIDE + jj[None, None, :])
            keep = _rng.keep_mask_from_index(idx, p8, ka, kb)
            p = p * keep.to(p.dtype) * _rng.keep_scale(p8)
        o = torch.matmul(p, v)  # [nh, L, d]
        outs.append(o.transpose(0, 1).reshape(L, nh * d))
        lses.append(lse.transpose(0, 1))
    out = torch.cat(outs, 0).to(qkv.dtype) if outs else qkv.new_zeros(0, nh * d)
    if return_lse:
        return out, (torch.cat(lses, 0) if lses else qkv.new_zeros(0, nh).float())
    return out


def embedding_layernorm(ids, pos_ids, type_ids, word_w, pos_w, type_w, gamma, beta, eps: float,
                        p8: int = 0, ka: int = 0, kb: int = 0):
    x = F.embedding(ids.long(), word_w).float()
    if pos_w is not None:
        x = x + F.embedding(pos_ids.long(), pos_w).float()
    if type_w is not None:
        if type_ids is None:
            x = x + type_w[0].float()
        else:
            x = x + F.embedding(type_ids.long(), type_w).float()
    x = F.layer_norm(x, (x.shape[-1],), gamma.float(), beta.float(), eps)
    x = _dropout(x, p8, ka, kb)
    return x.to(word_w.dtype)


def rmsnorm(x, w, eps: float):
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * r * w.float()).to(x.dtype)


def rope_cache(max_pos: int, d: int, theta: float, device="cpu"):
    inv = 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.float64, device=device) / d))
    t = torch.arange(max_pos, dtype=torch.float64, device=device)
    f = torch.outer(t, inv)
    return torch.cos(f).float(), torch.sin(f).float()


def rope(x, pos_ids, cos, sin):
    """x: [T, H, d] (HF rotate_half convention)."""
    d = x.shape[-1]
    c = cos[pos_ids.long()][:, None, :].repeat(1, 1, 2)
    s = sin[pos_ids.long()][:, None, :].repeat(1, 1, 2)
    xf = x.float()
    x1, x2 = xf[..., : d // 2], xf[..., d // 2:]
    rot = torch.cat([-x2, x1], dim=-1)
    return (xf * c + rot * s).to(x.dtype)


def swiglu(gate_up: torch.Tensor) -> torch.Tensor:
    """gate_up: [T, 2I] -> silu(gate) * up, [T, I]."""
    I = gate_up.shape[-1] // 2
    g, u = gate_up[..., :I].float(), gate_up[..., I:].float()
    return (F.silu(g) * u).to(gate_up.dtype)


def cross_entropy(logits, labels):
    return F.cross_entropy(logits.float(), labels.long())


@torch.no_grad()
def adamw_(master: torch.Tensor, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
           step: int, lr: float, beta1: float, beta2: float, eps: float, weight_decay: float,
           mode: str = "hf", param_out: Optional[torch.Tensor] = None, grad_scale: float = 1.0):
    """In-place AdamW on flat fp32 buffers.

    mode "hf": transformers.AdamW (4.35) — p -= lr*sqrt(1-b2^t)/(1-b1^t) * m/(sqrt(v)+eps);
               then p -= lr*wd*p  (eps OUTSIDE the bias correction).
    mode "torch": torch.optim.AdamW — p *= 1-lr*wd; p -= lr/(1-b1^t) * m/(sqrt(v)/sqrt(1-b2^t)+eps).
    """
    g = grad.float() * grad_scale
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    if mode == "hf":
        step_size = lr * math.sqrt(bc2) / bc1
        master.addcdiv_(m, v.sqrt().add_(eps), value=-step_size)
        if weight_decay > 0:
            master.add_(master, alpha=-lr * weight_decay)
    else:
        if weight_decay > 0:
            master.mul_(1 - lr * weight_decay)
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        master.addcdiv_(m, denom, value=-lr / bc1)
    if param_out is not None and param_out.data_ptr() != master.data_ptr():
        param_out.copy_(master)


def weighted_accumulate_(acc: torch.Tensor, x: torch.Tensor, w: float):
    acc.add_(x.float(), alpha=w)


def gossip_mix_(master: torch.Tensor, neighbours: Sequence[torch.Tensor], self_w: float,
                weights: Sequence[float], param_out: Optional[torch.Tensor] = None):
    acc = master.float() * self_w if self_w != 0.0 else torch.zeros_like(master, dtype=torch.float32)
    for t, w in zip(neighbours, weights):
        acc.add_(t.float(), alpha=w)
    master.copy_(acc)
    if param_out is not None and param_out.data_ptr() != master.data_ptr():
        param_out.copy_(master)


def delta_round_end_(y, x, cum, wire, param_out=None, d=None, cv=None, inv_l=0.0, scale=0.0):
    """Reference of the fused round end (same order of operations as the separate passes)."""
    n = y.numel()
    u = y - x
    cum.add_(u)
    wire[:n].copy_(cum)
    if cv is not None:
        c = x * inv_l
        c = c + (-inv_l) * y
        if d is not None:
            c = (-scale) * d + c
        cv.copy_(c)
        wire[n:].copy_(c)
    y.copy_(x)
    if param_out is not None and param_out.data_ptr() != y.data_ptr():
        param_out.copy_(y)


def block_sketch(x: torch.Tensor, dim: int, seed: int = 0x5EED) -> torch.Tensor:
    """Signed block sketch: sketch[k] = sum_{i in block k} s(i) * x[i], s(i) = ±1 from the hash.

    Unbiased for inner products: E[<S x, S y>] = <x, y>. Blocks are contiguous
    ceil(n/dim)-element chunks (no atomics on the GPU: one workgroup per block)."""
    n = x.numel()
    blk = (n + dim - 1) // dim
    ka, kb = _rng.derive_keys(seed, 0)
    idx = torch.arange(n, dtype=torch.int64, device=x.device)
    h = _rng.hash32(idx & _rng.M32, ka, kb)
    s = ((h & 1) * 2 - 1).to(torch.float32)
    xs = x.reshape(-1).float() * s
    pad = blk * dim - n
    if pad:
        xs = torch.cat([xs, xs.new_zeros(pad)])
    return xs.view(dim, blk).sum(1)

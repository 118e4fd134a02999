"""LoRA projections on MFMA (BASELINE config 5, Llama-3-8B LoRA: SURVEY.md §2.6): the frozen base
GEMM with the low-rank update fused into its tail segment, the tall-skinny low-rank products on
skinny.hip, and the fused LoRA SwiGLU MLP (split out of :mod:`bcfl.ops.functional`)."""
from __future__ import annotations

import os
from typing import Optional

import torch

from ._native import available as native_available, native, use_native
from .functional import (WGRAD_MIN_ROWS, _GEMM_PLAIN_NATIVE, _dgrad_gemm, _native_accum_ok, linear, swiglu, wgrad)


def _lora_k2(nr: int) -> int:
    """Low-rank columns appended to the base reduction, padded to whole 128-deep K-tile pairs."""
    return -(-nr // 128) * 128


# _LoRALinear on the tail-segment GEMMs (BCFL_LORA_TAIL=0: the two-GEMM path). At the Llama-3-8B
# shapes (M = 8192) the fused GEMM costs the base GEMM + 1-3 % (scripts/tail_diag.py) and config 5
# goes 17.05 -> 16.53 s/round (profiles/lora_tail_r3.json)
_LORA_TAIL = os.environ.get("BCFL_LORA_TAIL", "1") == "1"


def _lora_tail_ok(m: int, n: int, k: int, nn_: bool, *ts: torch.Tensor) -> bool:
    if not (_LORA_TAIL and _GEMM_PLAIN_NATIVE and all(t.dtype == torch.bfloat16 and t.stride(-1) == 1
                                       and t.stride(0) % 8 == 0 for t in ts)):
        return False
    return bool(native().lora_native_ok(m, n, k, nn_))


_EPI_PARTIAL = 5  # gemm8.hip fp32 split-K partials
# The fused LoRA path computes the four tall-skinny low-rank products with the library by default:
# same-box A/B at config 5 (2 lanes) 16.63 vs 17.07-17.09 s/round for the split-K 8-phase variant
# (BCFL_LORA_G8=1) — the library's small grids co-run with the other lane's GEMMs
# (profiles/lora_tail_r3.json)
_LORA_G8_SKINNY = os.environ.get("BCFL_LORA_G8", "0") == "1"
_LORA_PAD = 256   # the low-rank dimension padded to one 8-phase GEMM column tile
# the four tall-skinny low-rank products on skinny.hip (HBM-bound single passes over x / g);
# BCFL_LORA_SKINNY=0: the library GEMMs (A/B)
_LORA_SKINNY = os.environ.get("BCFL_LORA_SKINNY", "1") == "1"


def _skinny_ok(nr: int, M: int, N: int, K: int) -> bool:
    return (_LORA_SKINNY and nr <= 64 and nr % 8 == 0 and K % 64 == 0 and N % 64 == 0
            and native_available())


def _g8_skinny(A: torch.Tensor, B: torch.Tensor, b_col: bool, ways: int = 4) -> torch.Tensor:
    """C[M, 256] = A[M, K] B (B ROW [256, K] or COL [K, 256]) on the 8-phase GEMM with the reduction
    split ``ways`` ways (a 256-column output alone gives M / 128 workgroups, a quarter of the chip
    at M = 8k); the fp32 slice partials are summed in one pass."""
    K = A.shape[1]
    kc = -(-K // (ways * 128)) * 128
    n = -(-K // kc)
    if n == 1:
        return native().gemm8(A, B, False, b_col, 0, 0, None, None, None, 0, 1, 0)[0]
    part = native().gemm8(A, B, False, b_col, _EPI_PARTIAL, 0, None, None, None, 0, n, kc)[0]
    return part.sum(0).to(A.dtype)


class _LoRALinear(torch.autograd.Function):
    """y = x W^T + s (x A^T) Bbd^T for a FROZEN base W and LoRA adapters (A stacked [n r, K], one
    B_i [o_i, r] per output block i; Bbd = block-diagonal [N, n r]).

    GPU (M >= 1024 tokens), the low-rank dimension n r zero-padded to one 256-column tile:
      xa  = x A_pad^T                      ([M, 256], columns >= n r are zero)
      y   = [x | xa] [W | s Bbd_pad]^T     (the low-rank product as a TAIL segment of the base
                                            GEMM's reduction: no [M, N] delta written / re-read)
      gbs = g (s Bbd_pad)                  ([M, 256])
      dx  = [g | gbs] [W ; A]              (tail segment again)
      dA  = gbs^T x,  dB = s g^T xa
    The four tall-skinny products (xa, gbs, dA, dB) run on the library by default and on split-K
    8-phase GEMMs / the weight-gradient kernel with BCFL_LORA_G8=1: the library's kernels reduce
    M = 8k tokens in a handful of workgroups (16.9 % of config 5's kernel time,
    profiles/config5_kernel_stats_r3.md) but co-run with the other lane's GEMMs, and measured 2.6 %
    faster at the wall. Elsewhere (CPU, small M, other shapes): the low-rank GEMM writes the
    output and the base GEMM accumulates in place."""

    @staticmethod
    def forward(ctx, x, w, a, s, sizes, res, *bs):
        x2 = x.reshape(-1, x.shape[-1])
        if x2.stride(-1) != 1 or x2.stride(0) % 8:
            x2 = x2.contiguous()
        M, N, K = x2.shape[0], w.shape[0], w.shape[1]
        nr = a.shape[0]
        fused = (w.is_contiguous() and a.is_contiguous() and nr <= _LORA_PAD and M >= WGRAD_MIN_ROWS
                 and N % 256 == 0 and K % 256 == 0
                 and _lora_tail_ok(M, N, K, False, x2, w) and _lora_tail_ok(M, K, N, True, x2, w))
        ctx.fused = fused
        ctx.skinny = fused and _skinny_ok(nr, M, N, K)
        ctx.has_res = res is not None
        res2 = None
        if res is not None:
            res2 = res.reshape(-1, N)
            if res2.stride(-1) != 1 or res2.stride(0) % 8:
                res2 = res2.contiguous()
        if ctx.skinny:
            # xa [M, k2] (columns >= n r zero), s Bbd padded + its transpose (one packing kernel)
            xa_f, bb_p, bbt = _lora_skinny_operands(x2, a, bs, s)
            # the residual stream add rides on the GEMM epilogue (EPI_RESID)
            y = native().lora_fwd(x2, w, xa_f, bb_p, res2)
            res2 = None
            ctx.save_for_backward(x2, w, a, xa_f, bbt)
        elif fused:
            bbd = torch.block_diag(*bs)                   # [N, n r]
            k2 = _lora_k2(nr)
            if _LORA_G8_SKINNY:
                a_p = a.new_zeros(_LORA_PAD, K)
                a_p[:nr] = a
                xa_f = _g8_skinny(x2, a_p, False)         # [M, 256]
            else:
                xa_f = x2.new_zeros(M, _LORA_PAD)
                torch.mm(x2, a.t(), out=xa_f[:, :nr])
            bb_p = w.new_zeros(N, _LORA_PAD)
            torch.mul(bbd, s, out=bb_p[:, :nr])
            y = native().lora_fwd(x2, w, xa_f[:, :k2], bb_p[:, :k2])
            ctx.save_for_backward(x2, w, a, xa_f, bb_p)
        else:
            bbd = torch.block_diag(*bs)                   # [N, n r]
            xa = x2 @ a.t()                               # [M, n r]
            y = torch.mm(xa * s, bbd.t())                 # scale on the [M, n r] side
            if w.is_contiguous() and _native_accum_ok(M, N, K, False, x2, w, y):
                native().linear_fwd_acc(x2, w, y)         # base GEMM accumulates in its epilogue
            else:
                y.addmm_(x2, w.t())
            ctx.save_for_backward(x2, w, a, xa, bbd)
        ctx.s, ctx.sizes, ctx.xshape = s, sizes, x.shape
        if res2 is not None:
            y = y + res2
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, g):
        s, sizes = ctx.s, ctx.sizes
        g2 = g.reshape(-1, g.shape[-1])
        if g2.stride(-1) != 1 or g2.stride(0) % 8:
            g2 = g2.contiguous()
        dx = da = None
        dbs = [None] * len(sizes)
        if ctx.skinny:
            x2, w, a, xa_f, bbt = ctx.saved_tensors
            nr, k2 = a.shape[0], xa_f.shape[1]
            C = native()
            # gbs = g (s Bbd) [M, k2] (zero past n r): the dgrad tail operand and dA's left factor
            gbs = C.skinny_xwt(g2, bbt, k2, 1.0)
            if ctx.needs_input_grad[0]:
                dx = C.lora_dgrad(g2, w, gbs, a).view(ctx.xshape)
            if ctx.needs_input_grad[2]:
                da = C.skinny_ptx(gbs[:, :nr], x2, 1.0)           # (s g Bbd)^T x  [n r, K]
            if any(ctx.needs_input_grad[5:]):
                dbs = _lora_db(xa_f[:, :nr], g2, sizes, s)        # s (xa^T g) diagonal blocks^T
            return (dx, None, da, None, None, g if ctx.has_res else None, *dbs)
        if ctx.fused:
            x2, w, a, xa_f, bb_p = ctx.saved_tensors
            nr = a.shape[0]
            if _LORA_G8_SKINNY:
                gbs = _g8_skinny(g2, bb_p, True)          # [M, 256] = g (s Bbd_pad)
            else:
                gbs = g2.new_zeros(g2.shape[0], _LORA_PAD)
                torch.mm(g2, bb_p[:, :nr], out=gbs[:, :nr])
            if ctx.needs_input_grad[0]:
                dx = native().lora_dgrad(g2, w, gbs[:, :_lora_k2(nr)], a).view(ctx.xshape)
            if ctx.needs_input_grad[2]:
                da = (native().wgrad(gbs, x2, 256)[:nr] if _LORA_G8_SKINNY
                      else gbs[:, :nr].t() @ x2)          # (s g Bbd)^T x
            if any(ctx.needs_input_grad[5:]):
                full = (native().wgrad(g2, xa_f, 256)[:, :nr] if _LORA_G8_SKINNY
                        else g2.t() @ xa_f[:, :nr]).mul_(s)  # [N, n r]; block i = dB_i
                r = nr // len(sizes)
                o = 0
                for i, n in enumerate(sizes):
                    dbs[i] = full[o:o + n, i * r:(i + 1) * r].contiguous()
                    o += n
            return (dx, None, da, None, None, g if ctx.has_res else None, *dbs)
        x2, w, a, xa, bbd = ctx.saved_tensors
        gb = g2 @ bbd                                     # [M, n r]
        if ctx.needs_input_grad[0]:
            dx = _dgrad_gemm(g2, w) if w.is_contiguous() else g2 @ w
            dx.addmm_(gb, a, alpha=s)                     # LoRA input gradient, in place
            dx = dx.view(ctx.xshape)
        da = (gb.t() @ x2).mul_(s) if ctx.needs_input_grad[2] else None
        if any(ctx.needs_input_grad[5:]):
            full = (g2.t() @ xa).mul_(s)                  # [N, n r]; block i = dB_i
            r = xa.shape[1] // len(sizes)
            o = 0
            for i, n in enumerate(sizes):
                dbs[i] = full[o:o + n, i * r:(i + 1) * r].contiguous()
                o += n
        return (dx, None, da, None, None, g if ctx.has_res else None, *dbs)


def lora_linear(x: torch.Tensor, w: torch.Tensor, a: torch.Tensor, bs, s: float,
                residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Frozen base projection + LoRA delta (+ ``residual``), fused on the GPU (see
    :class:`_LoRALinear`: the residual add rides on the GEMM epilogue)."""
    if use_native(x, "lora") and not w.requires_grad and x.dtype == torch.bfloat16:
        return _LoRALinear.apply(x, w, a, float(s), tuple(int(b.shape[0]) for b in bs), residual,
                                 *bs)
    xa = linear(x, a)
    r = a.shape[0] // len(bs)
    outs = [linear(xa[..., i * r:(i + 1) * r], b) for i, b in enumerate(bs)]
    d = outs[0] if len(outs) == 1 else torch.cat(outs, dim=-1)
    y = linear(x, w) + d * s
    return y if residual is None else residual + y


def _lora_skinny_operands(x2, a, bs, s):
    """xa = x A^T ([M, k2], zero past n r), s Bbd zero-padded to k2 columns and its transpose
    [n r, N] (skinny.hip: one packing launch instead of block_diag / mul / pad / transpose)."""
    k2 = _lora_k2(a.shape[0])
    xa = native().skinny_xwt(x2, a, k2, 1.0)
    bb, bbt = native().lora_pack_b([b.contiguous() for b in bs], float(s), k2)
    return xa, bb, bbt


def _lora_db(xa: torch.Tensor, g2: torch.Tensor, sizes, s: float):
    """The adapters' B gradients dB_i = s (g^T xa)[block i] as contiguous row blocks of ONE
    [N, r] tensor (the reduce writes the diagonal blocks transposed: no slicing copies)."""
    full = native().skinny_ptx_bdiag(xa, g2, [int(n) for n in sizes], float(s))
    out, o = [], 0
    for n in sizes:
        out.append(full[o:o + n])
        o += n
    return out


class _LoRASwiGLUMLP(torch.autograd.Function):
    """Llama MLP with LoRA on both projections and SwiGLU inside the GEMM epilogues:

        gu  = x Wgu^T + s xa_g Bbd_g^T           act = silu(gate) * up     (ONE GEMM: EPI_SWIGLU)
        y   = res + act Wd^T + s xa_d Bbd_d^T                              (ONE GEMM: EPI_RESID)
      backward:
        dgu = SwiGLU'(gu) . (g Wd + gbs_d Ad)    (ONE GEMM: EPI_SWIGLU_BWD; dA never stored)
        dx  = dgu Wgu + gbs_g Ag                 (tail-segment dgrad)

    versus _LoRALinear + ops.swiglu it saves the SwiGLU forward pass (read gu, write act) and
    backward pass (read dA and gu, write dgu) and the dA tensor (config 5: swiglu fwd + bwd were
    2.8 % of kernel time, profiles/config5_kernel_stats_r3.md). The low-rank products run on
    skinny.hip (see :class:`_LoRALinear`). Reference: the HF LlamaMLP
    ``down_proj(act_fn(gate_proj(x)) * up_proj(x))`` the north star's config 5 trains with PEFT."""

    @staticmethod
    def forward(ctx, x, wgu, agu, sgu, ngu, wd, ad, sd, nd, res, *bs):
        C = native()
        bgu, bd = bs[:ngu], bs[ngu:]
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        res2 = res.reshape(-1, wd.shape[0]).contiguous()
        xa_g, bb_g, bbt_g = _lora_skinny_operands(x2, agu, bgu, sgu)
        act, gu = C.lora_fwd_swiglu(x2, wgu, xa_g, bb_g)
        xa_d, bb_d, bbt_d = _lora_skinny_operands(act, ad, bd, sd)
        y = C.lora_fwd(act, wd, xa_d, bb_d, res2)
        ctx.save_for_backward(x2, wgu, agu, xa_g, bbt_g, gu, act, wd, ad, xa_d, bbt_d)
        ctx.s = (sgu, sd)
        ctx.sizes = (tuple(int(b.shape[0]) for b in bgu), tuple(int(b.shape[0]) for b in bd))
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], wd.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, wgu, agu, xa_g, bbt_g, gu, act, wd, ad, xa_d, bbt_d = ctx.saved_tensors
        (sgu, sd), (zgu, zd) = ctx.s, ctx.sizes
        C = native()
        g2 = gy.reshape(-1, gy.shape[-1]).contiguous()
        nrd, nrg = ad.shape[0], agu.shape[0]
        gbs_d = C.skinny_xwt(g2, bbt_d, xa_d.shape[1], 1.0)
        dgu = C.lora_dgrad_swiglu(g2, wd, gbs_d, ad, gu)
        dad = C.skinny_ptx(gbs_d[:, :nrd], act, 1.0)
        dbd = _lora_db(xa_d[:, :nrd], g2, zd, sd)
        gbs_g = C.skinny_xwt(dgu, bbt_g, xa_g.shape[1], 1.0)
        dx = C.lora_dgrad(dgu, wgu, gbs_g, agu).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dag = C.skinny_ptx(gbs_g[:, :nrg], x2, 1.0)
        dbg = _lora_db(xa_g[:, :nrg], dgu, zgu, sgu)
        return (dx, None, dag, None, None, None, dad, None, None, gy, *dbg, *dbd)


# BCFL_LORA_MLP_FUSED=0: gate|up and down as two _LoRALinear + ops.swiglu (A/B)
_LORA_MLP_FUSED = os.environ.get("BCFL_LORA_MLP_FUSED", "1") == "1"


def _lora_mlp_fused_ok(x: torch.Tensor, wgu, agu, wd, ad) -> bool:
    M, H = x.numel() // x.shape[-1], x.shape[-1]
    I = wd.shape[1]
    return (_LORA_MLP_FUSED and use_native(x, "lora") and x.dtype == torch.bfloat16
            and not wgu.requires_grad and not wd.requires_grad and wgu.is_contiguous()
            and wd.is_contiguous() and agu.is_contiguous() and ad.is_contiguous()
            and wgu.shape == (2 * I, H) and wd.shape[0] == H and M >= WGRAD_MIN_ROWS
            and I % 256 == 0 and H % 256 == 0
            and _skinny_ok(agu.shape[0], M, 2 * I, H) and _skinny_ok(ad.shape[0], M, H, I)
            and bool(native().lora_native_ok(M, 2 * I, H, False))
            and bool(native().lora_native_ok(M, H, I, False))
            and bool(native().lora_native_ok(M, I, H, True))
            and bool(native().lora_native_ok(M, H, 2 * I, True)))


def lora_swiglu_mlp(x: torch.Tensor, wgu: torch.Tensor, agu: torch.Tensor, bgu, sgu: float,
                    wd: torch.Tensor, ad: torch.Tensor, bd, sd: float,
                    residual: torch.Tensor) -> torch.Tensor:
    """residual + down(swiglu(gate_up(x))) with LoRA adapters on both frozen projections
    (:class:`_LoRASwiGLUMLP` on the GPU; elsewhere the two :func:`lora_linear` + :func:`swiglu`)."""
    if _lora_mlp_fused_ok(x, wgu, agu, wd, ad):
        return _LoRASwiGLUMLP.apply(x, wgu, agu, float(sgu), len(bgu), wd, ad, float(sd), len(bd),
                                    residual, *bgu, *bd)
    a = swiglu(lora_linear(x, wgu, agu, bgu, sgu))
    return lora_linear(a, wd, ad, bd, sd, residual)

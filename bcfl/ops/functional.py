"""Public bcfl ops: autograd Functions that run the HIP/CDNA4 kernels on GPU tensors.

Dispatch rule (see :mod:`bcfl.ops._native`): CUDA(HIP) tensors -> ``bcfl._C`` kernels (raise if
the extension is missing); CPU tensors -> :mod:`bcfl.ops.ref` (autograd through torch ops).

Hot-path ops (SURVEY.md §2.6 device-op inventory K1–K11):
  * :func:`bias_dropout_add_layernorm` — K2: LN(dropout(y + b) + residual), one wave64 per row
  * :func:`bias_act`                   — K6: bias + GELU/gelu_new/ReLU/tanh epilogue
  * :func:`varlen_attention`           — K4: flash attention on packed rows (MFMA, online softmax)
  * :func:`embedding_layernorm`        — K1+K2: word+pos+type gather, sum, LN, dropout
  * :func:`rmsnorm`, :func:`rope_`, :func:`swiglu` — Llama path
"""
from __future__ import annotations

import math
import os
from typing import Optional, Sequence

import torch

from . import ref
from . import rng as _rng
from ._native import available as native_available, native, use_native

__all__ = ["bias_dropout_add_layernorm", "layernorm", "bias_act", "varlen_attention",
           "embedding_layernorm", "rmsnorm", "rope", "swiglu", "cross_entropy", "linear", "wgrad",
           "linear_act", "linear_after_act", "gemm_supported", "lora_linear", "lora_swiglu_mlp", "xent_stats_",
           "query_subset_attention", "set_wgrad_overlap", "wgrad_overlap_enabled", "join_wgrad"]


def _keys(p: float, training: bool):
    p8 = _rng.quantize_p(p) if (training and p > 0) else 0
    ka, kb = _rng.global_rng().next() if p8 else (0, 0)
    return p8, ka, kb


WGRAD_MIN_ROWS = 1024  # below this the weight-gradient GEMM is too small to split profitably


def wgrad_supported(g2: torch.Tensor, x2: torch.Tensor) -> bool:
    """Shapes the K9 split-M MFMA weight-gradient kernel takes (bf16, N and K multiples of 128)."""
    return (g2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and g2.shape[0] >= WGRAD_MIN_ROWS
            and g2.shape[1] % 128 == 0 and x2.shape[1] % 128 == 0 and g2.stride(1) == 1
            and x2.stride(1) == 1 and g2.stride(0) % 8 == 0 and x2.stride(0) % 8 == 0)


def wgrad(g2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """dW[N, K] = g2[M, N]^T x2[M, K]: K9 kernel on GPU for supported shapes, library GEMM otherwise."""
    if use_native(g2) and wgrad_supported(g2, x2):
        return native().wgrad(g2, x2)
    return g2.t().mm(x2)


# ----------------------------------------------------------------------------------------
# Overlapped weight gradients: the backward critical path is the chain of input-gradient GEMMs /
# attention / LayerNorm backward kernels; the weight gradients hang off it and are only needed
# by the optimizer. With overlap on, each dW (+db) is launched on a side HIP stream paired with
# the stream autograd runs on, so the K9 kernels fill the CUs the (often sub-wave) dgrad GEMMs
# leave idle; :func:`join_wgrad` makes the optimizer's stream wait for them. Contract: while
# overlap is on, every backward() must be followed by join_wgrad() before the gradients are read
# (LocalTrainer.step does this); parameters that already hold a .grad take the inline path.
# ----------------------------------------------------------------------------------------
_WG = {"enabled": False, "side": {}}


def set_wgrad_overlap(enabled: bool) -> None:
    """Side-stream weight gradients on / off (the weight-gradient kernel is the 8-phase one in
    both regimes; ``native().set_wgrad_kernel(False)`` / BCFL_WGRAD_G8=0 select the K9 kernel)."""
    _WG["enabled"] = bool(enabled)


def wgrad_overlap_enabled() -> bool:
    return _WG["enabled"]


def _side_stream(cur: "torch.cuda.Stream") -> "torch.cuda.Stream":
    key = (cur.device_index, cur.cuda_stream)
    s = _WG["side"].get(key)
    if s is None:
        s = _WG["side"][key] = torch.cuda.Stream(device=cur.device)
    return s


def join_wgrad(device=None) -> None:
    """Current stream waits for the weight gradients launched from it (no-op when none)."""
    if not _WG["side"]:
        return
    cur = torch.cuda.current_stream(device)
    s = _WG["side"].get((cur.device_index, cur.cuda_stream))
    if s is not None:
        cur.wait_stream(s)


def _wgrad_async(g2, x2, want_b):
    cur = torch.cuda.current_stream(g2.device)
    side = _side_stream(cur)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        if want_b:
            dw, db = native().wgrad_bias(g2, x2)
        else:
            dw, db = native().wgrad(g2, x2), None
    # operands are freed by autograd when this node returns; results are read on `cur`
    g2.record_stream(side)
    x2.record_stream(side)
    dw.record_stream(cur)
    if db is not None:
        db.record_stream(cur)
    return dw, db


# Forward / input-gradient GEMMs run on bcfl's own MFMA kernels: linear.hip routes every shape
# it can to the 8-phase LDS-DMA kernel (gemm8.hip), which matches or beats hipBLASLt on all eight
# BERT-base projection shapes (profiles/g8_v1_vs_hipblaslt.json), and keeps its register-staged
# tiles for the rest. BCFL_GEMM_PLAIN=0 sends the plain (epilogue-free) GEMMs back to the
# library (A/B runs); the fused-epilogue GEMMs (bias+GELU forward, GELU' dgrad) always run here.
_GEMM_PLAIN_NATIVE = os.environ.get("BCFL_GEMM_PLAIN", "1") == "1"


def _native_accum_ok(m: int, n: int, k: int, nn_: bool, *ts: torch.Tensor) -> bool:
    """The accumulate-into-C GEMM (beta = 1 epilogue) takes this shape natively (gemm8.hip)."""
    if not (_GEMM_PLAIN_NATIVE and all(t.dtype == torch.bfloat16 and t.stride(-1) == 1
                                       and t.stride(0) % 8 == 0 for t in ts)):
        return False
    return bool(native().gemm_native_ok(m, n, k, nn_, True))


def gemm_supported(x2: torch.Tensor, w: torch.Tensor, nn_: bool = False, op: str = "gemm") -> bool:
    """Shapes the linear.hip MFMA kernels take: bf16, 16-byte aligned contiguous rows, output
    features a multiple of 128 and reduction a multiple of 64 (``nn_``: the dgrad GEMM, whose
    output is the weight's input dim)."""
    if op == "gemm" and not _GEMM_PLAIN_NATIVE:
        return False
    out_f, in_f = w.shape
    n, k = (in_f, out_f) if nn_ else (out_f, in_f)
    return (x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and n % 128 == 0
            and k % 64 == 0 and x2.stride(-1) == 1 and x2.stride(0) % 8 == 0
            and w.is_contiguous() and use_native(x2, op))


def _fwd_gemm(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor]) -> torch.Tensor:
    x2 = x.reshape(-1, x.shape[-1])
    if gemm_supported(x2, w):
        return native().linear_fwd(x2, w, b, -1)[0].view(*x.shape[:-1], w.shape[0])
    return torch.nn.functional.linear(x, w, b)


def _dgrad_gemm(g2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    if gemm_supported(g2, w, nn_=True):
        return native().linear_dgrad(g2, w, None, -1)
    return g2.mm(w)


class ResidualTap:
    """Hands the residual-branch gradient of a bias-dropout-add-LayerNorm straight to the GEMM
    that consumes the same tensor (BERT: ``x`` feeds both the QKV projection and the attention
    LayerNorm's residual; ``x1`` feeds FFN-up and the output LayerNorm's residual).

    Without it autograd receives two [T, H] gradients for that tensor and sums them in a separate
    eager add pass. With it the LayerNorm backward parks ``dres`` here (its residual gradient is
    returned as None) and the consumer's input-gradient GEMM accumulates into it in place
    (``dres.addmm_(g, W)``, beta = 1 in the library epilogue): one launch and two [T, H] passes
    fewer per layer and direction. The consumer arms the tap in its forward (it always runs
    before the LayerNorm), and its backward always runs after the LayerNorm's (its output is
    upstream of the LayerNorm input); an unarmed tap leaves autograd's path untouched."""

    __slots__ = ("armed", "g")

    def __init__(self):
        self.armed = False
        self.g = None


def _dgrad_into(g2: torch.Tensor, w: torch.Tensor, tap: Optional[ResidualTap]) -> torch.Tensor:
    if tap is not None and tap.g is not None:
        acc, tap.g = tap.g.view(-1, w.shape[1]), None
        if use_native(g2) and w.is_contiguous() and _native_accum_ok(
                g2.shape[0], w.shape[1], w.shape[0], True, g2, w, acc):
            native().linear_dgrad_acc(g2, w, acc)   # acc += g2 W in the GEMM epilogue
            return acc
        return acc.addmm_(g2, w)
    return _dgrad_gemm(g2, w)


def _weight_grads(ctx, g2, x2, w, bias, need_w: bool, want_b: bool):
    """(dW, db) for y = x W^T + b: K9 split-M MFMA kernel (bias gradient fused in), optionally on
    the side stream (overlap) when AccumulateGrad will steal the result."""
    dw = db = None
    # The side-stream dW is only safe when AccumulateGrad STEALS it (no .grad yet): if a
    # gradient is already there, autograd adds into it on its own stream, reading dW before
    # the side-stream kernel finished -> compute it inline instead.
    steal = w.grad is None and (bias is None or bias.grad is None)
    if (need_w and _WG["enabled"] and not ctx.shared and steal and use_native(g2)
            and wgrad_supported(g2, x2)):
        dw, db = _wgrad_async(g2, x2, want_b)
    elif need_w:
        if want_b and use_native(g2) and wgrad_supported(g2, x2):
            dw, db = native().wgrad_bias(g2, x2)  # bias gradient fused into the K9 kernel
        else:
            dw = wgrad(g2, x2)
    if want_b and db is None:
        db = g2.sum(0)
    return dw, db


class _Linear(torch.autograd.Function):
    """y = x W^T (+ b). Forward / input-gradient GEMMs: linear.hip (MFMA, bias fused into the
    epilogue) where the shape allows, else the library; weight gradient: the split-M K9 kernel
    (gemm.hip), optionally on a side stream (overlap)."""

    @staticmethod
    def forward(ctx, x, w, b, tap=None):
        ctx.save_for_backward(x, w)
        ctx.tap = tap
        ctx.has_bias = b is not None
        # a parameter used several times per step gets its gradients summed by autograd on
        # autograd's stream, which a side-stream dW would race with
        ctx.shared = getattr(w, "_bcfl_shared", False) or getattr(b, "_bcfl_shared", False)
        ctx.bias = b
        return _fwd_gemm(x, w, b)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        N, K = w.shape
        g2 = g.reshape(-1, N)
        x2 = x.reshape(-1, K)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _dgrad_into(g2, w, ctx.tap).view(x.shape)
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        dw, db = _weight_grads(ctx, g2, x2, w, ctx.bias, ctx.needs_input_grad[1], want_b)
        return dx, dw, db, None


class _LinearAct(torch.autograd.Function):
    """(h, pre) with pre = x W^T + b and h = act(pre), in ONE GEMM (EPI_BIAS_ACT epilogue).
    ``pre`` carries the gradient: the NEXT layer (:class:`_LinearAfterAct`) returns dL/dpre
    directly (its dgrad epilogue applies act'), so this backward is dgrad + wgrad only — the
    bias+activation forward and backward passes over [T, I] disappear (K6)."""

    @staticmethod
    def forward(ctx, x, w, b, act_id, tap=None):
        x2 = x.reshape(-1, x.shape[-1])
        h, pre = native().linear_fwd(x2, w, b, int(act_id))
        ctx.save_for_backward(x, w)
        ctx.tap = tap
        ctx.has_bias = b is not None
        ctx.shared = getattr(w, "_bcfl_shared", False) or getattr(b, "_bcfl_shared", False)
        ctx.bias = b
        ctx.mark_non_differentiable(h)
        # h never receives a gradient: without this autograd materialises a zero [T, N] tensor
        # for it on every backward (a full fill pass over the FFN activation)
        ctx.set_materialize_grads(False)
        shp = (*x.shape[:-1], w.shape[0])
        return h.view(shp), pre.view(shp)

    @staticmethod
    def backward(ctx, _dh, dpre):
        if dpre is None:
            return None, None, None, None, None
        x, w = ctx.saved_tensors
        N, K = w.shape
        g2 = dpre.reshape(-1, N)
        x2 = x.reshape(-1, K)
        dx = _dgrad_into(g2, w, ctx.tap).view(x.shape) if ctx.needs_input_grad[0] else None
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        dw, db = _weight_grads(ctx, g2, x2, w, ctx.bias, ctx.needs_input_grad[1], want_b)
        return dx, dw, db, None, None


class _LinearAfterAct(torch.autograd.Function):
    """y = h W^T where h = act(pre) came from :class:`_LinearAct`; backward returns the gradient
    w.r.t. ``pre``: dgrad GEMM with the EPI_DACT epilogue (dh * act'(pre) in the same kernel)."""

    @staticmethod
    def forward(ctx, h, pre, w, act_id):
        ctx.save_for_backward(h, pre, w)
        ctx.act_id = int(act_id)
        ctx.shared = getattr(w, "_bcfl_shared", False)
        ctx.bias = None
        return _fwd_gemm(h, w, None)

    @staticmethod
    def backward(ctx, g):
        h, pre, w = ctx.saved_tensors
        N, K = w.shape
        g2 = g.reshape(-1, N)
        h2 = h.reshape(-1, K)
        dpre = None
        if ctx.needs_input_grad[1]:
            dpre = native().linear_dgrad(g2, w, pre.reshape(-1, K), ctx.act_id).view(pre.shape)
        dw, _ = _weight_grads(ctx, g2, h2, w, None, ctx.needs_input_grad[2], False)
        return None, dpre, dw, None


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


def _use_linear_fn(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (use_native(x) and (w.requires_grad or x.requires_grad) and torch.is_grad_enabled()
            and x.dtype == torch.bfloat16
            and w.shape[0] % 128 == 0 and w.shape[1] % 128 == 0 and x.numel() // w.shape[1] >= WGRAD_MIN_ROWS)


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None,
           tap: Optional[ResidualTap] = None) -> torch.Tensor:
    """Dense layer. GPU + bf16 + a weight that trains: :class:`_Linear` (linear.hip fwd/dgrad
    GEMMs, K9 wgrad); frozen / inference: the fused-epilogue forward GEMM alone; otherwise the
    plain library GEMM. ``tap``: see :class:`ResidualTap`."""
    if _use_linear_fn(x, w):
        if tap is not None:
            tap.armed = True
        return _Linear.apply(x, w, b, tap)
    if use_native(x) and not (torch.is_grad_enabled() and (w.requires_grad or x.requires_grad)):
        return _fwd_gemm(x, w, b)
    return torch.nn.functional.linear(x, w, b)


def linear_act(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], act: str = "gelu",
               tap: Optional[ResidualTap] = None):
    """(h, pre): h = act(x W^T + b). On the GPU fast path both come out of ONE GEMM and ``pre``
    must be handed to :func:`linear_after_act` (which routes the gradient); elsewhere ``pre`` is
    None and h is an ordinary autograd tensor."""
    aid = _ACT_ID[act]
    x2 = x.reshape(-1, x.shape[-1])
    if aid in (0, 1, 2) and (_use_linear_fn(x, w) or (use_native(x) and not torch.is_grad_enabled())) and \
            gemm_supported(x2, w, op="gemm_act"):
        if not torch.is_grad_enabled():
            h, _ = native().linear_fwd(x2, w, b, aid)
            return h.view(*x.shape[:-1], w.shape[0]), None
        if tap is not None:
            tap.armed = True
        return _LinearAct.apply(x, w, b, aid, tap)
    return bias_act(linear(x, w, tap=tap), b, act), None


def linear_after_act(h: torch.Tensor, pre: Optional[torch.Tensor], w: torch.Tensor,
                     act: str = "gelu") -> torch.Tensor:
    """y = h W^T for h from :func:`linear_act` (gradient routed to ``pre`` when given)."""
    if pre is not None and torch.is_grad_enabled() and pre.requires_grad:
        h2 = h.reshape(-1, h.shape[-1])
        if gemm_supported(h2, w, op="gemm_act") and gemm_supported(h2, w, nn_=True, op="gemm_act"):
            return _LinearAfterAct.apply(h, pre, w, _ACT_ID[act])
    return linear(h, w)


# ----------------------------------------------------------------------------------------
# K2: bias + dropout + residual + LayerNorm
# ----------------------------------------------------------------------------------------
class _BDALN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, bias, residual, gamma, beta, eps, p8, ka, kb, tap=None):
        C = native()
        out, z, mean, rstd = C.bdaln_fwd(y, bias, residual, gamma, beta, float(eps), int(p8),
                                         int(ka), int(kb))
        ctx.save_for_backward(z, mean, rstd, gamma)
        ctx.cfg = (p8, ka, kb, bias is not None, residual is not None, beta is not None)
        ctx.tap = tap
        return out

    @staticmethod
    def backward(ctx, dout):
        z, mean, rstd, gamma = ctx.saved_tensors
        p8, ka, kb, has_b, has_r, has_beta = ctx.cfg
        dy, dbias, dres, dgamma, dbeta = native().bdaln_bwd(dout.contiguous(), z, mean, rstd,
                                                            gamma, int(p8), int(ka), int(kb),
                                                            bool(has_b))
        if has_r and ctx.tap is not None:
            ctx.tap.g, dres = dres, None   # the consumer GEMM accumulates into it
        elif has_r and not p8 and _WG["enabled"]:
            # without dropout the kernel returns ONE buffer as dy and dres; autograd may sum the
            # residual's other gradient into it in place while the out-projection's side-stream
            # weight gradient is still reading dy (caught by scripts/overlap_diag.py: layer-0
            # attn_out / out weight gradients off by up to 17 %)
            dres = dres.clone()
        return (dy, dbias if has_b else None, dres if has_r else None, dgamma,
                dbeta if has_beta else None, None, None, None, None, None)


def bias_dropout_add_layernorm(y, bias, residual, gamma, beta, eps: float, p: float = 0.0,
                               training: bool = False, tap: Optional[ResidualTap] = None):
    """LayerNorm(dropout(y + bias) + residual). ``tap`` (armed by the GEMM that also reads
    ``residual``) routes the residual gradient into that GEMM's dgrad (:class:`ResidualTap`);
    only used with dropout on, where the kernel's residual gradient is its own buffer (p = 0
    aliases it with dy, which the out-projection's side-stream wgrad may still be reading)."""
    p8, ka, kb = _keys(p, training)
    if use_native(y, "bdaln"):
        use_tap = tap if (tap is not None and tap.armed and p8 and residual is not None
                          and residual.requires_grad) else None
        return _BDALN.apply(y.contiguous(), bias, residual, gamma, beta, eps, p8, ka, kb, use_tap)
    return ref.bias_dropout_add_layernorm(y, bias, residual, gamma, beta, eps, p8, ka, kb)


def layernorm(x, gamma, beta, eps: float):
    return bias_dropout_add_layernorm(x, None, None, gamma, beta, eps, 0.0, False)


# ----------------------------------------------------------------------------------------
# K6: bias + activation
# ----------------------------------------------------------------------------------------
_ACT_ID = {"gelu": 0, "gelu_new": 1, "gelu_tanh": 1, "relu": 2, "tanh": 3, "silu": 4}


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, bias, act_id):
        out = native().bias_act_fwd(y, bias, int(act_id))
        ctx.save_for_backward(y, bias)
        ctx.act_id = act_id
        ctx.has_b = bias is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        y, bias = ctx.saved_tensors
        dy, dbias = native().bias_act_bwd(dout.contiguous(), y, bias, int(ctx.act_id))
        return dy, (dbias if ctx.has_b else None), None


def bias_act(y, bias, act: str = "gelu"):
    if use_native(y, "bias_act"):
        return _BiasAct.apply(y.contiguous(), bias, _ACT_ID[act])
    return ref.bias_act(y, bias, act)


# ----------------------------------------------------------------------------------------
# K4: varlen flash attention on a packed qkv projection
# ----------------------------------------------------------------------------------------
class _VarlenAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cu, max_s, nh, nkv, d, scale, causal, p8, ka, kb, sched):
        C = native()
        out, lse, mask = C.attn_fwd(qkv, cu, int(max_s), int(nh), int(nkv), int(d), float(scale),
                                    bool(causal), int(p8), int(ka), int(kb), sched)
        ctx.save_for_backward(qkv, cu, out, lse, mask)
        ctx.cfg = (max_s, nh, nkv, d, scale, causal, p8, ka, kb)
        ctx.sched = sched
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, cu, out, lse, mask = ctx.saved_tensors
        max_s, nh, nkv, d, scale, causal, p8, ka, kb = ctx.cfg
        dqkv = native().attn_bwd(dout.contiguous(), qkv, out, lse, cu, int(max_s), int(nh),
                                 int(nkv), int(d), float(scale), bool(causal), int(p8), int(ka),
                                 int(kb), mask, ctx.sched)
        return dqkv, None, None, None, None, None, None, None, None, None, None, None


def varlen_attention(qkv: torch.Tensor, cu_seqlens: torch.Tensor, cu_host: Sequence[int],
                     max_seqlen: int, num_heads: int, num_kv_heads: int, head_dim: int,
                     dropout_p: float = 0.0, training: bool = False, causal: bool = False,
                     scale: Optional[float] = None,
                     sched: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qkv: [T, (nh + 2 nkv) * d] (q | k | v column blocks). Returns [T, nh * d].
    ``sched``: the batch's work order (:func:`bcfl.data.batching.attn_schedule`, on the device);
    None runs the blocks in batch order."""
    scale = 1.0 / math.sqrt(head_dim) if scale is None else scale
    p8, ka, kb = _keys(dropout_p, training)
    if use_native(qkv, "attn"):
        if sched is not None and (not sched.is_cuda or sched.device != qkv.device):
            sched = None
        return _VarlenAttn.apply(qkv.contiguous(), cu_seqlens, max_seqlen, num_heads,
                                 num_kv_heads, head_dim, scale, causal, p8, ka, kb, sched)
    return ref.varlen_attention(qkv, num_heads, num_kv_heads, head_dim, cu_host, scale, causal,
                                p8, ka, kb)


class _SubsetAttn(torch.autograd.Function):
    """Pooled-row attention on the GPU (subset_attention.hip, forward + backward)."""

    @staticmethod
    def forward(ctx, qkv, rows, cu, max_s, nh, nkv, d, scale, causal, p8, ka, kb):
        out, lse = native().subset_attn_fwd(qkv, cu, rows, int(max_s), int(nh), int(nkv), int(d),
                                            float(scale), bool(causal), int(p8), int(ka), int(kb))
        ctx.save_for_backward(qkv, rows, cu, out, lse)
        ctx.cfg = (max_s, nh, nkv, d, scale, causal, p8, ka, kb)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, rows, cu, out, lse = ctx.saved_tensors
        max_s, nh, nkv, d, scale, causal, p8, ka, kb = ctx.cfg
        dqkv = native().subset_attn_bwd(dout.contiguous(), qkv, out, lse, cu, rows, int(max_s),
                                        int(nh), int(nkv), int(d), float(scale), bool(causal),
                                        int(p8), int(ka), int(kb))
        return (dqkv,) + (None,) * 11


SUBSET_ATTN_MAX_KEYS = 6144  # subset_attention.hip LDS rows


def query_subset_attention(qkv: torch.Tensor, rows: torch.Tensor, cu_seqlens: torch.Tensor,
                           max_seqlen: int, num_heads: int, num_kv_heads: int, head_dim: int,
                           dropout_p: float = 0.0, training: bool = False, causal: bool = False,
                           scale: Optional[float] = None) -> torch.Tensor:
    """Attention of ONE query row per sequence (``rows[b]``, an absolute packed-token index inside
    sequence b) against all keys of sequence b. Returns [B, nh * d].

    Used for the LAST encoder layer of a sequence classifier, whose only consumed output is the
    pooled row (BERT/ALBERT/DistilBERT: the [CLS] row; Llama: the last token): the layer's other
    rows feed nothing, so the attention, output projection, FFN and LayerNorms run on B rows
    instead of T. Same math as :func:`varlen_attention` restricted to those queries, INCLUDING
    the dropout keep-mask (same element index (t * nh + h) * 8192 + key, same keys drawn), so the
    logits and every parameter gradient equal the full-layer computation. B x S_max scores: tiny,
    plain torch ops (autograd) on both devices."""
    scale = 1.0 / math.sqrt(head_dim) if scale is None else scale
    p8, ka, kb = _keys(dropout_p, training)
    B = int(rows.shape[0])
    if (use_native(qkv, "subset_attn") and qkv.dtype == torch.bfloat16 and head_dim in (32, 64, 128)
            and int(max_seqlen) <= SUBSET_ATTN_MAX_KEYS):
        return _SubsetAttn.apply(qkv.contiguous(), rows.to(torch.int32).contiguous(),
                                 cu_seqlens.to(torch.int32).contiguous(), int(max_seqlen),
                                 num_heads, num_kv_heads, head_dim, scale, causal, p8, ka, kb)
    dev = qkv.device
    nh, nkv, d = num_heads, num_kv_heads, head_dim
    cu = cu_seqlens[:B + 1].long()
    starts, lens = cu[:B], cu[1:B + 1] - cu[:B]
    rows = rows.long()
    S = max(int(max_seqlen), 1)
    j = torch.arange(S, device=dev)
    valid = j[None, :] < lens[:, None]                               # [B, S]
    if causal:
        valid = valid & (j[None, :] <= (rows - starts)[:, None])
    tok = torch.where(valid, starts[:, None] + j[None, :], starts[:, None])
    cdt = torch.float32
    q = qkv.index_select(0, rows)[:, : nh * d].reshape(B, nkv, nh // nkv, d).to(cdt)
    kv = qkv.index_select(0, tok.reshape(-1)).reshape(B, S, -1)[:, :, nh * d:]
    k = kv[:, :, : nkv * d].reshape(B, S, nkv, d).to(cdt)
    v = kv[:, :, nkv * d:].reshape(B, S, nkv, d).to(cdt)
    sc = torch.einsum("bgrd,bsgd->bgrs", q, k) * scale               # [B, nkv, rep, S]
    sc = sc.masked_fill(~valid[:, None, None, :], float("-inf"))
    pr = torch.softmax(sc, dim=-1)
    if p8 > 0:
        hh = torch.arange(nh, device=dev).reshape(1, nkv, nh // nkv, 1)
        idx = (rows.reshape(B, 1, 1, 1) * nh + hh) * ref.ATTN_DROP_STRIDE + j.reshape(1, 1, 1, S)
        keep = _rng.keep_mask_from_index(idx, p8, ka, kb)
        pr = pr * keep.to(pr.dtype) * _rng.keep_scale(p8)
    o = torch.einsum("bgrs,bsgd->bgrd", pr, v)
    return o.reshape(B, nh * d).to(qkv.dtype)


# ----------------------------------------------------------------------------------------
# K1 (+K2): embeddings gather-sum + LayerNorm + dropout
# ----------------------------------------------------------------------------------------
class _EmbLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, pos_ids, type_ids, word_w, pos_w, type_w, gamma, beta, eps, p8, ka, kb,
                ord_ids=None, ord_pos=None):
        C = native()
        out, z, mean, rstd = C.emb_ln_fwd(ids, pos_ids, type_ids, word_w, pos_w, type_w, gamma,
                                          beta, float(eps), int(p8), int(ka), int(kb))
        ctx.save_for_backward(ids, pos_ids, type_ids, z, mean, rstd, gamma, word_w, pos_w, type_w)
        ctx.cfg = (p8, ka, kb)
        ctx.order = (ord_ids, ord_pos)
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, pos_ids, type_ids, z, mean, rstd, gamma, word_w, pos_w, type_w = ctx.saved_tensors
        p8, ka, kb = ctx.cfg
        C = native()
        dword, dpos, dtype_, dgamma, dbeta = C.emb_ln_bwd(
            dout.contiguous(), ids, pos_ids, type_ids, z, mean, rstd, gamma, int(word_w.shape[0]),
            int(pos_w.shape[0]) if pos_w is not None else 0,
            int(type_w.shape[0]) if type_w is not None else 0, int(p8), int(ka), int(kb),
            *ctx.order)
        return (None, None, None, dword.to(word_w.dtype),
                dpos.to(pos_w.dtype) if pos_w is not None else None,
                dtype_.to(type_w.dtype) if type_w is not None else None,
                dgamma, dbeta, None, None, None, None, None, None)


def embedding_layernorm(ids, pos_ids, type_ids, word_w, pos_w, type_w, gamma, beta, eps: float,
                        p: float = 0.0, training: bool = False, order=None):
    """Embedding gather-sum + LayerNorm (+ dropout). ``order``: the batch's host-precomputed
    (ids, positions) stable sort orders, int32 [2, T] each (``PackedBatch.sort_ids`` /
    ``sort_pos``) — the table gradients then need no device sort."""
    p8, ka, kb = _keys(p, training)
    if use_native(word_w, "emb_ln"):
        oi, op = order if order is not None else (None, None)
        return _EmbLN.apply(ids, pos_ids, type_ids, word_w, pos_w, type_w, gamma, beta, eps, p8,
                            ka, kb, oi, op)
    return ref.embedding_layernorm(ids, pos_ids, type_ids, word_w, pos_w, type_w, gamma, beta,
                                   eps, p8, ka, kb)


# ----------------------------------------------------------------------------------------
# Llama path: RMSNorm, RoPE, SwiGLU
# ----------------------------------------------------------------------------------------
class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        out, rstd = native().rmsnorm_fwd(x, w, float(eps))
        ctx.save_for_backward(x, w, rstd)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, rstd = ctx.saved_tensors
        dx, dw = native().rmsnorm_bwd(dout.contiguous(), x, w, rstd, bool(w.requires_grad))
        return dx, (dw if w.requires_grad else None), None


def rmsnorm(x, w, eps: float):
    if use_native(x, "rmsnorm"):
        return _RMSNorm.apply(x.contiguous(), w, eps)
    return ref.rmsnorm(x, w, eps)


class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, pos_ids, cos, sin, nrot_heads, d):
        out = native().rope_fwd(qkv, pos_ids, cos, sin, int(nrot_heads), int(d), False)
        ctx.save_for_backward(pos_ids, cos, sin)
        ctx.cfg = (nrot_heads, d)
        return out

    @staticmethod
    def backward(ctx, dout):
        pos_ids, cos, sin = ctx.saved_tensors
        nrot, d = ctx.cfg
        dq = native().rope_fwd(dout.contiguous(), pos_ids, cos, sin, int(nrot), int(d), True)
        return dq, None, None, None, None, None


def rope(qkv: torch.Tensor, pos_ids, cos, sin, num_heads: int, num_kv_heads: int, head_dim: int):
    """Rotate the q and k column blocks of a packed [T, (nh+2nkv)*d] projection (v untouched)."""
    nrot = num_heads + num_kv_heads
    if use_native(qkv, "rope"):
        return _Rope.apply(qkv.contiguous(), pos_ids, cos, sin, nrot, head_dim)
    T = qkv.shape[0]
    qk = qkv[:, : nrot * head_dim].reshape(T, nrot, head_dim)
    qk = ref.rope(qk, pos_ids, cos, sin).reshape(T, nrot * head_dim)
    return torch.cat([qk, qkv[:, nrot * head_dim:]], dim=1)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        ctx.save_for_backward(gu)
        return native().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dout):
        (gu,) = ctx.saved_tensors
        return native().swiglu_bwd(dout.contiguous(), gu)


def swiglu(gate_up: torch.Tensor) -> torch.Tensor:
    if use_native(gate_up, "swiglu"):
        return _SwiGLU.apply(gate_up.contiguous())
    return ref.swiglu(gate_up)


class _XEnt(torch.autograd.Function):
    """K9: mean softmax cross-entropy, loss and gradient from ONE kernel (xent.hip)."""

    @staticmethod
    def forward(ctx, logits, labels):
        loss, grad = native().xent_fwd(logits, labels)
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g.to(grad.dtype), None


def cross_entropy(logits, labels):
    if use_native(logits, "xent") and logits.dim() == 2 and logits.dtype in (torch.bfloat16,
                                                                            torch.float32):
        return _XEnt.apply(logits.contiguous(), labels.to(torch.int32).contiguous())
    return torch.nn.functional.cross_entropy(logits.float(), labels.long())


@torch.no_grad()
def xent_stats_(logits: torch.Tensor, labels: torch.Tensor, acc4: torch.Tensor) -> None:
    """acc4 (fp64 [4]) += [correct, count, sum CE, sum CE / count] of one evaluation batch."""
    if use_native(logits, "xent") and logits.dtype in (torch.bfloat16, torch.float32):
        native().xent_stats(logits.contiguous(), labels.to(torch.int32).contiguous(), acc4)
        return
    lg, lab = logits.float(), labels.long()
    ce = torch.nn.functional.cross_entropy(lg, lab, reduction="sum")
    acc4[0] += (lg.argmax(-1) == lab).sum()
    acc4[1] += lab.numel()
    acc4[2] += ce
    acc4[3] += ce / lab.numel()


def dropout(x: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    """Dropout on small head tensors ([B, H] pooler output) with the counter-based hash RNG, so
    results are reproducible across processes (torch's global RNG is per process)."""
    p8, ka, kb = _keys(p, training)
    if p8 == 0:
        return x
    if use_native(x, "dropout") and x.dtype in (torch.bfloat16, torch.float32):
        # one hash kernel -> multiplier m = keep / (1 - p); autograd: one multiply each way
        return x * native().drop_mask(x, x.numel(), int(p8), int(ka), int(kb)).view_as(x)
    keep = _rng.keep_mask(x.numel(), p8, ka, kb, device=x.device).view_as(x)
    return x * keep.to(x.dtype) * _rng.keep_scale(p8)

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
        dout = dout.contiguous()
        probe = _PROBE.get("bdaln")
        if probe is not None:   # scripts/kernel_determinism.py DET_PROBE: inputs at kernel time
            probe.append({"in": [t.clone() for t in (dout, z, mean, rstd, gamma)],
                          "keys": (int(p8), int(ka), int(kb)), "has_b": bool(has_b)})
        dy, dbias, dres, dgamma, dbeta = native().bdaln_bwd(dout, z, mean, rstd,
                                                            gamma, int(p8), int(ka), int(kb),
                                                            bool(has_b))
        if probe is not None:
            probe[-1]["out"] = [t.clone() for t in (dy, dres)]
            probe[-1]["in_after"] = [t.clone() for t in (dout, z, mean, rstd, gamma)]
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


_RESIDUAL_TAP = os.environ.get("BCFL_RESIDUAL_TAP", "1") == "1"   # 0: autograd sums (A/B runs)
_PROBE: dict = {}   # debugging hooks (scripts/kernel_determinism.py): op name -> record list


def bias_dropout_add_layernorm(y, bias, residual, gamma, beta, eps: float, p: float = 0.0,
                               training: bool = False, tap: Optional[ResidualTap] = None):
    """LayerNorm(dropout(y + bias) + residual). ``tap`` (armed by the GEMM that also reads
    ``residual``) routes the residual gradient into that GEMM's dgrad (:class:`ResidualTap`);
    only used with dropout on, where the kernel's residual gradient is its own buffer (p = 0
    aliases it with dy, which the out-projection's side-stream wgrad may still be reading)."""
    p8, ka, kb = _keys(p, training)
    if use_native(y, "bdaln"):
        use_tap = tap if (tap is not None and tap.armed and p8 and residual is not None
                          and residual.requires_grad and _RESIDUAL_TAP) else None
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


# LoRA projections (bcfl/ops/lora.py) stay reachable as bcfl.ops.functional.*
from .lora import _lora_mlp_fused_ok, lora_linear, lora_swiglu_mlp  # noqa: E402,F401

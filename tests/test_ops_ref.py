"""CPU checks of the op definitions (the torch references the HIP kernels are tested against)."""
import hashlib
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from bcfl import ops
from bcfl.ops import ref, rng
from bcfl.ops.flat import merkle_from_leaves


def test_hash_matches_python_int_impl():
    ka, kb = rng.derive_keys(123, 7)
    idx = torch.arange(0, 5000, 37, dtype=torch.int64)
    got = rng.hash32(idx, ka, kb).tolist()

    def h(x):
        x = (x ^ ka) & 0xFFFFFFFF
        x ^= x >> 16
        x = (x * 0x7FEB352D) & 0xFFFFFFFF
        x ^= kb
        x ^= x >> 15
        x = (x * 0x846CA68B) & 0xFFFFFFFF
        x ^= x >> 16
        return x
    assert got == [h(int(i)) for i in idx]


def test_dropout_rate_and_determinism():
    p8 = rng.quantize_p(0.1)
    ka, kb = rng.derive_keys(5, 0)
    m1 = rng.keep_mask(1 << 18, p8, ka, kb)
    m2 = rng.keep_mask(1 << 18, p8, ka, kb)
    assert torch.equal(m1, m2)
    assert abs(1 - m1.float().mean().item() - p8 / 256) < 4e-3
    ka2, kb2 = rng.derive_keys(5, 1)
    m3 = rng.keep_mask(1 << 18, p8, ka2, kb2)
    agree = (m1 == m3).float().mean().item()
    assert abs(agree - (1 - 2 * 0.0977 * 0.9023)) < 0.01  # independent masks


def test_varlen_attention_matches_padded_sdpa():
    torch.manual_seed(0)
    nh, d = 3, 16
    lens = [5, 17, 1, 9]
    cu = np.concatenate([[0], np.cumsum(lens)])
    T = int(cu[-1])
    qkv = torch.randn(T, 3 * nh * d)
    out = ref.varlen_attention(qkv, nh, nh, d, cu, 1 / math.sqrt(d))
    for b, L in enumerate(lens):
        s, e = cu[b], cu[b + 1]
        q = qkv[s:e, :nh * d].view(L, nh, d).transpose(0, 1)
        k = qkv[s:e, nh * d:2 * nh * d].view(L, nh, d).transpose(0, 1)
        v = qkv[s:e, 2 * nh * d:].view(L, nh, d).transpose(0, 1)
        o = F.scaled_dot_product_attention(q, k, v).transpose(0, 1).reshape(L, nh * d)
        torch.testing.assert_close(out[s:e], o, atol=1e-5, rtol=1e-5)


def test_varlen_attention_gqa_causal():
    torch.manual_seed(1)
    nh, nkv, d = 4, 2, 8
    lens = [7, 3]
    cu = np.concatenate([[0], np.cumsum(lens)])
    qkv = torch.randn(int(cu[-1]), (nh + 2 * nkv) * d)
    out = ref.varlen_attention(qkv, nh, nkv, d, cu, 1 / math.sqrt(d), causal=True)
    s, e = 0, 7
    q = qkv[s:e, :nh * d].view(7, nh, d).transpose(0, 1)
    k = qkv[s:e, nh * d:(nh + nkv) * d].view(7, nkv, d).transpose(0, 1).repeat_interleave(2, 0)
    v = qkv[s:e, (nh + nkv) * d:].view(7, nkv, d).transpose(0, 1).repeat_interleave(2, 0)
    o = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(0, 1).reshape(7, nh * d)
    torch.testing.assert_close(out[s:e], o, atol=1e-5, rtol=1e-5)


def test_bias_dropout_add_ln_ref():
    torch.manual_seed(0)
    y, b, r = torch.randn(10, 32), torch.randn(32), torch.randn(10, 32)
    g, be = torch.randn(32), torch.randn(32)
    out = ref.bias_dropout_add_layernorm(y, b, r, g, be, 1e-12)
    torch.testing.assert_close(out, F.layer_norm(y + b + r, (32,), g, be, 1e-12))
    p8 = rng.quantize_p(0.5)
    ka, kb = rng.derive_keys(1, 1)
    out2 = ref.bias_dropout_add_layernorm(y, b, r, g, be, 1e-12, p8, ka, kb)
    keep = rng.keep_mask(320, p8, ka, kb).view(10, 32).float()
    torch.testing.assert_close(out2, F.layer_norm((y + b) * keep * 2 + r, (32,), g, be, 1e-12))


def test_adamw_modes():
    torch.manual_seed(0)
    p0 = torch.randn(1000)
    grads = [torch.randn(1000) for _ in range(5)]
    # torch mode == torch.optim.AdamW
    p = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([p], lr=1e-2, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01)
    master, m, v = p0.clone(), torch.zeros(1000), torch.zeros(1000)
    for t, g in enumerate(grads, 1):
        p.grad = g.clone()
        opt.step()
        ref.adamw_(master, g, m, v, t, 1e-2, 0.9, 0.999, 1e-6, 0.01, "torch")
    torch.testing.assert_close(master, p.detach(), atol=1e-6, rtol=1e-6)
    # hf mode: transformers 4.35 AdamW formula, eps outside the bias correction
    master, m, v = p0.clone(), torch.zeros(1000), torch.zeros(1000)
    pm, mm, vm = p0.double().clone(), torch.zeros(1000, dtype=torch.float64), torch.zeros(1000, dtype=torch.float64)
    for t, g in enumerate(grads, 1):
        ref.adamw_(master, g, m, v, t, 1e-2, 0.9, 0.999, 1e-6, 0.0, "hf")
        gd = g.double()
        mm = 0.9 * mm + 0.1 * gd
        vm = 0.999 * vm + 0.001 * gd * gd
        step = 1e-2 * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        pm = pm - step * mm / (vm.sqrt() + 1e-6)
    torch.testing.assert_close(master.double(), pm, atol=1e-6, rtol=1e-6)


def test_gossip_mix_and_accumulate():
    a, b, c = torch.randn(100), torch.randn(100), torch.randn(100).bfloat16()
    x = a.clone()
    ops.gossip_mix_(x, [b, c], 0.5, [0.25, 0.25])
    torch.testing.assert_close(x, 0.5 * a + 0.25 * b + 0.25 * c.float())
    acc = torch.zeros(100)
    ops.weighted_accumulate_(acc, a, 0.3)
    ops.weighted_accumulate_(acc, b, 0.7)
    torch.testing.assert_close(acc, 0.3 * a + 0.7 * b)


def test_block_sketch_inner_product():
    torch.manual_seed(0)
    n = 1 << 16
    x = torch.randn(n)
    y = 0.6 * x + 0.8 * torch.randn(n)
    sx, sy = ref.block_sketch(x, 4096), ref.block_sketch(y, 4096)
    cos_true = F.cosine_similarity(x, y, dim=0).item()
    cos_est = F.cosine_similarity(sx, sy, dim=0).item()
    assert abs(cos_true - cos_est) < 0.05
    assert ref.block_sketch(x, 4096).shape == (4096,)


def test_merkle_root_host():
    buf = torch.arange(100000, dtype=torch.float32)
    b = buf.numpy().tobytes()
    leaf = 1 << 12
    leaves = [hashlib.sha256(b"\x00" + b[i:i + leaf]).digest() for i in range(0, len(b), leaf)]
    assert ops.merkle_root_sha256(buf, leaf) == merkle_from_leaves(leaves)
    d = ops.leaf_digests_sha256(buf, leaf)
    assert d.shape == (len(leaves), 32) and bytes(d[3].numpy()) == leaves[3]
    from bcfl.trust.graph import native_available
    if native_available():
        from bcfl import _host
        assert _host.merkle_root_hex(buf.numpy(), leaf) == merkle_from_leaves(leaves).hex()


def test_flat_adamw_clipping_matches_torch_clip_grad_norm():
    """FlatAdamW(max_grad_norm) == torch.nn.utils.clip_grad_norm_ + the same AdamW step (CPU
    reference path; the GPU kernel is pinned in tests/test_gpu_kernels.py)."""
    import torch
    from bcfl.parallel.flat import FlatAdamW, FlatParams
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(37, 5)), torch.nn.Parameter(torch.randn(11))]
    flat = FlatParams(ps, "cpu", torch.float32)
    ref_ps = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FlatAdamW(flat, lr=1e-2, mode="torch", max_grad_norm=0.5)
    ropt = torch.optim.AdamW(ref_ps, lr=1e-2, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.0)
    for _ in range(3):
        gs = [torch.randn_like(p) * 3 for p in ps]
        for p, q, g in zip(ps, ref_ps, gs):
            p.grad, q.grad = g.clone(), g.clone()
        tn = torch.nn.utils.clip_grad_norm_(ref_ps, 0.5)
        opt.step()
        ropt.step()
        assert float(opt.last_grad_norm) == pytest.approx(float(tn), rel=1e-5)
        flat.zero_grad()
    for p, q in zip(ps, ref_ps):
        torch.testing.assert_close(p.detach(), q.detach(), atol=1e-6, rtol=1e-5)

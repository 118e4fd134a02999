"""GPU numerics: every HIP kernel vs the PyTorch fp32 reference of the same op (bcfl.ops.ref).

Run on the MI355X box: ``python -m pytest tests -m gpu``. These tests REQUIRE the native
extension (no eager fallback on the GPU path)."""
import hashlib
import math

import numpy as np
import pytest
import torch

from bcfl import ops
from bcfl.ops import _native, ref, rng

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert ops.native_available(), ops.load_error()
    assert "bcfl/_C" in ops.native().__file__.replace("\\", "/")


def _close(a, b, atol, rtol=2e-2):
    torch.testing.assert_close(a.float(), b.float(), atol=atol, rtol=rtol)


def _grads_close(ga, gb, tol=3e-2):
    # relative Frobenius error: robust for bf16 gradients of mixed scale
    for x, y in zip(ga, gb):
        if x is None and y is None:
            continue
        x, y = x.float(), y.float()
        err = (x - y).norm() / (y.norm() + 1e-6)
        assert err < tol, f"relative grad error {err:.4f}"


@pytest.mark.parametrize("H", [64, 128, 768, 1024])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("with_res", [True, False])
def test_bdaln_fwd_bwd(H, p, with_res):
    torch.manual_seed(0)
    T = 333
    y = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = (0.1 * torch.randn(H, device=DEV)).bfloat16().requires_grad_(True)
    r = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True) if with_res else None
    g = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16().requires_grad_(True)
    be = (0.1 * torch.randn(H, device=DEV)).bfloat16().requires_grad_(True)
    rng.manual_seed(7)
    out = ops.bias_dropout_add_layernorm(y, b, r, g, be, 1e-12, p, True)
    rng.manual_seed(7)
    p8, ka, kb = (rng.quantize_p(p), *rng.global_rng().next()) if p > 0 else (0, 0, 0)
    leaves = [t.detach().float().requires_grad_(True) for t in (y, b, g, be)]
    rf = r.detach().float().requires_grad_(True) if with_res else None
    ref_out = ref.bias_dropout_add_layernorm(leaves[0], leaves[1], rf, leaves[2], leaves[3], 1e-12, p8, ka, kb)
    _close(out, ref_out, 3e-2)
    go = torch.randn_like(out)
    out.backward(go)
    ref_out.backward(go.float())
    ours = [y.grad, b.grad, g.grad, be.grad] + ([r.grad] if with_res else [])
    theirs = [l.grad for l in leaves] + ([rf.grad] if with_res else [])
    _grads_close(ours, theirs)


@pytest.mark.parametrize("act", ["gelu", "gelu_new", "relu", "tanh", "silu"])
def test_bias_act(act):
    torch.manual_seed(0)
    y = torch.randn(257, 3072, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = (0.2 * torch.randn(3072, device=DEV)).bfloat16().requires_grad_(True)
    out = ops.bias_act(y, b, act)
    yf, bf = y.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    r = ref.bias_act(yf, bf, act)
    _close(out, r, 2e-2)
    go = torch.randn_like(out)
    out.backward(go)
    r.backward(go.float())
    _grads_close([y.grad, b.grad], [yf.grad, bf.grad])


def _attn_case(lens, nh, nkv, d, causal, p, sched=False, late_boost=0.0):
    from bcfl.data.batching import attn_schedule
    torch.manual_seed(1)
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    T = int(cu[-1])
    x = 0.5 * torch.randn(T, (nh + 2 * nkv) * d, device=DEV)
    if late_boost:  # keys past position 200 of every row score far above the first tile's max
        pos = torch.from_numpy(np.concatenate([np.arange(n) for n in lens])).to(DEV)
        x[pos > 200, nh * d:(nh + nkv) * d] *= late_boost
    qkv = x.bfloat16().requires_grad_(True)
    cu_d = torch.from_numpy(cu).to(DEV)
    sc = attn_schedule(cu).to(DEV) if sched else None
    rng.manual_seed(3)
    out = ops.varlen_attention(qkv, cu_d, cu, max(lens), nh, nkv, d, p, True, causal, sched=sc)
    rng.manual_seed(3)
    p8, ka, kb = (rng.quantize_p(p), *rng.global_rng().next()) if p > 0 else (0, 0, 0)
    qf = qkv.detach().float().requires_grad_(True)
    r = ref.varlen_attention(qf, nh, nkv, d, cu, 1 / math.sqrt(d), causal, p8, ka, kb)
    _close(out, r, 2e-2)
    go = torch.randn_like(out)
    out.backward(go)
    r.backward(go.float())
    _grads_close([qkv.grad], [qf.grad], 3e-2)
    return out.detach(), qkv.grad


@pytest.mark.parametrize("lens", [[1, 5, 64, 65, 127, 128, 129], [512, 300, 200], [33],
                                  [1100, 700, 90]])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_bert(lens, p):
    _attn_case(lens, 12, 12, 64, False, p)


@pytest.mark.parametrize("causal,p", [(False, 0.1), (True, 0.0)])
def test_attention_schedule_is_bitwise(causal, p):
    """The longest-first work order (attn_schedule) changes only WHEN a block runs: outputs and
    gradients are bit-identical to batch order."""
    lens = [90, 513, 7, 260, 1000, 129]
    a = _attn_case(lens, 12, 12, 64, causal, p)
    b = _attn_case(lens, 12, 12, 64, causal, p, sched=True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_late_max_rescale(p):
    """Scores that grow far past the first key tile's max exercise the forward's deferred
    rescale (RESCALE_LOG2)."""
    _attn_case([300, 450, 64], 12, 12, 64, False, p, late_boost=6.0)


def test_attention_dropout_d32_and_causal():
    _attn_case([1, 70, 200, 333], 4, 4, 32, False, 0.1)
    _attn_case([1, 70, 200, 333], 4, 4, 64, True, 0.1)


@pytest.mark.parametrize("lens", [[1, 70, 200], [256]])
def test_attention_gqa_causal_d128(lens):
    _attn_case(lens, 8, 2, 128, True, 0.0)


def test_attention_lse():
    torch.manual_seed(2)
    lens = [100, 37]
    cu = np.array([0, 100, 137], dtype=np.int32)
    qkv = torch.randn(137, 3 * 4 * 64, device=DEV).bfloat16()
    out, lse, _ = ops.native().attn_fwd(qkv, torch.from_numpy(cu).to(DEV), 100, 4, 4, 64, 0.125, False, 0, 0, 0)
    _, rl = ref.varlen_attention(qkv.float(), 4, 4, 64, cu, 0.125, return_lse=True)
    _close(lse, rl, 1e-2, 1e-3)


@pytest.mark.parametrize("p,skew", [(0.0, False), (0.1, False), (0.1, True)])
def test_embedding_layernorm(p, skew):
    torch.manual_seed(0)
    V, P, H, T = 1000, 128, 768, 3000 if skew else 300
    ids = torch.randint(0, V, (T,), device=DEV, dtype=torch.int32)
    if skew:  # Zipf-like: runs far longer than the 32-row segment chunk, plus many singletons
        ids[: T // 2] = 7
        ids[T // 2: T // 2 + 300] = 3
    pos = torch.randint(0, P, (T,), device=DEV, dtype=torch.int32)
    pos = torch.randint(0, P, (T,), device=DEV, dtype=torch.int32)
    ws = [(0.02 * torch.randn(*s, device=DEV)).bfloat16().requires_grad_(True) for s in ((V, H), (P, H), (2, H))]
    g = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16().requires_grad_(True)
    be = (0.1 * torch.randn(H, device=DEV)).bfloat16().requires_grad_(True)
    rng.manual_seed(11)
    out = ops.embedding_layernorm(ids, pos, None, *ws, g, be, 1e-12, p, True)
    rng.manual_seed(11)
    p8, ka, kb = (rng.quantize_p(p), *rng.global_rng().next()) if p > 0 else (0, 0, 0)
    leaves = [t.detach().float().requires_grad_(True) for t in (*ws, g, be)]
    r = ref.embedding_layernorm(ids, pos, None, *leaves[:3], leaves[3], leaves[4], 1e-12, p8, ka, kb)
    _close(out, r, 3e-2)
    go = torch.randn_like(out)
    out.backward(go)
    r.backward(go.float())
    _grads_close([w.grad for w in ws] + [g.grad, be.grad], [l.grad for l in leaves])
    if skew:  # the long runs themselves, and bitwise determinism of the segmented sums
        # row 7 sums 1500 token rows (|grad| ~ 1e3, bf16 ulp ~ 8): compare by relative norm
        _grads_close([ws[0].grad[7], ws[0].grad[3]], [leaves[0].grad[7], leaves[0].grad[3]], 1e-2)
        g1 = ws[0].grad.clone()
        for w in ws:
            w.grad = None
        rng.manual_seed(11)
        ops.embedding_layernorm(ids, pos, None, *ws, g, be, 1e-12, p, True).backward(go)
        assert torch.equal(ws[0].grad, g1)


def test_rmsnorm_rope_swiglu():
    torch.manual_seed(0)
    T, H = 129, 512
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16().requires_grad_(True)
    out = ops.rmsnorm(x, w, 1e-5)
    xf, wf = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    r = ref.rmsnorm(xf, wf, 1e-5)
    _close(out, r, 3e-2)
    go = torch.randn_like(out)
    out.backward(go)
    r.backward(go.float())
    _grads_close([x.grad, w.grad], [xf.grad, wf.grad])
    # RoPE on a packed [T, (nh + 2 nkv) d] projection
    nh, nkv, d = 4, 2, 64
    qkv = torch.randn(T, (nh + 2 * nkv) * d, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    pos = torch.arange(T, device=DEV, dtype=torch.int32) % 100
    cos, sin = ref.rope_cache(256, d, 10000.0, DEV)
    o = ops.rope(qkv, pos, cos, sin, nh, nkv, d)
    qf = qkv.detach().float().requires_grad_(True)
    nrot = nh + nkv
    rq = torch.cat([ref.rope(qf[:, :nrot * d].reshape(T, nrot, d), pos, cos, sin).reshape(T, -1),
                    qf[:, nrot * d:]], 1)
    _close(o, rq, 3e-2)
    go = torch.randn_like(o)
    o.backward(go)
    rq.backward(go.float())
    _grads_close([qkv.grad], [qf.grad])
    # SwiGLU
    gu = torch.randn(T, 2 * 256, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    s = ops.swiglu(gu)
    gf = gu.detach().float().requires_grad_(True)
    rs_ = ref.swiglu(gf)
    _close(s, rs_, 3e-2)
    go = torch.randn_like(s)
    s.backward(go)
    rs_.backward(go.float())
    _grads_close([gu.grad], [gf.grad])


@pytest.mark.parametrize("mode", ["hf", "torch"])
def test_fused_adamw(mode):
    torch.manual_seed(0)
    n = 1 << 20
    master = torch.randn(n, device=DEV)
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    p_out = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    rm, rmm, rvv = master.clone(), m.clone(), v.clone()
    for t in range(1, 4):
        g = torch.randn(n, device=DEV).bfloat16()
        ops.adamw_(master, g, m, v, t, 1e-3, 0.9, 0.999, 1e-6, 0.01, mode, p_out)
        ref.adamw_(rm, g.float(), rmm, rvv, t, 1e-3, 0.9, 0.999, 1e-6, 0.01, mode)
    _close(master, rm, 1e-5, 1e-5)
    _close(p_out, rm, 1e-2)


@pytest.mark.parametrize("mode,with_corr", [("hf", False), ("torch", False), ("hf", True)])
def test_multi_tensor_adamw(mode, with_corr):
    torch.manual_seed(0)
    sizes = [768, 2, 3072 * 768, 5, 30522 * 768, 64] + [777] * 45  # > one 40-tensor group
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += (n + 63) // 64 * 64
    master = torch.randn(o, device=DEV)
    m, v = torch.zeros(o, device=DEV), torch.zeros(o, device=DEV)
    p_out = torch.zeros(o, device=DEV, dtype=torch.bfloat16)
    rm, rmm, rvv = master.clone(), m.clone(), v.clone()
    # drift correction (fl/drift.py): p -= corr_lr * corr fused into the same pass
    corr = torch.randn(o, device=DEV) if with_corr else None
    for t in range(1, 3):
        grads = [torch.randn(n, device=DEV).bfloat16() for n in sizes]
        ops.adamw_multi_(master, grads, offs, m, v, t, 1e-3, 0.9, 0.999, 1e-6, 0.01, mode, p_out,
                         corr=corr, corr_lr=5e-4)
        for g, of in zip(grads, offs):
            n = g.numel()
            ref.adamw_(rm[of:of + n], g.float(), rmm[of:of + n], rvv[of:of + n], t, 1e-3, 0.9,
                       0.999, 1e-6, 0.01, mode)
            if corr is not None:
                rm[of:of + n] -= 5e-4 * corr[of:of + n]
    _close(master, rm, 1e-5, 1e-5)
    _close(m, rmm, 1e-6, 1e-5)
    mask = torch.zeros(o, dtype=torch.bool, device=DEV)
    for n, of in zip(sizes, offs):
        mask[of:of + n] = True
    _close(p_out[mask], rm[mask], 1e-2)
    assert (p_out[~mask] == 0).all()  # padding untouched


def test_flat_ops():
    torch.manual_seed(0)
    n = (1 << 18) + 64
    x = torch.randn(n, device=DEV)
    nb = [torch.randn(n, device=DEV), torch.randn(n, device=DEV).bfloat16()]
    y = x.clone()
    po = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    ops.gossip_mix_(y, nb, 0.5, [0.3, 0.2], po)
    _close(y, 0.5 * x + 0.3 * nb[0] + 0.2 * nb[1].float(), 1e-5, 1e-5)
    _close(po, y, 1e-2)
    z = x.clone()
    ops.axpby_(z, nb[1], 2.0, -1.0)
    _close(z, 2 * nb[1].float() - x, 1e-5, 1e-5)
    c = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    ops.cast_copy_(c, x)
    assert torch.equal(c, x.bfloat16())
    refb = torch.zeros(n, device=DEV)
    q = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    ops.native().delta_encode(x, refb, q)
    assert torch.equal(q, x.bfloat16()) and torch.equal(refb, x.bfloat16().float())
    sk = ops.block_sketch(x, 4096)
    _close(sk, ref.block_sketch(x.cpu(), 4096).to(DEV), 1e-3, 1e-4)


@pytest.mark.parametrize("wire", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("with_cv,with_d", [(True, True), (True, False), (False, False)])
def test_delta_round_end_matches_reference(wire, with_cv, with_d):
    """Fused round end of the round-complete gossip (elementwise.hip delta_round_end_kernel) vs
    the fp32 reference: own update u = y - x, cumulative sum, wire image, control variate
    (x - y) / L - s d, own-progress retraction and the bf16 parameter copy."""
    torch.manual_seed(1)
    n = (1 << 18) + 64
    y, x, cum = (torch.randn(n, device=DEV) for _ in range(3))
    d = torch.randn(n, device=DEV) if with_d else None
    cv = torch.zeros(n, device=DEV) if with_cv else None
    wire_t = torch.zeros(2 * n if with_cv else n, device=DEV, dtype=wire)
    po = torch.zeros(n, device=DEV, dtype=torch.bfloat16)
    ry, rx, rc = y.cpu(), x.cpu(), cum.cpu()
    rcv = torch.zeros(n) if with_cv else None
    rwire = torch.zeros(wire_t.numel())
    rpo = torch.zeros(n)
    ops.delta_round_end_(y, x, cum, wire_t, po, d, cv, 1.0 / 3.5e-4, 0.75)
    ref.delta_round_end_(ry, rx, rc, rwire, rpo, d.cpu() if with_d else None, rcv, 1.0 / 3.5e-4, 0.75)
    torch.cuda.synchronize()
    _close(y, ry.to(DEV), 1e-6, 1e-6)
    _close(cum, rc.to(DEV), 1e-6, 1e-6)
    # the wire's aux half carries c ~ 1e3 (x / L): fp32 agrees to an ulp or two (FMA contraction)
    atol, rtol = (1e-2, 1e-2) if wire == torch.bfloat16 else (1e-2, 1e-5)
    _close(wire_t, rwire.to(DEV, wire), atol, rtol)
    _close(po, ry.to(DEV), 2e-2)
    if with_cv:
        _close(cv, rcv.to(DEV), 1e-2, 1e-5)
    assert torch.equal(x.cpu(), rx)   # the round-start record is only read


@pytest.mark.parametrize("nbytes", [4 * 1000, 4096 * 37 + 1024, 1 << 22])
def test_sha256_merkle_matches_hashlib(nbytes):
    g = torch.Generator().manual_seed(0)
    host = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, generator=g)
    dev = host.to(DEV)
    leaf = 4096
    b = host.numpy().tobytes()
    leaves = [hashlib.sha256(b"\x00" + b[i:i + leaf]).digest() for i in range(0, len(b), leaf)]
    d = ops.leaf_digests_sha256(dev, leaf).cpu()
    assert [bytes(d[i].numpy()) for i in range(d.shape[0])] == leaves
    from bcfl.ops.flat import merkle_from_leaves
    assert ops.merkle_root_sha256(dev, leaf) == merkle_from_leaves(leaves)


def test_bert_model_gpu_matches_cpu_reference():
    from bcfl.data.batching import make_packed_batch
    from bcfl.data.registry import load_split
    from bcfl.models import build_model
    m_cpu = build_model("tiny-bert", 2, seed=0).eval()
    m_gpu = build_model("tiny-bert", 2, seed=0, device=DEV, dtype=torch.bfloat16).eval()
    ds = load_split("tiny", "train", 2048, 128)
    b = make_packed_batch(ds, np.arange(0, 200, 7))
    with torch.no_grad():
        lc = m_cpu(b)
        lg = m_gpu(b.to(DEV)).float().cpu()
    _close(lg, lc, 5e-2, 5e-2)


def test_federation_gpu_smoke(tmp_path):
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    D.set_runtime_for_tests(None)
    cfg = FLConfig(mode="serverless", model="bert-base-2l", dataset="imdb", num_clients=2,
                   num_rounds=2, train_samples=64, test_samples=32, global_test_samples=64,
                   out_dir=str(tmp_path), reference_prints=False, anomaly_filter="both")
    fed = Federation(cfg, verbose=False)
    h = fed.run()
    assert len(h) == 2 and all(np.isfinite(r["train_loss"]) for r in h)
    assert fed.ledger.verify() == -1
    D.set_runtime_for_tests(None)

@pytest.mark.parametrize("M,N,K", [(11264, 768, 768), (11264, 2304, 768), (5000, 768, 3072),
                                   (1088, 4096, 4096), (2048, 128, 256)])
def test_wgrad_split_m(M, N, K):
    """K9 weight gradient vs fp32 torch: split-M partials (S > 1), single split (S == 1), a
    reduction length that is not a multiple of the 64-row step, strided row views."""
    torch.manual_seed(0)
    g = torch.randn(M, N + 64, device=DEV).bfloat16()[:, 64:]  # strided rows
    x = torch.randn(M, K, device=DEV).bfloat16()
    assert ops.functional.wgrad_supported(g, x)
    out = ops.native().wgrad(g, x)
    refv = g.float().t() @ x.float()
    err = (out.float() - refv).norm() / refv.norm()
    assert err < 5e-3, err
    out2 = ops.native().wgrad(g, x)
    assert torch.equal(out, out2)  # deterministic split reduction
    ow, db = ops.native().wgrad_bias(g, x)  # fused bias gradient = column sums of g
    assert torch.equal(ow, out)
    rb = g.float().sum(0)
    assert ((db.float() - rb).norm() / rb.norm()) < 5e-3


def test_linear_autograd_uses_wgrad_kernel():
    torch.manual_seed(0)
    x = torch.randn(4096, 768, device=DEV).bfloat16().requires_grad_(True)
    w = (0.02 * torch.randn(2304, 768, device=DEV)).bfloat16().requires_grad_(True)
    b = torch.zeros(2304, device=DEV).bfloat16().requires_grad_(True)
    y = ops.linear(x, w, b)
    assert y.grad_fn is not None and "Linear" in type(y.grad_fn).__name__
    g = torch.randn_like(y)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), g)
    rx, rw, rb = torch.autograd.grad(torch.nn.functional.linear(x.float(), w.float(), b.float()),
                                     (x, w, b), g.float())
    _grads_close((gx, gw, gb), (rx, rw, rb), tol=1e-2)



@pytest.mark.parametrize("model", ["bert-base-2l", "albert-base-v2"])
def test_overlapped_wgrad_matches_inline(model):
    """Side-stream weight gradients (the 8-phase kernel on a paired stream, joined before the
    optimizer) give the inline path's parameter gradients; ALBERT's shared layer opts out.
    Bitwise in practice (scripts/overlap_diag.py); compared at 1e-3 relative so a stray fp32 ULP
    cannot fail it while a stream-ordering race cannot pass: the round-3 suite caught one (without
    dropout the LayerNorm backward's dy and residual gradient were one buffer, summed into in place
    while the out-projection's side-stream weight gradient still read it: 17 % error in layer 0)."""
    from bcfl.data.batching import make_packed_batch
    from bcfl.data.registry import load_split
    from bcfl.models import build_model, special_tokens
    cls_id, sep_id, vocab = special_tokens(model)
    ds = load_split("imdb", "train", vocab, 512, 1234, cls_id, sep_id)
    b = make_packed_batch(ds, np.arange(0, 25000, 1563)[:16]).to(DEV)
    grads = {}
    for ov in (False, True):
        ops.set_wgrad_overlap(ov)
        rng.manual_seed(7)  # identical dropout keys for both passes
        try:
            m = build_model(model, 2, device=DEV, dtype=torch.bfloat16, seed=0, dropout=0.0)
            m.train()
            loss = ops.cross_entropy(m(b), b.labels)
            loss.backward()
            ops.join_wgrad()
            grads[ov] = [p.grad.clone() for p in m.parameters() if p.grad is not None]
        finally:
            ops.set_wgrad_overlap(False)
    assert len(grads[False]) == len(grads[True])
    _grads_close(grads[True], grads[False], tol=1e-3)


# ---------------------------------------------------------------------------------------------
# linear.hip: dense-layer GEMMs with fused epilogues vs fp32 references
_LIN_SHAPES = [(11264, 768, 768), (1000, 2304, 768), (333, 3072, 768), (2048, 768, 3072),
               (1088, 4096, 4096), (64, 128, 64)]


@pytest.fixture(params=["0", "1"], ids=["tile128", "tile256"])
def lin_tile(request, monkeypatch):
    monkeypatch.setenv("BCFL_LINEAR_TILE", request.param)
    return int(request.param)


@pytest.mark.parametrize("M,N,K", _LIN_SHAPES)
@pytest.mark.parametrize("epi", ["store", "bias", "gelu", "gelu_new"])
def test_linear_fwd_epilogues(M, N, K, epi, lin_tile):
    torch.manual_seed(0)
    C = ops.native()
    xs = torch.randn(M, K + 64, device=DEV).bfloat16()
    x = xs[:, :K]  # strided rows (ld = K + 64)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).bfloat16()
    b = torch.randn(N, device=DEV).bfloat16() if epi != "store" else None
    act = {"store": -1, "bias": -1, "gelu": 0, "gelu_new": 1}[epi]
    out = C.linear_fwd(x, w, b, act)
    ref = x.float() @ w.float().t() + (b.float() if b is not None else 0)
    if act < 0:
        _close(out[0], ref, 2e-2, 2e-2)
    else:
        h, pre = out
        _close(pre, ref, 2e-2, 2e-2)
        fn = torch.nn.functional.gelu
        _close(h, fn(pre.float(), approximate="none" if act == 0 else "tanh"), 2e-2, 2e-2)


@pytest.mark.parametrize("M,N,K", _LIN_SHAPES)
@pytest.mark.parametrize("with_act", [False, True])
def test_linear_dgrad(M, N, K, with_act, lin_tile):
    """dx[M, K] = g[M, N] W[N, K] (NN: hardware-transposed W tiles), optionally * gelu'(pre)."""
    if K % 128:
        pytest.skip("dgrad output dim must be a multiple of 128 (library GEMM otherwise)")
    torch.manual_seed(1)
    C = ops.native()
    g = torch.randn(M, N, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * N ** -0.5).bfloat16()
    pre = torch.randn(M, K, device=DEV).bfloat16() if with_act else None
    dx = C.linear_dgrad(g, w, pre, 0 if with_act else -1)
    ref = g.float() @ w.float()
    if with_act:
        p = pre.float().requires_grad_(True)
        torch.nn.functional.gelu(p).backward(ref)
        ref = p.grad
    _close(dx, ref, 2e-2, 2e-2)


def test_fused_ffn_autograd_matches_reference():
    """linear_act + linear_after_act (GEMM epilogues carry bias+GELU and GELU') == the unfused
    library path, forward and every gradient."""
    import os
    torch.manual_seed(2)
    T, H, I = 2048, 768, 3072
    x0 = torch.randn(T, H, device=DEV).bfloat16()
    w1 = (torch.randn(I, H, device=DEV) * 0.02).bfloat16()
    b1 = (torch.randn(I, device=DEV) * 0.1).bfloat16()
    w2 = (torch.randn(H, I, device=DEV) * 0.02).bfloat16()
    gy = torch.randn(T, H, device=DEV).bfloat16()
    res = {}
    for route in ("bcfl", "torch"):
        os.environ["BCFL_TORCH_OPS"] = "" if route == "bcfl" else "gemm,gemm_act"
        _native.refresh_env()
        try:
            x = x0.clone().requires_grad_(True)
            p1, q1, p2 = (t.clone().requires_grad_(True) for t in (w1, b1, w2))
            h, pre = ops.linear_act(x, p1, q1, "gelu")
            assert (pre is not None) == (route == "bcfl")
            y = ops.linear_after_act(h, pre, p2, "gelu")
            y.backward(gy)
            res[route] = [y, x.grad, p1.grad, q1.grad, p2.grad]
        finally:
            os.environ["BCFL_TORCH_OPS"] = ""
            _native.refresh_env()
    for name, a, b in zip(("y", "dx", "dW1", "db1", "dW2"), res["bcfl"], res["torch"]):
        # both sides are bf16 results of fp32 accumulations with different rounding points
        # (fused epilogue vs bf16 GEMM output + separate bias/GELU): compare normwise
        err = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert err < 1e-2, (name, err)


@pytest.mark.parametrize("nh,nkv,d,causal,p", [(12, 12, 64, False, 0.0), (12, 12, 64, False, 0.1),
                                               (8, 2, 128, True, 0.0), (4, 4, 32, False, 0.1)])
def test_subset_attention_matches_torch_reference(nh, nkv, d, causal, p):
    """subset_attention.hip (fwd + bwd, dropout keep bits, GQA, causal last-token rows) == the
    torch implementation of the same pooled-row attention (BCFL_TORCH_OPS=subset_attn)."""
    import os
    torch.manual_seed(3)
    lens = np.array([37, 300, 5, 129, 64])
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    T = int(cu[-1])
    rows = torch.from_numpy(cu[1:] - 1 if causal else cu[:-1]).to(DEV)
    cu_d = torch.from_numpy(cu).to(DEV)
    x0 = torch.randn(T, (nh + 2 * nkv) * d, device=DEV).bfloat16()
    g = torch.randn(len(lens), nh * d, device=DEV).bfloat16()
    ops.rng.global_rng().load_state({"seed": 5, "counter": 0})
    res = {}
    for route in ("bcfl", "torch"):
        os.environ["BCFL_TORCH_OPS"] = "" if route == "bcfl" else "subset_attn"
        _native.refresh_env()
        try:
            ops.rng.global_rng().load_state({"seed": 5, "counter": 0})
            x = x0.clone().requires_grad_(True)
            o = ops.query_subset_attention(x, rows, cu_d, int(lens.max()), nh, nkv, d, p, True, causal)
            o.backward(g)
            res[route] = (o.float(), x.grad.float())
        finally:
            os.environ["BCFL_TORCH_OPS"] = ""
            _native.refresh_env()
    _close(res["bcfl"][0], res["torch"][0], 2e-2, 2e-2)
    _close(res["bcfl"][1], res["torch"][1], 2e-2, 2e-2)


def test_native_dropout_mask_matches_hash_layout():
    import os
    x = torch.randn(32, 768, device=DEV).bfloat16()
    ops.rng.global_rng().load_state({"seed": 9, "counter": 4})
    y = ops.dropout(x, 0.1, True)
    os.environ["BCFL_TORCH_OPS"] = "dropout"
    _native.refresh_env()
    try:
        ops.rng.global_rng().load_state({"seed": 9, "counter": 4})
        r = ops.dropout(x, 0.1, True)
    finally:
        os.environ["BCFL_TORCH_OPS"] = ""
        _native.refresh_env()
    assert torch.equal(y == 0, r == 0)           # identical keep decisions
    _close(y, r, 1e-2, 1e-2)


@pytest.mark.parametrize("T,with_res", [(1000, False), (2048, False), (4096, False),
                                        (4096, True), (1000, True)])
def test_lora_linear_fused_matches_unfused(T, with_res):
    """ops.lora_linear == the unfused x W^T + cat(xa_i B_i^T) * s path, forward and gradients.
    T = 1000: the two-GEMM path (low-rank product written first, base GEMM accumulating);
    T >= 1024: every product on the 8-phase GEMM (split-K skinny GEMMs, tail segments, weight-
    gradient kernel; since round 4 the four tall-skinny products on skinny.hip). ``with_res``:
    + a residual stream input, added in the GEMM epilogue (EPI_RESID) on the fused path."""
    import os
    torch.manual_seed(4)
    K, r = 512, 16
    sizes = [512, 128, 128]
    x0 = torch.randn(T, K, device=DEV).bfloat16()
    w = (torch.randn(sum(sizes), K, device=DEV) * 0.05).bfloat16()
    a0 = (torch.randn(len(sizes) * r, K, device=DEV) * 0.05).bfloat16()
    b0 = [(torch.randn(n, r, device=DEV) * 0.05).bfloat16() for n in sizes]
    g = torch.randn(T, sum(sizes), device=DEV).bfloat16()
    r0 = torch.randn(T, sum(sizes), device=DEV).bfloat16()
    res = {}
    for route in ("bcfl", "torch"):
        os.environ["BCFL_TORCH_OPS"] = "" if route == "bcfl" else "lora"
        _native.refresh_env()
        try:
            x = x0.clone().requires_grad_(True)
            a = a0.clone().requires_grad_(True)
            bs = [b.clone().requires_grad_(True) for b in b0]
            rr = r0.clone().requires_grad_(True) if with_res else None
            y = ops.lora_linear(x, w, a, bs, 2.0, rr)
            y.backward(g)
            res[route] = [y, x.grad, a.grad] + [b.grad for b in bs] + ([rr.grad] if with_res else [])
        finally:
            os.environ["BCFL_TORCH_OPS"] = ""
            _native.refresh_env()
    for u, v in zip(res["bcfl"], res["torch"]):
        err = ((u.float() - v.float()).norm() / v.float().norm()).item()
        assert err < 1e-2, err


@pytest.mark.parametrize("M,N,K,nr", [(1000, 768, 512, 48), (7680, 3072, 768, 48),
                                       (2048, 512, 1024, 16), (512, 256, 256, 160)])
def test_lora_tail_gemms_match_fp32(M, N, K, nr):
    """gemm8.hip tail segment: lora_fwd = x W^T + xa bb^T and lora_dgrad = g W + gb A in ONE
    GEMM (low-rank columns zero-padded to whole 128-deep K-tile pairs; the COL A operand's rows
    past nr read as zero), vs fp32 torch. Covers BM 256 / 128, the persistent grid (7680 x 3072)
    and a tail of two K-tile pairs (nr = 160)."""
    torch.manual_seed(M + N + nr)
    C = ops.native()
    k2 = -(-nr // 128) * 128
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    xa = torch.zeros(M, k2, device=DEV, dtype=torch.bfloat16)
    xa[:, :nr] = torch.randn(M, nr, device=DEV).bfloat16()
    bb = torch.zeros(N, k2, device=DEV, dtype=torch.bfloat16)
    bb[:, :nr] = (torch.randn(N, nr, device=DEV) * 0.1).bfloat16()
    assert C.lora_native_ok(M, N, K, False)
    y = C.lora_fwd(x, w, xa, bb)
    ref_y = x.float() @ w.float().t() + xa.float() @ bb.float().t()
    _close(y, ref_y, 5e-2, 2e-2)
    g = torch.randn(M, N, device=DEV).bfloat16()
    gb = torch.zeros(M, k2, device=DEV, dtype=torch.bfloat16)
    gb[:, :nr] = torch.randn(M, nr, device=DEV).bfloat16()
    gb[:, nr:] = 7.0  # padding columns are ignored: the A operand's rows past nr read as zero
    a = (torch.randn(nr, K, device=DEV) * 0.1).bfloat16()
    assert C.lora_native_ok(M, K, N, True)
    dx = C.lora_dgrad(g, w, gb, a)
    ref_dx = g.float() @ w.float() + gb[:, :nr].float() @ a.float()
    _close(dx, ref_dx, 5e-2, 2e-2)


@pytest.mark.parametrize("sizes,r", [([512, 128, 128], 16), ([768, 768], 16), ([1024], 16), ([256, 64, 64], 8)])
def test_lora_pack_b_and_block_diagonal_db(sizes, r):
    """skinny.hip LoRA helpers: lora_pack_b = (s Bbd zero-padded to k2 columns, its [n r, N]
    transpose) in one launch; skinny_ptx_bdiag = the adapters' dB_i = s (xa^T g)[block i]^T as
    contiguous row blocks of one [N, r] tensor."""
    torch.manual_seed(sum(sizes) + r)
    C = ops.native()
    N, nr, k2, s = sum(sizes), len(sizes) * r, 128, 2.0
    bs = [torch.randn(o, r, device=DEV).bfloat16() for o in sizes]
    bb, bbt = C.lora_pack_b(bs, s, k2)
    ref = torch.zeros(N, k2, device=DEV)
    ref[:, :nr] = torch.block_diag(*[b.float() for b in bs]) * s
    assert torch.equal(bb, ref.bfloat16())
    assert torch.equal(bbt, ref[:, :nr].t().contiguous().bfloat16())
    M = 3000
    xa = torch.randn(M, nr, device=DEV).bfloat16()
    g = torch.randn(M, N, device=DEV).bfloat16()
    out = C.skinny_ptx_bdiag(xa, g, sizes, s)
    full = s * (xa.float().t() @ g.float())
    o = 0
    for i, n in enumerate(sizes):
        _close(out[o:o + n], full[i * r:(i + 1) * r, o:o + n].t(), 2e-2, 2e-2)
        o += n


@pytest.mark.parametrize("M,H,I,nr", [(2048, 512, 768, 32), (8192, 1024, 1536, 32), (1500, 256, 512, 16)])
def test_lora_swiglu_epilogues_match_fp32(M, H, I, nr):
    """gemm8.hip EPI_SWIGLU: [gate|up] = x Wgu^T + xa bb^T with each output tile pairing gate
    columns with the same up columns (B half-tile 1 read I rows further), act = silu(gate) up;
    EPI_SWIGLU_BWD: dgu = SwiGLU'(gu) . (g Wd + gb Ad) with dA never stored. vs fp32 torch."""
    torch.manual_seed(M + I)
    C = ops.native()
    k2 = -(-nr // 128) * 128
    x = torch.randn(M, H, device=DEV).bfloat16()
    wgu = (torch.randn(2 * I, H, device=DEV) * 0.05).bfloat16()
    xa = torch.zeros(M, k2, device=DEV, dtype=torch.bfloat16)
    xa[:, :nr] = torch.randn(M, nr, device=DEV).bfloat16()
    bb = torch.zeros(2 * I, k2, device=DEV, dtype=torch.bfloat16)
    bb[:, :nr] = (torch.randn(2 * I, nr, device=DEV) * 0.1).bfloat16()
    act, gu = C.lora_fwd_swiglu(x, wgu, xa, bb)
    ref_gu = x.float() @ wgu.float().t() + xa.float() @ bb.float().t()
    _close(gu, ref_gu, 5e-2, 2e-2)
    g_, u_ = gu.float()[:, :I], gu.float()[:, I:]      # the kernel's own bf16 projection
    _close(act, torch.nn.functional.silu(g_) * u_, 2e-2, 2e-2)
    wd = (torch.randn(H, I, device=DEV) * 0.05).bfloat16()
    gy = torch.randn(M, H, device=DEV).bfloat16()
    gb = torch.zeros(M, k2, device=DEV, dtype=torch.bfloat16)
    gb[:, :nr] = torch.randn(M, nr, device=DEV).bfloat16()
    ad = (torch.randn(nr, I, device=DEV) * 0.1).bfloat16()
    dgu = C.lora_dgrad_swiglu(gy, wd, gb, ad, gu)
    dA = (gy.float() @ wd.float() + gb[:, :nr].float() @ ad.float()).bfloat16().float()
    sg = torch.sigmoid(g_)
    ref_dg = dA * u_ * sg * (1 + g_ * (1 - sg))
    ref_du = dA * g_ * sg
    _close(dgu[:, :I], ref_dg, 5e-2, 2e-2)
    _close(dgu[:, I:], ref_du, 5e-2, 2e-2)


@pytest.mark.parametrize("T", [2048, 4096])
def test_lora_swiglu_mlp_matches_unfused(T):
    """ops.lora_swiglu_mlp (SwiGLU forward / backward in the GEMM epilogues, one autograd node for
    the whole LoRA MLP) == two ops.lora_linear + ops.swiglu on the torch route: output and every
    gradient (input, residual, both A's and all B's)."""
    import os
    from bcfl.ops import functional as F
    torch.manual_seed(T)
    H, I, r = 512, 768, 16
    x0 = torch.randn(T, H, device=DEV).bfloat16()
    r0 = torch.randn(T, H, device=DEV).bfloat16()
    wgu = (torch.randn(2 * I, H, device=DEV) * 0.05).bfloat16()
    wd = (torch.randn(H, I, device=DEV) * 0.05).bfloat16()
    agu0 = (torch.randn(2 * r, H, device=DEV) * 0.05).bfloat16()
    ad0 = (torch.randn(r, I, device=DEV) * 0.05).bfloat16()
    bgu0 = [(torch.randn(I, r, device=DEV) * 0.05).bfloat16() for _ in range(2)]
    bd0 = [(torch.randn(H, r, device=DEV) * 0.05).bfloat16()]
    gy = torch.randn(T, H, device=DEV).bfloat16()
    assert F._lora_mlp_fused_ok(x0, wgu, agu0, wd, ad0)
    res = {}
    for route in ("bcfl", "torch"):
        os.environ["BCFL_TORCH_OPS"] = "" if route == "bcfl" else "lora"
        _native.refresh_env()
        try:
            x, rr = x0.clone().requires_grad_(True), r0.clone().requires_grad_(True)
            agu, ad = agu0.clone().requires_grad_(True), ad0.clone().requires_grad_(True)
            bgu = [b.clone().requires_grad_(True) for b in bgu0]
            bd = [b.clone().requires_grad_(True) for b in bd0]
            y = ops.lora_swiglu_mlp(x, wgu, agu, bgu, 2.0, wd, ad, bd, 2.0, rr)
            y.backward(gy)
            res[route] = [y, x.grad, rr.grad, agu.grad, ad.grad] + [b.grad for b in bgu + bd]
        finally:
            os.environ["BCFL_TORCH_OPS"] = ""
            _native.refresh_env()
    for i, (u, v) in enumerate(zip(res["bcfl"], res["torch"])):
        err = ((u.float() - v.float()).norm() / v.float().norm()).item()
        assert err < 2e-2, (i, err)


@pytest.mark.parametrize("B,C", [(32, 2), (7, 41), (256, 40), (300, 3)])
def test_xent_kernels_match_torch(B, C):
    torch.manual_seed(B + C)
    lg = (torch.randn(B, C, device=DEV) * 3).bfloat16().requires_grad_(True)
    lab = torch.randint(0, C, (B,), device=DEV)
    loss = ops.cross_entropy(lg, lab)
    (loss * 2.0).backward()
    ref_lg = lg.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(ref_lg, lab)
    (ref * 2.0).backward()
    _close(loss, ref, 1e-4, 1e-4)
    _close(lg.grad, ref_lg.grad, 1e-3, 2e-2)
    acc = torch.zeros(4, dtype=torch.float64, device=DEV)
    ops.xent_stats_(lg.detach(), lab, acc)
    ops.xent_stats_(lg.detach(), lab, acc)
    ce = torch.nn.functional.cross_entropy(lg.detach().float(), lab, reduction="sum").double()
    want = torch.stack([2 * (lg.detach().float().argmax(-1) == lab).sum().double(),
                        torch.tensor(2.0 * B, device=DEV, dtype=torch.float64), 2 * ce, 2 * ce / B])
    torch.testing.assert_close(acc, want, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("model", ["bert-base-2l", "distilbert"])
def test_residual_tap_matches_autograd_sum(model, monkeypatch):
    """LayerNorm residual gradients routed into the consumer's dgrad GEMM (ops.ResidualTap,
    beta = 1 accumulation) give the same parameter gradients as autograd's separate sum."""
    from bcfl.data.batching import make_packed_batch
    from bcfl.data.registry import load_split
    from bcfl.models import build_model, special_tokens
    import bcfl.models.bert as mb
    import bcfl.models.distilbert as md
    cls_id, sep_id, vocab = special_tokens(model)
    ds = load_split("imdb", "train", vocab, 512, 1234, cls_id, sep_id)
    b = make_packed_batch(ds, np.arange(0, 25000, 1563)[:16]).to(DEV)
    used = []

    class Rec(ops.ResidualTap):
        __slots__ = ()

        def __setattr__(self, k, v):
            if k == "g" and v is not None:
                used.append(1)
            object.__setattr__(self, k, v)

    grads = {}
    for on in (False, True):
        tap = Rec if on else (lambda: None)
        monkeypatch.setattr(mb.ops, "ResidualTap", tap)
        monkeypatch.setattr(md.ops, "ResidualTap", tap)
        rng.manual_seed(7)
        m = build_model(model, 2, device=DEV, dtype=torch.bfloat16, seed=0)
        m.train()
        loss = ops.cross_entropy(m(b), b.labels)
        loss.backward()
        ops.join_wgrad()
        grads[on] = [p.grad.float().clone() for p in m.parameters() if p.grad is not None]
    assert used, "no residual gradient was routed through a tap"
    assert len(grads[False]) == len(grads[True])
    for a, c in zip(grads[False], grads[True]):
        assert ((a - c).norm() / a.norm().clamp_min(1e-12)) < 2e-2


def test_multi_tensor_adamw_sums_second_gradient():
    """adamw_mt with grads2 == adamw_mt on (g1 + g2) (micro-batch replicas' gradients)."""
    torch.manual_seed(0)
    shapes = [(768, 768), (3072,), (33,)]
    offs, o = [], 0
    for s in shapes:
        offs.append(o)
        o += (math.prod(s) + 63) // 64 * 64
    g1 = [torch.randn(s, device=DEV).bfloat16() for s in shapes]
    g2 = [torch.randn(s, device=DEV).bfloat16() for s in shapes]
    gs = [(a.float() + b.float()).bfloat16() for a, b in zip(g1, g2)]
    res = []
    for grads, grads2 in ((g1, g2), (gs, None)):
        torch.manual_seed(1)
        master = torch.randn(o, device=DEV)
        m_, v_ = torch.zeros(o, device=DEV), torch.zeros(o, device=DEV)
        ops.adamw_multi_(master, grads, offs, m_, v_, 1, 1e-3, 0.9, 0.999, 1e-6, 0.0, "hf",
                         grads2=grads2)
        res.append((master, m_, v_))
    # g1 + g2 in fp32 inside the kernel vs a bf16-rounded sum: m differs by bf16 rounding only
    for a, b in zip(res[0], res[1]):
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)) < 1e-2


def test_embedding_grads_with_host_sort_order_are_identical():
    """Table gradients from the host-precomputed stable sort orders (ClientLoader presort) are
    bitwise identical to the device-sort path."""
    from bcfl.data.batching import make_packed_batch, pad_packed, presort
    from bcfl.data.registry import load_split
    torch.manual_seed(0)
    ds = load_split("imdb", "train", 30522, 512)
    b = presort(pad_packed(make_packed_batch(ds, np.arange(0, 25000, 997)[:24]), 256)).to(DEV)
    assert b.sort_ids.shape == (2, b.num_tokens) and b.sort_ids.dtype == torch.int32
    H = 768
    word = (0.02 * torch.randn(30522, H, device=DEV)).bfloat16().requires_grad_(True)
    posw = (0.02 * torch.randn(512, H, device=DEV)).bfloat16().requires_grad_(True)
    typ = (0.02 * torch.randn(2, H, device=DEV)).bfloat16().requires_grad_(True)
    g = torch.ones(H, device=DEV).bfloat16().requires_grad_(True)
    be = torch.zeros(H, device=DEV).bfloat16().requires_grad_(True)
    go = torch.randn(b.num_tokens, H, device=DEV).bfloat16()
    outs = []
    for order in (None, b.order()):
        rng.manual_seed(3)
        y = ops.embedding_layernorm(b.input_ids, b.position_ids, None, word, posw, typ, g, be,
                                    1e-12, 0.1, True, order=order)
        outs.append(torch.autograd.grad(y, (word, posw, typ, g, be), go))
    for a, c in zip(*outs):
        assert torch.equal(a, c)


@pytest.mark.parametrize("with_g2", [False, True])
def test_grad_clip_coef_and_clipped_adamw(with_g2):
    """Fused global-norm clipping (FLConfig.max_grad_norm): the multi-tensor norm kernel equals
    the fp64 norm of the concatenated gradients, the coefficient is torch's clip_grad_norm_
    (min(1, max / (norm + 1e-6))), and adamw_mt with the device coefficient equals AdamW on the
    clipped gradients — with no host read in between."""
    torch.manual_seed(1)
    sizes = [768, 3, 3072 * 768, 5, 777] + [129] * 45
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += (n + 63) // 64 * 64
    grads = [torch.randn(n, device=DEV).bfloat16() for n in sizes]
    g2 = [torch.randn(n, device=DEV).bfloat16() for n in sizes] if with_g2 else None
    full = [g.double() + (g2[i].double() if g2 else 0) for i, g in enumerate(grads)]
    norm = float(torch.cat(full).norm())
    for max_norm in (norm * 0.25, norm * 4):
        c = ops.grad_clip_coef(grads, max_norm, g2)
        assert c.is_cuda and c.dtype == torch.float32
        assert float(c[1]) == pytest.approx(norm, rel=1e-5)
        assert float(c[0]) == pytest.approx(min(1.0, max_norm / (norm + 1e-6)), rel=1e-5)
    c = ops.grad_clip_coef(grads, norm * 0.25, g2)
    master = torch.randn(o, device=DEV)
    m, v = torch.zeros(o, device=DEV), torch.zeros(o, device=DEV)
    rm, rmm, rvv = master.clone(), m.clone(), v.clone()
    ops.adamw_multi_(master, grads, offs, m, v, 1, 1e-3, 0.9, 0.999, 1e-6, 0.0, "hf",
                     grads2=g2, gscale=c)
    k = float(c[0])
    for gf, of in zip(full, offs):
        n = gf.numel()
        ref.adamw_(rm[of:of + n], (gf * k).float(), rmm[of:of + n], rvv[of:of + n], 1, 1e-3, 0.9,
                   0.999, 1e-6, 0.0, "hf")
    _close(m, rmm, 1e-6, 1e-5)
    _close(master, rm, 1e-5, 1e-5)


@pytest.mark.parametrize("M,K,R,cz", [(8192, 4096, 48, 128), (8000, 4096, 16, 128),
                                      (777, 1024, 32, 32), (8192, 14336, 32, 128)])
def test_skinny_xwt_matches_fp32(M, K, R, cz):
    """LoRA tall-skinny product out = scale * X W^T (skinny.hip), zero columns past R."""
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(R, K, device=DEV) * K ** -0.5).bfloat16()
    out = ops.native().skinny_xwt(x, w, cz, 2.0)
    ref_ = 2.0 * (x.float() @ w.float().t())
    assert out.shape == (M, cz)
    _close(out[:, :R], ref_, 2e-2, 2e-2)
    assert (out[:, R:] == 0).all()
    assert torch.equal(out, ops.native().skinny_xwt(x, w, cz, 2.0))   # deterministic slices


@pytest.mark.parametrize("M,N,R", [(8192, 4096, 48), (8000, 6144, 16), (640, 1024, 32),
                                   (8192, 28672, 32)])
def test_skinny_ptx_matches_fp32(M, N, R):
    """LoRA adapter-gradient product out = scale * P^T X over the M tokens (skinny.hip: both
    operands through LDS, hardware-transposed reads)."""
    torch.manual_seed(1)
    p = torch.randn(M, R, device=DEV).bfloat16()
    x = torch.randn(M, N, device=DEV).bfloat16()
    out = ops.native().skinny_ptx(p, x, 0.5)
    ref_ = 0.5 * (p.float().t() @ x.float())
    assert out.shape == (R, N)
    _close(out, ref_, 2e-2, 2e-2)
    assert torch.equal(out, ops.native().skinny_ptx(p, x, 0.5))


@pytest.mark.parametrize("T,H", [(1000, 4096), (65, 1024)])
def test_rmsnorm_wide_rows_frozen_weight(T, H):
    """Wide-row RMSNorm (Llama H = 4096, packed-bf16 rows, 16-byte lanes) with a FROZEN weight
    (LoRA: no weight gradient) vs the fp32 reference, forward and input gradient."""
    torch.manual_seed(3)
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    out = ops.rmsnorm(x, w, 1e-5)
    xf = x.detach().float().requires_grad_(True)
    r = ref.rmsnorm(xf, w.float(), 1e-5)
    _close(out, r, 3e-2)
    go = torch.randn_like(out)
    out.backward(go)
    r.backward(go.float())
    _grads_close([x.grad], [xf.grad])

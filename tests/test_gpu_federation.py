"""GPU correctness of the concurrent paths the bench runs: interleaved client lanes on their own
HIP streams (with and without side-stream weight gradients) must reproduce one-lane training
BITWISE (the bcfl kernels are deterministic), and concurrent large GEMMs on two streams (the
shape class that once deadlocked hipBLASLt Stream-K) must complete and agree with one stream."""
import os

import numpy as np
import pytest
import torch

from bcfl import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _run(tmp, lanes, overlap, **kw):
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    D.set_runtime_for_tests(None)
    kw.setdefault("num_rounds", 2)
    cfg = FLConfig(mode="serverless", model="bert-base-2l", dataset="imdb", num_clients=4,
                   train_samples=64, test_samples=32, global_test_samples=64,
                   out_dir=tmp, reference_prints=False, client_lanes=lanes, overlap_wgrad=overlap,
                   async_gossip=False, gossip_transport="rccl", ledger=True, save_every=0,
                   dropout=0.1, drift_correction="scaffold", wgrad_slots=64, **kw)
    fed = Federation(cfg, verbose=False)
    assert len(fed.lanes) == lanes
    h = fed.run()
    torch.cuda.synchronize()
    out = (torch.stack([fed.client_master[c] for c in range(4)]).cpu(),
           [r["train_loss"] for r in h], [b["update_root"] for b in fed.ledger.blocks()])
    D.set_runtime_for_tests(None)
    return out


@pytest.mark.parametrize("lanes,overlap", [(3, False), (3, True), (1, True)])
def test_gpu_lanes_match_sequential(tmp_path, lanes, overlap):
    """Every BERT GEMM (the 8-phase gemm8 kernels, including the weight gradients), the
    attention and the reductions are bcfl's own deterministic kernels, so concurrent lanes and
    side-stream weight gradients reproduce one-lane training BIT FOR BIT: masters, loss curve
    and the ledger's update roots, at the same weight-gradient split count (``wgrad_slots``; the
    auto value differs between one lane and several). (The K9 weight-gradient kernel of gemm.hip only serves shapes
    that are not 256-multiples — ALBERT's 128-wide embedding projection — and is pinned by
    tests/test_gpu_kernels.py::test_wgrad_split_m.)"""
    a = _run(str(tmp_path / "ref"), 1, False)
    b = _run(str(tmp_path / "x"), lanes, overlap)
    assert torch.isfinite(a[0]).all()
    d = (a[0] - b[0]).abs().max().item()
    assert torch.equal(a[0], b[0]), f"lane run differs from one lane by {d:.3e}"
    assert a[1] == b[1]
    assert a[2] == b[2]


def test_gpu_prefetched_batches_match_inline(tmp_path):
    """Round r + 1's training batches packed on the host prefetch thread (pinned staging while
    round r trains) are the inline batches: bit-identical masters, losses and ledger roots."""
    a = _run(str(tmp_path / "inline"), 1, True, prefetch_batches=False, num_rounds=3)
    b = _run(str(tmp_path / "pref"), 1, True, prefetch_batches=None, num_rounds=3)  # auto: on
    assert torch.isfinite(a[0]).all()
    assert torch.equal(a[0], b[0]) and a[1] == b[1] and a[2] == b[2]


def test_gpu_lanes_close_to_sequential(tmp_path):
    """Numerically the lane path IS the sequential computation (with the regime's own
    weight-gradient kernel choice, i.e. no pinning: tolerance-level agreement)."""
    a = _run(str(tmp_path / "ref"), 1, False)
    b = _run(str(tmp_path / "x"), 3, False)
    # Adam turns any reordered-reduction gradient difference into an O(lr) step difference
    assert float((a[0] - b[0]).abs().max()) < 2e-4
    assert a[1] == pytest.approx(b[1], rel=1e-3)


def test_gpu_deterministic_runs_are_bitwise_reproducible(tmp_path):
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    outs = []
    for i in range(2):
        D.set_runtime_for_tests(None)
        cfg = FLConfig(mode="serverless", model="bert-base-2l", dataset="imdb", num_clients=4,
                       num_rounds=2, train_samples=64, test_samples=32, global_test_samples=64,
                       out_dir=str(tmp_path / str(i)), reference_prints=False, save_every=0,
                       deterministic=True, dropout=0.1, drift_correction="scaffold")
        fed = Federation(cfg, verbose=False)
        assert len(fed.lanes) <= 1 and not ops.wgrad_overlap_enabled()
        fed.run()
        outs.append(torch.stack([fed.client_master[c] for c in range(4)]).cpu())
        D.set_runtime_for_tests(None)
    assert torch.equal(outs[0], outs[1])


def test_gpu_concurrent_llama_shaped_gemms_complete():
    """Two lanes' Llama-3-8B projections ([T,4096]x[4096,14336]-class) at the same time."""
    torch.manual_seed(0)
    T = 2048
    xs = [torch.randn(T, 4096, device=DEV, dtype=torch.bfloat16) for _ in range(2)]
    ws = [torch.randn(14336, 4096, device=DEV, dtype=torch.bfloat16) * 0.02,
          torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16) * 0.02]
    ref = [[x @ w.t() for w in ws] for x in xs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(DEV) for _ in range(2)]
    outs = [[None, None], [None, None]]
    for it in range(4):
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                for j, w in enumerate(ws):
                    outs[i][j] = xs[i] @ w.t()
    torch.cuda.synchronize()
    for i in range(2):
        for j in range(2):
            assert torch.equal(outs[i][j], ref[i][j])


@pytest.mark.parametrize("mode", ["serverless", "server"])
def test_gpu_overlapped_global_eval_matches_inline(tmp_path, mode):
    """Global evaluation on the side stream (snapshot + eval replica, result filed one round
    later) scores the same model on the same rows as the inline path, and the training it
    overlaps is unaffected (same client states / global model)."""
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    outs = []
    for ov in (False, True):
        D.set_runtime_for_tests(None)
        cfg = FLConfig(mode=mode, model="bert-base-2l", dataset="imdb", num_clients=4,
                       num_rounds=3, train_samples=64, test_samples=32, global_test_samples=96,
                       out_dir=str(tmp_path / str(ov)), reference_prints=False, save_every=0,
                       client_lanes=1, overlap_wgrad=False, dropout=0.1,
                       async_gossip=True, gossip_transport="mailbox", overlap_global_eval=ov)
        fed = Federation(cfg, verbose=False)
        assert (fed.eval_stream is not None) == ov
        h = fed.run()
        state = (torch.stack([fed.client_master[c] for c in range(4)]) if mode == "serverless"
                 else fed.global_master.unsqueeze(0))
        outs.append(([r["global_acc"] for r in h], [r["global_loss"] for r in h],
                     [r["global_eval_rows"] for r in h], list(fed.global_accuracies),
                     state.cpu()))
        D.set_runtime_for_tests(None)
    (a_acc, a_loss, a_rows, a_g, a_m), (b_acc, b_loss, b_rows, b_g, b_m) = outs
    assert None not in b_acc and b_rows == a_rows == [96] * 3
    assert b_g == b_acc and a_g == a_acc
    # concurrency may reorder library reductions (~1e-7): allow one borderline row to flip
    assert all(abs(x - y) <= 1.0 / 96 + 1e-9 for x, y in zip(a_acc, b_acc))
    assert b_loss == pytest.approx(a_loss, rel=1e-3)
    # concurrent evaluation can only reorder library reductions of the training GEMMs
    assert float((a_m - b_m).abs().max()) < 2e-4


def test_gpu_deferred_local_eval_matches_inline(tmp_path):
    """One client per rank (the 8-GPU layout): the local evaluation of the trained model runs on
    the eval side stream from a snapshot and is filed the next round; the scores, the metrics
    lines and the training it overlaps equal the inline path's."""
    import json
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    outs = []
    for ov in (False, True):
        D.set_runtime_for_tests(None)
        out = str(tmp_path / str(ov))
        cfg = FLConfig(mode="serverless", model="bert-base-2l", dataset="imdb", num_clients=1,
                       num_rounds=3, train_samples=64, test_samples=32, global_test_samples=64,
                       out_dir=out, reference_prints=False, save_every=0, overlap_wgrad=False,
                       dropout=0.1, async_gossip=True, gossip_transport="mailbox",
                       overlap_global_eval=ov, eval_local=True)
        fed = Federation(cfg, verbose=False)
        assert fed._defer_local_eval() == ov
        h = fed.run()
        loc = [json.loads(l) for l in open(os.path.join(out, "metrics.jsonl")) if '"local_acc"' in l]
        outs.append(([r["distributed_acc"] for r in h], [(x["round"], x["local_acc"]) for x in loc],
                     fed.flat.master.detach().cpu()))
        D.set_runtime_for_tests(None)
    (a_d, a_l, a_m), (b_d, b_l, b_m) = outs
    assert None not in b_d and b_d == a_d
    assert sorted(b_l) == sorted(a_l)
    assert float((a_m - b_m).abs().max()) < 2e-4


@pytest.mark.parametrize("drift", ["none", "scaffold"])
def test_gpu_overlapped_optimizer_is_bitwise(tmp_path, drift):
    """Per-layer AdamW launched from the gradient hooks on a side stream mid-backward (one-lane
    ranks) gives bitwise the same models as the one-pass AdamW after the backward."""
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    outs = []
    for oo in (False, True):
        D.set_runtime_for_tests(None)
        cfg = FLConfig(mode="serverless", model="bert-base-2l", dataset="imdb", num_clients=1,
                       num_rounds=2, train_samples=96, test_samples=32, global_test_samples=64,
                       out_dir=str(tmp_path / f"{oo}"), reference_prints=False, save_every=0,
                       dropout=0.1, overlap_wgrad=True, overlap_optimizer=oo,
                       drift_correction=drift)
        fed = Federation(cfg, verbose=False)
        assert fed.opt.overlap_active() == oo
        h = fed.run()
        outs.append((fed.flat.master.detach().cpu(), fed.flat.param.detach().cpu(),
                     [r["train_loss"] for r in h]))
        D.set_runtime_for_tests(None)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]


def test_gpu_micro_batch_clients_match_full_batch(tmp_path):
    """Server mode trains one client at a time: with micro_batches=2 (2 concurrent micro-batches
    on 2 streams) the run tracks the full-batch run (dropout off; bf16 gradient sums round
    differently, so compare losses / parameters, not bits)."""
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    outs = []
    for mb in (1, 2):
        D.set_runtime_for_tests(None)
        cfg = FLConfig(mode="server", model="bert-base-2l", dataset="imdb", num_clients=2,
                       num_rounds=2, train_samples=64, test_samples=32, global_test_samples=64,
                       out_dir=str(tmp_path / str(mb)), reference_prints=False, save_every=0,
                       dropout=0.0, micro_batches=mb, overlap_wgrad=False)
        fed = Federation(cfg, verbose=False)
        assert fed.micro_split == (1 if mb == 1 else 2)
        h = fed.run()
        outs.append(([r["train_loss"] for r in h], [r["global_acc"] for r in h],
                     fed.global_master.cpu()))
        D.set_runtime_for_tests(None)
    (la, aa, ma), (lb, ab, mb_) = outs
    assert lb == pytest.approx(la, rel=2e-2)
    assert torch.isfinite(mb_).all()
    assert float((ma - mb_).abs().max()) < 5e-3


def _run_server(tmp, lanes):
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    D.set_runtime_for_tests(None)
    cfg = FLConfig(mode="server", model="bert-base-2l", dataset="imdb", num_clients=4,
                   num_rounds=2, train_samples=64, test_samples=32, global_test_samples=64,
                   out_dir=tmp, reference_prints=False, client_lanes=lanes, overlap_wgrad=False,
                   ledger=True, save_every=0, dropout=0.1)
    fed = Federation(cfg, verbose=False)
    assert len(fed.lanes) == lanes
    h = fed.run()
    torch.cuda.synchronize()
    out = (fed.global_master.cpu(), [r["train_loss"] for r in h], [r["global_acc"] for r in h])
    D.set_runtime_for_tests(None)
    return out


def test_gpu_server_lanes_close_to_sequential(tmp_path):
    """Server FedAvg with the hosted clients on concurrent lanes (per-lane partial sums) tracks
    one-lane training within the lanes tolerance (fp32 sum order of the lane partials)."""
    a = _run_server(str(tmp_path / "a"), 1)
    b = _run_server(str(tmp_path / "b"), 3)
    assert torch.isfinite(b[0]).all()
    assert float((a[0] - b[0]).abs().max()) < 2e-4
    assert a[1] == pytest.approx(b[1], rel=1e-3)


def test_gpu_lanes_run_has_no_unordered_stream_access(tmp_path, monkeypatch):
    """the 3-lane federation (lanes on their own streams, the eval side stream,
    the checkpoint copy stream) under the happens-before checker (BCFL_DEBUG_STREAMS): every
    buffer one stream writes and another touches is ordered by an event — no race is reported."""
    monkeypatch.setenv("BCFL_DEBUG_STREAMS", "1")
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    D.set_runtime_for_tests(None)
    cfg = FLConfig(mode="serverless", model="bert-base-2l", dataset="imdb", num_clients=4,
                   num_rounds=2, train_samples=64, test_samples=32, global_test_samples=64,
                   out_dir=str(tmp_path), reference_prints=False, client_lanes=3,
                   overlap_wgrad=False, async_gossip=False, gossip_transport="rccl", ledger=True,
                   save_every=1, dropout=0.1, drift_correction="scaffold")
    fed = Federation(cfg, verbose=False)
    fed.run()
    D.set_runtime_for_tests(None)
    assert fed.stream_races is not None, "the checker did not run"
    assert fed.stream_races == [], "\n".join(fed.stream_races)


def test_gpu_eval_graph_replays_match_eager(tmp_path, monkeypatch):
    """The side stream's evaluations replayed from hipGraphs (captured on their second use)
    return exactly the eager scores: global and deferred local accuracy / loss, every round."""
    import json
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    outs = []
    for graphs in ("0", "1"):
        monkeypatch.setenv("BCFL_EVAL_GRAPHS", graphs)
        D.set_runtime_for_tests(None)
        out = str(tmp_path / graphs)
        cfg = FLConfig(mode="serverless", model="bert-base-2l", dataset="imdb", num_clients=1,
                       num_rounds=4, train_samples=64, test_samples=32, global_test_samples=64,
                       out_dir=out, reference_prints=False, save_every=0, overlap_wgrad=False,
                       dropout=0.1, async_gossip=True, gossip_transport="mailbox",
                       overlap_global_eval=True, eval_local=True)
        fed = Federation(cfg, verbose=False)
        h = fed.run()
        loc = [json.loads(l) for l in open(os.path.join(out, "metrics.jsonl")) if '"local_acc"' in l]
        outs.append(([(r["global_acc"], r["global_loss"], r["distributed_acc"]) for r in h],
                     [(x["round"], x["local_acc"], x["local_loss"]) for x in loc],
                     sum(v is not None for v in getattr(fed, "_eval_graphs", {}).values()),
                     fed.flat.master.detach().cpu()))
        D.set_runtime_for_tests(None)
    (a_h, a_l, a_n, a_m), (b_h, b_l, b_n, b_m) = outs
    assert a_n == 0 and b_n == 3   # global + the two local snapshot buffers
    assert a_h == b_h and a_l == b_l
    assert torch.equal(a_m, b_m)

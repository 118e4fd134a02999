"""Multi-process (gloo, world 2) tests of the distributed paths — the CPU stand-in for the 8-GPU
node. Key property: N real ranks give BIT-IDENTICAL models to 1 rank hosting N virtual clients."""
import os

import pytest
import torch

from dist_utils import run_world


def _cfg(mode, out, **kw):
    from bcfl.config import FLConfig
    base = dict(mode=mode, model="tiny-bert", dataset="tiny", num_clients=2, num_rounds=2,
                train_samples=48, test_samples=16, global_test_samples=32, batch_size=16, lr=1e-3,
                out_dir=out, partition="label_shards", reference_prints=False, save_every=0,
                device="cpu", backend="gloo")
    base.update(kw)
    return FLConfig(**base)


def _fed_worker(rank, world, mode, out, kw):
    from bcfl.fl import Federation
    fed = Federation(_cfg(mode, out, **kw), verbose=False)
    fed.run()
    res = {"master": fed.flat.master.clone(), "acc": torch.tensor(fed.global_accuracies)}
    if fed.ledger is not None:
        res["tip"] = fed.ledger.tip
        res["consensus"] = fed.ledger.consensus_check()
    return res


def _single(mode, out, **kw):
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    D.set_runtime_for_tests(None)
    nt = torch.get_num_threads()
    torch.set_num_threads(2)  # same intra-op threading as the workers -> same reduction order
    try:
        fed = Federation(_cfg(mode, out, **kw), verbose=False)
        fed.run()
    finally:
        torch.set_num_threads(nt)
    m = fed.flat.master.clone()
    D.set_runtime_for_tests(None)
    return m, fed


def test_p2p_exchange(tmp_path):
    res = run_world(_p2p_worker, 2, str(tmp_path))
    assert torch.equal(res[0], torch.arange(1000, dtype=torch.float32) + 1000)
    assert torch.equal(res[1], torch.arange(1000, dtype=torch.float32))


def _p2p_worker(rank, world):
    from bcfl.parallel import dist as D
    D.init_runtime("cpu", "gloo")
    send = torch.arange(1000, dtype=torch.float32) + 1000 * rank
    recv = torch.empty(1000)
    h = D.p2p_exchange([(send, 1 - rank)], [(recv, 1 - rank)])
    h.wait()
    return recv


def test_server_fedavg_ranks_equal_virtual(tmp_path):
    res = run_world(_fed_worker, 2, str(tmp_path / "d"), "server", str(tmp_path / "d"), {})
    assert torch.equal(res[0]["master"], res[1]["master"])
    single, _ = _single("server", str(tmp_path / "s"))
    assert torch.equal(res[0]["master"], single)
    assert res[0]["consensus"] and res[0]["tip"] == res[1]["tip"]


def test_serverless_sync_ranks_equal_virtual(tmp_path):
    # fp32 wire: full topology + average mixing = the reference's mean of snapshots; both clients
    # end every round on the bit-identical model, and 2 ranks == 2 virtual clients on 1 rank
    kw = {"async_gossip": False, "wire_dtype": "fp32"}
    res = run_world(_fed_worker, 2, str(tmp_path / "d"), "serverless", str(tmp_path / "d"), kw)
    assert torch.equal(res[0]["master"], res[1]["master"])
    single, fed = _single("serverless", str(tmp_path / "s"), **kw)
    assert torch.equal(res[0]["master"], single)


def test_serverless_bf16_delta_wire_close(tmp_path):
    # bf16 error-feedback deltas: neighbours differ only by bf16 rounding of ONE round's delta
    kw = {"async_gossip": False, "wire_dtype": "bf16", "num_rounds": 3}
    res = run_world(_fed_worker, 2, str(tmp_path / "d"), "serverless", str(tmp_path / "d"), kw)
    diff = (res[0]["master"] - res[1]["master"]).abs().max().item()
    assert diff < 1e-4
    single, _ = _single("serverless", str(tmp_path / "s"), **kw)
    assert torch.equal(res[0]["master"], single)


def test_serverless_async_runs_and_mixes(tmp_path):
    kw = {"async_gossip": True, "num_rounds": 3, "anomaly_filter": "both", "gossip_transport": "rccl"}
    res = run_world(_fed_worker, 2, str(tmp_path / "d"), "serverless", str(tmp_path / "d"), kw)
    a, b = res[0]["master"], res[1]["master"]
    assert torch.isfinite(a).all() and torch.isfinite(b).all()
    # mixing pulled the clients together relative to independent training
    single, _ = _single("serverless", str(tmp_path / "s"), **kw)
    torch.testing.assert_close(a, single, atol=1e-6, rtol=0)
    assert res[0]["consensus"]


def test_serverless_ring_four_ranks(tmp_path):
    kw = {"num_clients": 4, "topology": "ring", "mixing": "metropolis", "async_gossip": False,
          "wire_dtype": "fp32", "num_rounds": 2}
    res = run_world(_fed_worker, 4, str(tmp_path / "d"), "serverless", str(tmp_path / "d"), kw)
    single, _ = _single("serverless", str(tmp_path / "s"), **kw)
    torch.testing.assert_close(res[0]["master"], single, atol=1e-6, rtol=0)


def test_round_robin_pairs_cover_every_link():
    from bcfl.trust.probe import round_robin_pairs
    for w in (2, 3, 4, 5, 8):
        rounds = round_robin_pairs(w)
        seen = [p for r in rounds for p in r]
        assert len(seen) == len(set(seen)) == w * (w - 1) // 2
        for r in rounds:  # pairs of one round are disjoint
            flat = [x for p in r for x in p]
            assert len(flat) == len(set(flat))


def _probe_worker(rank, world):
    from bcfl.parallel import dist as D
    from bcfl.trust.probe import measure_bandwidth, probe_and_filter
    D.init_runtime("cpu", "gloo")
    bw = measure_bandwidth(nbytes=1 << 18, iters=2)
    excl = probe_and_filter(torch.zeros(1), num_clients=8, nbytes=1 << 18, iters=2)
    return {"bw": torch.tensor(bw), "excluded": torch.tensor(excl, dtype=torch.int64)}


def test_bandwidth_probe_gloo(tmp_path):
    res = run_world(_probe_worker, 4, str(tmp_path))
    bw = res[0]["bw"]
    assert bw.shape == (4, 4)
    assert torch.all(torch.diag(bw) == 0)
    off = bw[~torch.eye(4, dtype=torch.bool)]
    assert torch.all(off > 0)
    for r in res[1:]:  # every rank holds the same gathered matrix
        assert torch.equal(r["bw"], bw)
    # never a majority excluded; excluded clients come from whole ranks (2 clients per rank)
    ex = res[0]["excluded"].tolist()
    assert len(ex) <= 2 and len(ex) % 2 == 0


def _liveness_worker(rank, world, out):
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    D.init_runtime("cpu", "gloo")
    fed = Federation(_cfg("serverless", out, num_rounds=5, inject_drop=[1], liveness_timeout=1,
                          async_gossip=False, wire_dtype="bf16"), verbose=False)
    fed.run()
    return {"dead": torch.tensor(sorted(fed.gossip.dead), dtype=torch.int64),
            "hist_dead": torch.tensor([len(h["dead_peers"]) for h in fed.history])}


def test_gossip_liveness_dead_peer_is_dropped(tmp_path):
    res = run_world(_liveness_worker, 2, str(tmp_path), str(tmp_path / "o"))
    # client 1 (rank 1) stops publishing: rank 0 declares it dead once the timeout passes
    assert res[0]["dead"].tolist() == [1]
    assert res[0]["hist_dead"][0] == 0 and res[0]["hist_dead"][-1] == 1


def _torn_worker(rank, world):
    from bcfl.parallel import dist as D
    from bcfl.parallel.gossip import GossipEngine
    D.init_runtime("cpu", "gloo")
    x = torch.full((64,), float(rank + 1))
    eng = GossipEngine(2, {rank: x}, {0: [1], 1: [0]}, "bf16_delta", async_gossip=False)
    eng.seed_replicas(torch.zeros(64))
    eng.publish(0)
    if rank == 1:  # tear the message: head / tail versions differ
        eng.send_hdr[1][7] += 1
    eng.launch(0)
    eng.finish()
    return {"torn": torch.tensor(eng.torn), "replica": eng.replica[1 - rank].clone()}


def test_gossip_torn_message_not_applied(tmp_path):
    res = run_world(_torn_worker, 2, str(tmp_path))
    assert int(res[0]["torn"]) == 1 and torch.all(res[0]["replica"] == 0)  # rank 1's message rejected
    assert int(res[1]["torn"]) == 0 and torch.all(res[1]["replica"] == 1.0)


def test_info_passing_benchmark_gloo(tmp_path):
    import json as _json
    import sys as _sys
    _sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from benchmarks.info_passing import _cpu_worker
    out = str(tmp_path / "r.json")
    run_world(_cpu_worker, 3, str(tmp_path), 50_000, out)
    res = _json.load(open(out))
    assert res["world"] == 3 and len(res["sources"]) == 3
    for s in res["sources"]:
        assert s["measured_sync_s"] > 0 and s["measured_async_s"] > 0
        assert s["predicted_async_s"] <= s["predicted_sync_s"]


def test_server_bf16_wire_close_to_fp32(tmp_path):
    """server_wire_dtype=bf16: delta-coded all-to-all + all-gather (fp32 accumulate, half the
    wire bytes) lands within bf16 rounding of the UPDATE of the fp32 all-reduce result."""
    res = run_world(_fed_worker, 2, str(tmp_path / "d"), "server", str(tmp_path / "d"),
                    {"server_wire_dtype": "bf16"})
    assert torch.equal(res[0]["master"], res[1]["master"])  # every rank ends on the same model
    ref = run_world(_fed_worker, 2, str(tmp_path / "r"), "server", str(tmp_path / "r"), {})
    from bcfl.models import build_model
    init = torch.cat([p.detach().reshape(-1) for p in build_model("tiny-bert", 2, seed=42).parameters()])
    upd = (ref[0]["master"] - res[0]["master"]).abs().max()
    step = (ref[0]["master"][: init.numel()] - init).abs().max()
    assert 0 < upd <= 0.02 * step


def test_all_reduce_bf16_matches_sum(tmp_path):
    res = run_world(_bf16_ar_worker, 3, str(tmp_path))
    want = sum(torch.linspace(-1, 1, 1001) * (r + 1) for r in range(3))
    for r in res:
        assert torch.allclose(r, want, rtol=1e-2, atol=1e-2)
        assert torch.equal(r, res[0])


def _bf16_ar_worker(rank, world):
    from bcfl.parallel import dist as D
    D.init_runtime("cpu", "gloo")
    x = torch.linspace(-1, 1, 1001) * (rank + 1)
    nbytes = D.all_reduce_bf16_(x)
    per = -(-(-(-1001 // world)) // 64) * 64   # 1/world chunk, padded to 128-byte multiples
    assert nbytes == 2 * (world - 1) * per * 2
    return x


def test_deterministic_async_is_reproducible(tmp_path):
    kw = {"async_gossip": True, "deterministic": True, "num_rounds": 3}
    a = run_world(_fed_worker, 2, str(tmp_path / "a"), "serverless", str(tmp_path / "a"), kw)
    b = run_world(_fed_worker, 2, str(tmp_path / "b"), "serverless", str(tmp_path / "b"), kw)
    for x, y in zip(a, b):
        assert torch.equal(x["master"], y["master"])


def _bench_path_worker(rank, world, out, kw):
    """The bench's federation on 8 ranks (one client per rank), a few rounds."""
    torch.set_num_threads(1)
    from bcfl.config import get_preset
    from bcfl.fl import Federation
    cfg = get_preset("baseline3_learnable", model="tiny-bert", dataset="tiny", device="cpu",
                     backend="gloo", num_rounds=3, train_samples=32, test_samples=16,
                     global_test_samples=32, batch_size=16, max_seq_len=64, out_dir=out,
                     reference_prints=False, save_every=1, **kw)
    fed = Federation(cfg, verbose=False)
    hist = fed.run()
    res = {"master": fed.flat.master.clone(), "tip": fed.ledger.tip, "height": torch.tensor(len(fed.ledger)),
           "loss": torch.tensor([h["train_loss"] for h in hist])}
    if fed.ledger_audit is not None:
        res["audit_checked"] = torch.tensor(fed.ledger_audit["checked"])
        res["audit_mismatched"] = torch.tensor(fed.ledger_audit["mismatched"])
    if not fed.collective_free:
        res["consensus"] = torch.tensor(fed.ledger.consensus_check())
    import json as _json
    res["verdicts"] = sorted((_json.loads(b["payload"])["src_round"], b["client"], b["verdict"])
                             for b in fed.ledger.blocks() if b["kind"] == "verdict")
    res["collective_free"] = bool(fed.collective_free)
    return res


@pytest.mark.slow
def test_bench_path_world8_mailbox(tmp_path):
    """Exactly the bench configuration (async one-sided mailbox gossip, bf16 wire, Merkle
    verification, drift correction, per-round checkpoints) on 8 gloo ranks: every rank finishes,
    every accepted update matches its sender's commitment in the cross-rank ledger audit."""
    res = run_world(_bench_path_worker, 8, str(tmp_path / "d"), str(tmp_path / "d"), {})
    for r in res:
        assert torch.isfinite(r["master"]).all() and torch.isfinite(r["loss"]).all()
        assert int(r["audit_checked"]) > 0 and int(r["audit_mismatched"]) == 0
    assert os.path.exists(tmp_path / "d" / "global" / "model.safetensors")


@pytest.mark.slow
def test_bench_path_world8_anomaly_filter_consensus(tmp_path):
    """Same on 8 ranks with the update anomaly filter on. Round 6: the filter runs inside the
    asynchronous round-complete application (no collective), so every rank keeps its own chain —
    and every rank reaches the SAME verdict on every source of every complete round it applied
    (each judges identical payloads), every accepted update matches its sender's commitment."""
    res = run_world(_bench_path_worker, 8, str(tmp_path / "d"), str(tmp_path / "d"),
                    {"anomaly_filter": "both", "wire_dtype": "bf16"})
    for r in res:
        assert r["collective_free"]
        assert int(r["audit_checked"]) > 0 and int(r["audit_mismatched"]) == 0
    rounds = set.intersection(*[{t for t, _, _ in r["verdicts"]} for r in res])
    assert rounds, "no complete round was judged on every rank"
    views = [[v for v in r["verdicts"] if v[0] in rounds] for r in res]
    assert all(v == views[0] for v in views)
    assert len(views[0]) == 8 * len(rounds)   # one verdict per source per judged round


def _server_liveness_worker(rank, world, out, exit_after):
    from bcfl.fl import Federation
    fed = Federation(_cfg("server", out, num_clients=3, num_rounds=4, server_transport="mailbox",
                          # generous: a LIVE rank slowed by a loaded CPU (parallel test workers)
                          # must not miss the deadline; the dead rank costs one wait, once
                          server_timeout_s=15.0), verbose=False)
    rounds = exit_after if rank == world - 1 else fed.cfg.num_rounds
    for r in range(rounds):
        fed.run_round(r)
    if rank == world - 1:   # this rank "crashes": leaves without finishing, posts nothing more
        return {"rounds": torch.tensor(rounds)}
    fed.finish(audit=False)
    blocks = [b for b in fed.ledger.blocks() if b["kind"] == "global"]
    import json as _json
    absent = [_json.loads(b["payload"] or "{}").get("absent_ranks", []) for b in blocks]
    return {"rounds": torch.tensor(len(fed.history)), "G": fed.global_master.clone(),
            "live_w": torch.tensor([h["live_weight"] for h in fed.history], dtype=torch.float64),
            "absent": [list(a) for a in absent],
            "acc": torch.tensor([h["global_acc"] for h in fed.history])}


def test_server_mailbox_fedavg_survives_a_dead_rank(tmp_path):
    """Flower FedAvg accept_failures semantics without a server: rank 2 stops after round 1; the
    survivors finish every round, leave it out, re-normalise the weights over the live ranks
    (3 equal clients: 1 -> 2/3) and record the absentee in their ledgers."""
    res = run_world(_server_liveness_worker, 3, str(tmp_path / "d"), str(tmp_path / "d"), 2)
    assert int(res[2]["rounds"]) == 2
    for r in res[:2]:
        assert int(r["rounds"]) == 4 and torch.isfinite(r["G"]).all()
        lw = r["live_w"].tolist()
        assert lw[:2] == pytest.approx([1.0, 1.0]) and lw[2:] == pytest.approx([2 / 3, 2 / 3])
        assert r["absent"][:2] == [[], []] and r["absent"][2] == [2]
    assert torch.equal(res[0]["G"], res[1]["G"])   # same live set -> bit-identical global model


def test_server_mailbox_equals_allreduce_when_all_live(tmp_path):
    a = run_world(_fed_worker, 2, str(tmp_path / "a"), "server", str(tmp_path / "a"),
                  {"server_transport": "mailbox"})
    b = run_world(_fed_worker, 2, str(tmp_path / "b"), "server", str(tmp_path / "b"), {})
    assert torch.equal(a[0]["master"], a[1]["master"])
    torch.testing.assert_close(a[0]["master"], b[0]["master"], atol=1e-6, rtol=0)


def _server_lagging_worker(rank, world, out, join_after, transport="mailbox"):
    import json as _json
    import time as _time
    from bcfl.fl import Federation
    # the deadline only has to separate "not started yet" (rank 1 waits on a flag) from a live
    # rank on a loaded CPU (parallel test workers): 1 s was flaky there, 4 s is not
    fed = Federation(_cfg("server", out, num_clients=2, num_rounds=10, server_transport=transport,
                          server_timeout_s=4.0), verbose=False)
    go, joined = os.path.join(out, "rank0_alone.flag"), os.path.join(out, "rank1_joined.flag")

    def wait_for(path):   # test-only gates on ROUND progress (no wall-clock assumptions)
        t0 = _time.time()
        while not os.path.exists(path):
            if _time.time() - t0 > 300:
                raise TimeoutError(path)
            _time.sleep(0.01)
    if rank == 1:
        wait_for(go)       # rank 1 is slow to start: rank 0 aggregates `join_after` epochs alone
    r = 0
    while r < fed.cfg.num_rounds:
        if rank == 0 and r == join_after + 2:
            wait_for(joined)   # rank 0 is still running when rank 1 joins (any CPU speed)
        fed.run_round(r)
        if rank == 0 and r == join_after - 1:
            open(go, "w").close()
        if rank == 1 and not os.path.exists(joined):
            open(joined, "w").close()
        r = fed.next_round(r)
    fed.finish()
    rounds = [b for b in fed.ledger.blocks() if b["kind"] == "global"]
    pay = [_json.loads(b["payload"] or "{}") for b in rounds]
    fin = [b for b in fed.ledger.blocks() if b["kind"] == "final_check"]
    return {"G": fed.global_master.clone(),
            "absent": [list(p.get("absent_ranks", [])) for p in pay],
            "mismatch": [list(p.get("view_mismatch", [])) for p in pay],
            "rejoined": [list(p.get("rejoined_ranks", [])) for p in pay],
            "skipped": [int(p.get("epochs_skipped", 0)) for p in pay],
            "rounds_run": torch.tensor(len(fed.history)),
            "final_split": torch.tensor(int(bool(fed.final_check and fed.final_check["split"]))),
            "final_blocks": torch.tensor(len(fin)),
            "audit_checked": torch.tensor(fed.ledger_audit["checked"]),
            "audit_mismatched": torch.tensor(fed.ledger_audit["mismatched"])}


@pytest.mark.parametrize("transport", ["mailbox", "mailbox_rs"])
def test_server_mailbox_slow_rank_rejoins_and_split_is_flagged(tmp_path, transport):
    """ADVICE r3 / VERDICT r4 #3: a rank that misses deadlines (slow, not dead) must not be excluded
    for good, must not report the epochs it skipped as trained, and a split must never be silent.
    Rank 1 joins only after rank 0 has aggregated 3 epochs alone (gated on rank 0's rounds, not on
    sleeps): rank 1 joins the federation's current epoch and records the skipped ones; the split
    of that epoch is reported (view_mismatch); rank 0 waits for rank 1 again; at the end every
    rank's final global-model root is compared (ledger ``final_check``) — equal models, or a
    split flagged on every rank. Both mailbox transports (the reduce-scatter path now
    takes the same epoch catch-up rule and waits for a lagging rank again)."""
    res = run_world(_server_lagging_worker, 2, str(tmp_path / "d"), str(tmp_path / "d"), 3,
                    transport)
    r0, r1 = res
    assert r0["absent"][0] == [1]                      # rank 0 timed out on the late rank 1
    assert r1["absent"][0] == []                       # ... which joined rank 0's epoch
    # the jump is on record (rank 0 aggregated >= 2 epochs alone before rank 1's first post; how
    # many exactly depends on how long rank 1 takes to start)
    assert r1["skipped"][0] >= 2 and sum(r0["skipped"]) == 0
    assert int(r1["rounds_run"]) < int(r0["rounds_run"])        # ... and not run as rounds
    assert any(m for m in r0["mismatch"] + r1["mismatch"])   # the split is reported
    assert r0["absent"][-1] == [] and r1["absent"][-1] == []  # rank 1 came back
    for r in res:
        assert int(r["final_blocks"]) == 1             # final roots compared on every rank
        assert int(r["audit_checked"]) > 0 and int(r["audit_mismatched"]) == 0
    if torch.equal(r0["G"], r1["G"]):
        assert int(r0["final_split"]) == 0 and int(r1["final_split"]) == 0
    else:                                              # a final split is always flagged
        assert int(r0["final_split"]) == 1 and int(r1["final_split"]) == 1


def test_server_mailbox_reduce_scatter_equals_allreduce_world8(tmp_path):
    """server FedAvg as a one-shot reduce-scatter + all-gather over the one-sided
    mailboxes (each of 8 ranks owns 1/8 of the flat buffer; each peer receives 1/8 of the model
    per phase) reaches the all-reduce's global model on every rank (fp32 summation order only)
    and every accepted shard matches its sender's committed root in the cross-rank ledger audit."""
    kw = {"num_clients": 8, "num_rounds": 2, "train_samples": 32, "test_samples": 16,
          "global_test_samples": 32}
    a = run_world(_fed_worker, 8, str(tmp_path / "a"), "server", str(tmp_path / "a"), kw)
    b = run_world(_fed_worker, 8, str(tmp_path / "b"), "server", str(tmp_path / "b"),
                  {**kw, "server_transport": "mailbox_rs"})
    for r in range(8):
        assert torch.equal(b[r]["master"], b[0]["master"])
    torch.testing.assert_close(b[0]["master"], a[0]["master"], atol=1e-6, rtol=0)


def _rs_dead_worker(rank, world, out):
    from bcfl.fl import Federation
    fed = Federation(_cfg("server", out, num_clients=3, num_rounds=4, server_transport="mailbox_rs",
                          server_timeout_s=15.0), verbose=False)
    rounds = 2 if rank == world - 1 else fed.cfg.num_rounds
    for r in range(rounds):
        fed.run_round(r)
    if rank == world - 1:
        return {"rounds": torch.tensor(rounds)}
    fed.finish(audit=False)
    return {"rounds": torch.tensor(len(fed.history)), "G": fed.global_master.clone(),
            "live_w": torch.tensor([h["live_weight"] for h in fed.history], dtype=torch.float64),
            "wait": torch.tensor([h["wait_s"] for h in fed.history], dtype=torch.float64),
            "absent": [list(h.get("absent_ranks", [])) for h in fed.history]}


def test_server_mailbox_reduce_scatter_survives_a_dead_rank(tmp_path):
    """The reduce-scatter path under a rank that stops after round 1: the survivors finish every
    round, leave it out of their shards' sums (weights re-normalised 1 -> 2/3) and agree on the
    global model except on the dead owner's shard, where each keeps its own normalised partial."""
    res = run_world(_rs_dead_worker, 3, str(tmp_path / "d"), str(tmp_path / "d"))
    assert int(res[2]["rounds"]) == 2
    for r in res[:2]:
        assert int(r["rounds"]) == 4 and torch.isfinite(r["G"]).all()
        assert r["live_w"].tolist()[:2] == pytest.approx([1.0, 1.0])
        assert r["live_w"].tolist()[2:] == pytest.approx([2 / 3, 2 / 3])
        assert r["absent"][2:] == [[2], [2]]
        # the dead rank costs ONE timeout (round 2, where it is still counted live);
        # afterwards its reduce shard and its owner shard are only checked, never waited on
        assert float(r["wait"][3]) < 5.0, r["wait"].tolist()


@pytest.mark.slow
def test_server_world8_allreduce_equals_mailbox_fedavg(tmp_path):
    """on 8 ranks (one client each, the 8-GPU layout) server FedAvg through the
    collective all-reduce, through the bf16-delta all-to-all + all-gather wire and through the
    one-sided mailbox FedAvg reach the same global model (fp32 paths: summation order only;
    bf16 wire: within the rounding of one round's update)."""
    kw = {"num_clients": 8, "num_rounds": 2, "train_samples": 32, "test_samples": 16,
          "global_test_samples": 32}
    a = run_world(_fed_worker, 8, str(tmp_path / "a"), "server", str(tmp_path / "a"), kw)
    b = run_world(_fed_worker, 8, str(tmp_path / "b"), "server", str(tmp_path / "b"),
                  {**kw, "server_transport": "mailbox"})
    c = run_world(_fed_worker, 8, str(tmp_path / "c"), "server", str(tmp_path / "c"),
                  {**kw, "server_wire_dtype": "bf16"})
    for r in range(8):
        assert torch.equal(a[r]["master"], a[0]["master"])
        assert torch.equal(b[r]["master"], b[0]["master"])
        assert torch.equal(c[r]["master"], c[0]["master"])
    torch.testing.assert_close(b[0]["master"], a[0]["master"], atol=1e-6, rtol=0)
    torch.testing.assert_close(c[0]["master"], a[0]["master"], atol=2e-4, rtol=0)


def _global_avg_worker(rank, world, out, kw):
    import numpy as _np
    from bcfl.ckpt import hf_layout, read_safetensors
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    fed = Federation(_cfg("serverless", out, **kw), verbose=False)
    fed.run()
    mine = torch.stack([fed.client_master[c] for c in fed.local_clients]) if fed.multi \
        else fed.flat.master.clone()[None]
    allm = D.all_gather_object(mine)
    res = {"models": torch.cat(allm)}
    if rank == 0:
        sd = read_safetensors(os.path.join(out, "global", "model.safetensors"))
        vec = torch.full((fed.flat.numel,), float("nan"))
        for name, off, shape in hf_layout(fed.model, fed.flat):
            vec[off:off + int(_np.prod(shape))] = sd[name].reshape(-1).float()
        res["global"] = vec
    return res


@pytest.mark.parametrize("transport", ["mailbox", "rccl"])
def test_serverless_global_checkpoint_is_the_mean_world2(tmp_path, transport):
    """VERDICT r5 #4 on 2 ranks x 2 clients: ``global/model.safetensors`` == the mean of ALL four
    client masters (fp32, atol 1e-6) — through one all-reduce in lock-step mode, and under the
    collective-free round-complete protocol because every client model at a round end IS the
    federation mean of the complete rounds (the final round closes synchronously)."""
    kw = {"num_clients": 4, "num_rounds": 3, "save_every": 1, "ledger": False}
    if transport == "rccl":
        kw.update(async_gossip=False, gossip_transport="rccl", topology="ring")
    else:
        kw.update(gossip_transport="mailbox")
    res = run_world(_global_avg_worker, 2, str(tmp_path / "d"), str(tmp_path / "d"), kw)
    models = res[0]["models"]
    assert models.shape[0] == 4
    g = res[0]["global"]
    cov = ~torch.isnan(g)          # the flat buffer's alignment padding is in no HF tensor
    assert float(cov.float().mean()) > 0.99
    torch.testing.assert_close(g[cov], models.mean(0)[cov], atol=1e-6, rtol=0)

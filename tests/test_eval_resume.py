"""Global evaluation sharded over client models, per-rank ledger resume, checkpoint round
consistency and gossip ledger records across checkpoints (CPU; multi-rank cases on gloo)."""
import json
import os

import numpy as np
import pytest
import torch

from dist_utils import run_world


def _cfg(out, **kw):
    from bcfl.config import FLConfig
    base = dict(model="tiny-bert", dataset="tiny", num_clients=4, num_rounds=2, train_samples=32,
                test_samples=16, global_test_samples=40, batch_size=16, lr=1e-3, out_dir=out,
                partition="label_shards", reference_prints=False, device="cpu", backend="gloo",
                async_ckpt=False, save_every=0)
    base.update(kw)
    return FLConfig(**base)


@pytest.fixture
def fresh():
    from bcfl.parallel import dist as D
    D.set_runtime_for_tests(None)
    yield
    D.set_runtime_for_tests(None)


def test_sharded_global_eval_scores_every_client_on_disjoint_rows(tmp_path, fresh):
    from bcfl.fl import Federation
    fed = Federation(_cfg(str(tmp_path), gossip_transport="mailbox"), verbose=False)
    rows = [fed._global_eval_rows(0, c) for c in range(4)]
    allr = np.concatenate(rows)
    assert len(allr) == 40 and len(set(allr.tolist())) == 40          # disjoint, covers the draw
    assert sorted(allr.tolist()) == sorted(fed.global_test_idx(0).tolist())
    sets = fed._global_eval_sets(0)
    assert [c for c, _ in sets] == [0, 1, 2, 3]
    h = fed.run()
    assert all(r["global_eval_rows"] == 40 for r in h)
    fa = fed.federation_accuracy()
    assert fa["rows"] == 40 and fa["round"] == 1 and fa["ranks"] == 1
    assert fa["accuracy"] == pytest.approx(h[-1]["global_acc"])


def test_client0_eval_keeps_whole_draw_on_one_model(tmp_path, fresh):
    from bcfl.fl import Federation
    fed = Federation(_cfg(str(tmp_path), gossip_transport="mailbox", global_eval_models="client0"),
                     verbose=False)
    assert [c for c, _ in fed._global_eval_sets(0)] == [None]
    h = fed.run()
    assert all(r["global_eval_rows"] == 40 for r in h)


def _eval_worker(rank, world, out):
    from bcfl.fl import Federation
    fed = Federation(_cfg(out, gossip_transport="mailbox", num_clients=2), verbose=False)
    h = fed.run()
    fa = fed.federation_accuracy()
    return {"rows_rank": torch.tensor([r["global_eval_rows"] for r in h]),
            "fa_rows": torch.tensor(fa["rows"]), "fa_ranks": torch.tensor(fa["ranks"]),
            "fa_acc": torch.tensor(fa["accuracy"])}


def test_sharded_eval_two_ranks_gathers_the_whole_draw(tmp_path):
    res = run_world(_eval_worker, 2, str(tmp_path / "d"), str(tmp_path / "d"))
    for r in res:
        assert r["rows_rank"].tolist() == [20, 20]     # each rank: its client's half
        assert int(r["fa_rows"]) == 40 and int(r["fa_ranks"]) == 2
    assert float(res[0]["fa_acc"]) == float(res[1]["fa_acc"])


def _resume_worker(rank, world, out, phase):
    from bcfl.fl import Federation
    kw = dict(num_clients=2, gossip_transport="mailbox", save_every=1, save_clients=True,
              save_resume_state=True, num_rounds=3)
    if phase == 1:
        fed = Federation(_cfg(out, **kw), verbose=False)
        fed.run(rounds=2)
        blocks = fed.ledger.blocks()
    else:
        fed = Federation(_cfg(out, resume=out, **kw), verbose=False)
        assert fed.start_round == 2
        fed.run()
        blocks = fed.ledger.blocks()
    return {"tip": fed.ledger.tip, "height": torch.tensor(len(blocks)),
            "hashes": [b["hash"] for b in blocks], "path": os.path.basename(fed.ledger.path),
            "audit_mismatched": torch.tensor((fed.ledger_audit or {}).get("mismatched", 0)),
            "audit_checked": torch.tensor((fed.ledger_audit or {}).get("checked", 0))}


def test_multirank_mailbox_resume_continues_each_ranks_own_chain(tmp_path):
    """Collective-free runs keep one chain per rank (ledger.jsonl, ledger.rank1.jsonl); a resumed
    rank must continue ITS chain (every rank used to reload rank 0's)."""
    out = str(tmp_path / "d")
    a = run_world(_resume_worker, 2, str(tmp_path / "p1"), out, 1)
    assert a[0]["path"] == "ledger.jsonl" and a[1]["path"] == "ledger.rank1.jsonl"
    assert a[0]["tip"] != a[1]["tip"]
    b = run_world(_resume_worker, 2, str(tmp_path / "p2"), out, 2)
    for r in (0, 1):
        h1 = a[r]["hashes"]
        assert b[r]["hashes"][:len(h1)] == h1          # continues its own blocks
        assert int(b[r]["height"]) > len(h1)
        assert int(b[r]["audit_mismatched"]) == 0 and int(b[r]["audit_checked"]) > 0


def test_resume_rejects_files_from_different_rounds(tmp_path, fresh):
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    out = str(tmp_path / "x")
    kw = dict(gossip_transport="mailbox", save_every=1, save_resume_state=True, num_rounds=3)
    Federation(_cfg(out, **kw), verbose=False).run(rounds=2)
    st = json.load(open(os.path.join(out, "global", "state.json")))
    st["round"] = 0   # pretend global/ is older than resume/rank0.pt
    json.dump(st, open(os.path.join(out, "global", "state.json"), "w"))
    D.set_runtime_for_tests(None)
    with pytest.raises(RuntimeError, match="different rounds"):
        Federation(_cfg(out, resume=out, **kw), verbose=False)


def _records_worker(rank, world, out, save):
    from bcfl.fl import Federation
    fed = Federation(_cfg(out, num_clients=2, gossip_transport="rccl", async_gossip=True,
                          num_rounds=4, save_every=1 if save else 0, save_resume_state=save),
                     verbose=False)
    fed.run()
    kinds = [b["kind"] for b in fed.ledger.blocks()]
    return {"verify": torch.tensor(kinds.count("verify")), "update": torch.tensor(kinds.count("update"))}


def test_checkpoint_does_not_drop_gossip_verify_blocks(tmp_path):
    """GossipEngine.state_dict() completes the in-flight exchange; the verify blocks it produces
    must still reach the ledger (they were cleared by the next end_of_round)."""
    with_ck = run_world(_records_worker, 2, str(tmp_path / "a"), str(tmp_path / "a"), True)
    without = run_world(_records_worker, 2, str(tmp_path / "b"), str(tmp_path / "b"), False)
    assert int(without[0]["verify"]) > 0
    assert int(with_ck[0]["verify"]) == int(without[0]["verify"])

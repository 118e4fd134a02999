import numpy as np
import pytest
import torch

from bcfl.config import PRESETS, FLConfig, get_preset, parse_cli
from bcfl.data.batching import ClientLoader, make_packed_batch, make_padded_batch
from bcfl.data.partition import global_test_indices, partition_clients
from bcfl.data.registry import DATASETS, get_dataset, load_split


def test_presets_cover_reference_scripts():
    for name in ["server_IID", "server_NonIID", "serverless_IID", "serverless_NonIID",
                 "server_IID_IMDB", "server_NonIID_IMDB", "server_iid_medical_transcriptions",
                 "server_noniid_medical_transcriptions", "serverless_IID_IMDB",
                 "serverless_NonIID_IMDB", "serverless_NonIID_medical_transcriptions",
                 "serverless_iid_medical_transcriptions", "serverless_cancer_biobert",
                 "serverless_cancer_albert_iid", "serverless_covid_iid",
                 "serverless_cancer_biobert_notebook"]:
        cfg = get_preset(name)
        assert cfg.num_rounds >= 2 and cfg.batch_size == 32 and cfg.lr == 5e-5
    assert get_preset("serverless_NonIID").model == "albert-base-v2"
    assert get_preset("server_IID").model == "biobert"
    assert get_preset("server_IID").num_clients == 20


def test_cli_overrides():
    cfg = parse_cli(["--preset", "serverless_NonIID", "--num-clients", "8", "--model", "bert-base",
                     "--async-gossip", "false", "--lr", "1e-4", "--inject-byzantine", "3:-1.0"])
    assert cfg.num_clients == 8 and cfg.model == "bert-base" and cfg.async_gossip is False
    assert cfg.lr == 1e-4 and cfg.inject_byzantine == {3: -1.0}
    assert cfg.partition == "label_shards"


def test_config_roundtrip():
    cfg = FLConfig(num_clients=3)
    assert cfg.replace(num_rounds=7).num_rounds == 7
    with pytest.raises(KeyError):
        cfg.replace(nonsense=1)


def test_synthetic_split_shapes():
    ds = load_split("imdb", "train", 30522, 512)
    assert len(ds) == 25000 and ds.num_classes == 2
    # label-sorted like HF imdb
    assert (np.diff(ds.labels) >= 0).all()
    L = ds.lengths
    assert L.max() <= 512 and L.min() >= 8
    assert 150 < np.median(L) < 320
    assert (ds.tokens[ds.offsets[:-1]] == 101).all() and (ds.tokens[ds.offsets[1:] - 1] == 102).all()
    assert ds.tokens.max() < 30522
    med = load_split("medical", "train", 28996, 512)
    assert len(med) == 12000 and med.num_classes == 40 and np.median(med.lengths) < 60


def test_partitions():
    spec = get_dataset("imdb")
    tr = load_split("imdb", "train", 30522, 512).labels
    te = load_split("imdb", "test", 30522, 512).labels
    ref = partition_clients("ref_contiguous", spec, tr, te, 10, 240, 60)
    assert all(len(s.train) == 240 and len(s.test) == 60 for s in ref)
    assert ref[3].train[0] == 900 and ref[3].test[0] == 900 + 240
    # the reference's Non-IID shards of label-sorted IMDB are single-class label 0
    assert all(np.unique(tr[s.train]).tolist() == [0] for s in ref)
    ls = partition_clients("label_shards", spec, tr, te, 8, 240, 60)
    cls = [int(np.unique(tr[s.train])[0]) for s in ls]
    assert cls == [0, 0, 0, 0, 1, 1, 1, 1]
    iid = partition_clients("iid_random", spec, tr, te, 4, 100, 100, seed=1, round_idx=2)
    assert len({tuple(s.train) for s in iid}) == 4
    again = partition_clients("iid_random", spec, tr, te, 4, 100, 100, seed=1, round_idx=2)
    assert all((a.train == b.train).all() for a, b in zip(iid, again))
    shared = partition_clients("shared_random", spec, tr, te, 4, 100, 100)
    assert all((s.train == shared[0].train).all() for s in shared)
    dr = partition_clients("dirichlet", spec, tr, te, 5, 200, 50, alpha=0.1)
    assert all(len(s.train) == 200 for s in dr)
    g = global_test_indices(25000, 100, 42, None)
    assert len(g) == 100 and len(set(g)) == 100


def test_packed_batch_matches_padded():
    ds = load_split("tiny", "train", 2048, 128)
    idx = np.array([3, 17, 40, 41, 100])
    pb = make_packed_batch(ds, idx)
    pad = make_padded_batch(ds, idx)
    assert pb.cu_host[-1] == pad.attention_mask.sum()
    mask = pad.attention_mask.bool()
    assert torch.equal(pb.input_ids.long(), pad.input_ids[mask])
    for b in range(len(idx)):
        s, e = pb.cu_host[b], pb.cu_host[b + 1]
        assert torch.equal(pb.position_ids[s:e], torch.arange(e - s, dtype=torch.int32))
    assert pb.max_seqlen == int(ds.lengths[idx].max())


def test_client_loader_epochs():
    ds = load_split("tiny", "train", 2048, 128)
    ld = ClientLoader(ds, np.arange(70), batch_size=32, shuffle=True, seed=3)
    assert len(ld) == 3
    b0 = ld.device_batches("cpu", epoch=0)
    b1 = ld.device_batches("cpu", epoch=1)
    assert [b.batch_size for b in b0] == [32, 32, 6]
    assert not torch.equal(b0[0].labels, b1[0].labels) or not torch.equal(b0[0].input_ids, b1[0].input_ids)


def test_config_rejects_unknown_choices():
    import pytest
    from bcfl.config import FLConfig
    for kw in ({"mixing": "choco"}, {"server_wire_dtype": "fp16"}, {"drift_correction": "x"},
               {"mode": "p2p"},
               {"deterministic": True, "async_gossip": True, "gossip_transport": "mailbox"}):
        with pytest.raises(ValueError):
            FLConfig(**kw)
    FLConfig(deterministic=True, async_gossip=True)  # auto transport -> lock-step engine


def test_compat_presets_reproduce_reference_partitions():
    """Per-script partition semantics: the _compat presets run what the
    reference scripts actually do; the plain presets keep a real Non-IID split."""
    import numpy as np
    from bcfl.data.partition import partition_clients
    from bcfl.data.registry import get_dataset, load_split

    def parts(name, n=None):
        cfg = get_preset(name)
        spec = get_dataset(cfg.dataset)
        tr = load_split(cfg.dataset, "train", 30522, 128, 1234, 101, 102)
        te = load_split(cfg.dataset, "test", 30522, 128, 1234, 101, 102)
        return cfg, tr, partition_clients(cfg.partition, spec, tr.labels, te.labels,
                                          n or cfg.num_clients, cfg.train_samples,
                                          cfg.test_samples, cfg.seed)

    # E2 compat: every client holds the same 240 / 60 rows of the shuffled split, both classes
    cfg, tr, ps = parts("server_NonIID_IMDB_compat")
    assert len(ps) == 20 and all(np.array_equal(p.train, ps[0].train) for p in ps)
    assert len(ps[0].train) == 240 and len(ps[0].test) == 60
    assert len(np.unique(tr.labels[ps[0].train])) == 2
    # E4 compat: one shared IID 1000/1000 draw
    cfg, tr, ps = parts("server_noniid_medical_transcriptions_compat")
    assert all(np.array_equal(p.train, ps[0].train) for p in ps) and len(ps[0].train) == 1000
    assert len(np.unique(tr.labels[ps[0].train])) > 20
    # E6 compat: contiguous unshuffled shards [300k, 300k+240) -> all label 0 on label-sorted IMDB
    cfg, tr, ps = parts("serverless_NonIID_IMDB_compat")
    assert [int(p.train[0]) for p in ps[:3]] == [0, 300, 600]
    assert all((tr.labels[p.train] == 0).all() for p in ps)
    # the plain Non-IID presets: clients see different single classes
    cfg, tr, ps = parts("serverless_NonIID_IMDB")
    assert {int(tr.labels[p.train][0]) for p in ps} == {0, 1}
    assert all(len(np.unique(tr.labels[p.train])) == 1 for p in ps)


def test_attn_schedule_covers_every_block_longest_first():
    from bcfl.data.batching import attn_schedule, pad_packed
    cu = np.array([0, 90, 603, 603, 870, 1870, 1999])
    s = attn_schedule(cu).numpy()
    lens = np.diff(cu)
    want = sorted((b, k) for b in range(len(lens)) for k in range(-(-lens[b] // 128)))
    for row in s:
        got = [(int(e) >> 12, int(e) & 4095) for e in row]
        assert sorted(got) == want                       # every block once, empty rows none
        L = [lens[b] for b, _ in got]
        assert L == sorted(L, reverse=True)              # longest sequence first
    q = [(int(e) >> 12, int(e) & 4095) for e in s[0]][:8]
    assert q[0] == (4, 7) and q[-1] == (4, 0)            # query blocks: last block first
    k = [(int(e) >> 12, int(e) & 4095) for e in s[1]][:8]
    assert k[0] == (4, 0)                                # key blocks: first block first
    ds = load_split("tiny", "train", 2048, 128)
    b = pad_packed(make_packed_batch(ds, np.arange(10)), 64)
    assert b.attn_sched is not None and b.attn_sched.shape[0] == 2
    assert int(b.attn_sched.shape[1]) == int(sum(-(-n // 128) for n in np.diff(b.cu_host)))

"""Real-text path: reference CSVs + offline WordPiece (skipped when the CSVs are not mounted)."""
import numpy as np
import pytest

from bcfl.data import text

pytestmark = pytest.mark.skipif(not text.available("medical_csv"), reason="reference CSVs not mounted")


def test_medical_csv_split_shapes_and_labels():
    from bcfl.data.registry import load_split
    tr = load_split("medical_csv", "train", 30522, 128)
    te = load_split("medical_csv", "test", 30522, 128)
    assert len(tr) == 12000 and len(te) == 3000
    assert tr.num_classes == 40 and set(np.unique(tr.labels)) == set(range(40))
    lens = tr.lengths
    assert lens.min() >= 2 and lens.max() <= 128  # a few CSV descriptions are empty
    rows = [tr.row(i) for i in range(50)]
    assert all(r[0] == 101 and r[-1] == 102 for r in rows)
    assert tr.tokens.max() < 30522 and (tr.tokens[(tr.tokens != 101) & (tr.tokens != 102)] >= 100).all()
    # reference file order kept: row 0 is the first CSV record (label 17)
    assert tr.labels[0] == 17


def test_wordpiece_layout_and_roundtrip():
    tok = text.tokenizer("medical_csv", 4096)
    assert tok.vocab["[PAD]"] == 0 and tok.vocab["[UNK]"] == 100 and tok.vocab["[CLS]"] == 101
    assert max(tok.vocab.values()) < 4096
    ids = tok.encode_batch(["Autopsy of a white female who died of acute combined drug intoxication."], 64)[0]
    pieces = [t for t, _ in sorted(tok.vocab.items(), key=lambda x: x[1])]
    inv = {i: t for t, i in tok.vocab.items()}
    words = [inv[i] for i in ids[1:-1]]
    assert "autopsy" in "".join(w.replace("##", "") for w in words)
    assert 100 not in ids.tolist()  # in-vocabulary sentence: no [UNK]
    assert len(pieces) <= 4096


def test_selfdriving_holdout_split():
    from bcfl.data.registry import load_split
    tr = load_split("selfdriving_csv", "train", 1024, 64)
    te = load_split("selfdriving_csv", "test", 1024, 64)
    assert len(tr) == 400 and len(te) == 100 and tr.num_classes == 3


def test_federation_on_real_text(tmp_path):
    from bcfl.config import FLConfig
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D
    D.set_runtime_for_tests(None)
    cfg = FLConfig(mode="serverless", model="tiny-bert", dataset="medical_csv", num_clients=2,
                   num_rounds=1, train_samples=64, test_samples=32, global_test_samples=32,
                   batch_size=16, lr=1e-3, out_dir=str(tmp_path), partition="ref_contiguous",
                   reference_prints=False, device="cpu", save_every=0, max_seq_len=64)
    fed = Federation(cfg, verbose=False)
    h = fed.run()
    assert fed.num_labels == 40 and 0.0 <= h[-1]["global_acc"] <= 1.0
    D.set_runtime_for_tests(None)

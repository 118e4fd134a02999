"""Real-text datasets from the reference's local CSV files + an offline-trained WordPiece tokenizer.

The reference ships CSVs it never loads: ``Dataset/train_file_mt.csv`` /
``Dataset/test_file_mt.csv`` (Medical Transcriptions: ``description`` -> ``medical_specialty``,
40 classes, 12000 / 3000 rows) and ``Dataset/sentiment_analysis_self_driving_vehicles.csv``
(``Text`` -> ``Sentiment``, 3 classes, 500 rows). Its scripts tokenize with a pretrained HF
WordPiece vocab (``AutoTokenizer.from_pretrained``, ``src/Servercase/server_IID_IMDB.py:73``); there
is no network here, so the vocabulary is TRAINED on the training split with the HF ``tokenizers``
library (the same Rust WordPiece implementation, BERT normalizer + pre-tokenizer, lower-cased) and
laid out like BERT's: ``[PAD]=0``, ``[UNK]=100``, ``[CLS]``/``[SEP]`` = the model's ids, word pieces
from 104 up. Rows keep file order (the reference's contiguous Non-IID shards slice the file).

CSV files are read with the ``csv`` module only (text, no deserialisation). Data location:
``$BCFL_DATA_DIR`` (default: the read-only reference checkout's ``Dataset/``).
"""
from __future__ import annotations

import csv
import functools
import os
from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np

from .synthetic import TokenDataset

DATA_DIR_DEFAULT = "/root/reference/Dataset"
RESERVED = 104  # ids below this are specials / unused (BERT layout)


def data_dir() -> str:
    return os.environ.get("BCFL_DATA_DIR", DATA_DIR_DEFAULT)


@dataclass(frozen=True)
class CsvSource:
    train_file: str
    test_file: str        # "" -> deterministic holdout split of train_file
    text_col: str
    label_col: str
    holdout: float = 0.2


CSV_SOURCES: Dict[str, CsvSource] = {
    "medical_csv": CsvSource("train_file_mt.csv", "test_file_mt.csv", "description",
                             "medical_specialty"),
    "selfdriving_csv": CsvSource("sentiment_analysis_self_driving_vehicles.csv", "", "Text",
                                 "Sentiment"),
}


def available(name: str) -> bool:
    src = CSV_SOURCES[name]
    return os.path.exists(os.path.join(data_dir(), src.train_file))


def _read(path: str, text_col: str, label_col: str) -> Tuple[List[str], List[str]]:
    texts, labels = [], []
    with open(path, newline="", encoding="utf-8") as fh:
        for r in csv.DictReader(fh):
            texts.append(r[text_col] or "")
            labels.append((r[label_col] or "").strip())
    return texts, labels


@functools.lru_cache(maxsize=8)
def _raw(name: str) -> Tuple[Tuple[List[str], List[str]], Tuple[List[str], List[str]], List[str]]:
    src = CSV_SOURCES[name]
    d = data_dir()
    tr = _read(os.path.join(d, src.train_file), src.text_col, src.label_col)
    if src.test_file:
        te = _read(os.path.join(d, src.test_file), src.text_col, src.label_col)
    else:  # fixed holdout: every k-th row goes to test
        k = max(int(round(1.0 / src.holdout)), 2)
        idx_te = [i for i in range(len(tr[0])) if i % k == k - 1]
        idx_tr = [i for i in range(len(tr[0])) if i % k != k - 1]
        te = ([tr[0][i] for i in idx_te], [tr[1][i] for i in idx_te])
        tr = ([tr[0][i] for i in idx_tr], [tr[1][i] for i in idx_tr])
    names = sorted(set(tr[1]) | set(te[1]), key=lambda s: (not s.lstrip("-").isdigit(), int(s) if s.lstrip("-").isdigit() else 0, s))
    return tr, te, names


def num_classes(name: str) -> int:
    return len(_raw(name)[2])


def split_sizes(name: str) -> Tuple[int, int]:
    tr, te, _ = _raw(name)
    return len(tr[0]), len(te[0])


class WordPiece:
    """Offline-trained WordPiece (HF ``tokenizers``) with BERT's id layout."""

    def __init__(self, texts: Sequence[str], vocab_size: int, cls_id: int = 101, sep_id: int = 102):
        from tokenizers import Tokenizer, models, normalizers, pre_tokenizers, trainers
        if vocab_size <= RESERVED + 64:
            raise ValueError(f"vocab_size {vocab_size} too small for a WordPiece vocabulary")
        tok = Tokenizer(models.WordPiece(unk_token="[UNK]"))
        tok.normalizer = normalizers.BertNormalizer(lowercase=True)
        tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
        specials = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
        tok.train_from_iterator(list(texts), trainers.WordPieceTrainer(
            vocab_size=vocab_size - RESERVED + len(specials), special_tokens=specials))
        pieces = sorted((i, t) for t, i in tok.get_vocab().items() if t not in specials)
        vocab = {"[PAD]": 0, "[UNK]": 100, "[CLS]": cls_id, "[SEP]": sep_id, "[MASK]": 103}
        used = set(vocab.values())
        for k in range(1, RESERVED):
            if k not in used:
                vocab[f"[unused{k}]"] = k
        nxt = RESERVED
        for _, t in pieces:
            if nxt >= vocab_size:
                break
            vocab[t] = nxt
            nxt += 1
        self.vocab = vocab
        out = Tokenizer(models.WordPiece(vocab=vocab, unk_token="[UNK]"))
        out.normalizer = tok.normalizer
        out.pre_tokenizer = tok.pre_tokenizer
        self.tok = out
        self.cls_id, self.sep_id = cls_id, sep_id

    def encode_batch(self, texts: Sequence[str], max_len: int) -> List[np.ndarray]:
        body = max_len - 2
        outs = []
        for e in self.tok.encode_batch(list(texts), add_special_tokens=False):
            ids = np.asarray(e.ids[:body], dtype=np.int32)
            outs.append(np.concatenate([[self.cls_id], ids, [self.sep_id]]).astype(np.int32))
        return outs


@functools.lru_cache(maxsize=8)
def tokenizer(name: str, vocab_size: int, cls_id: int = 101, sep_id: int = 102) -> WordPiece:
    tr, _, _ = _raw(name)
    return WordPiece(tr[0], vocab_size, cls_id, sep_id)


def load_csv_split(name: str, split: str, vocab_size: int, max_len: int = 512, cls_id: int = 101,
                   sep_id: int = 102) -> TokenDataset:
    tr, te, names = _raw(name)
    texts, labels = tr if split == "train" else te
    lid = {s: i for i, s in enumerate(names)}
    rows = tokenizer(name, vocab_size, cls_id, sep_id).encode_batch(texts, max_len)
    offsets = np.zeros(len(rows) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum([len(r) for r in rows])
    toks = np.concatenate(rows).astype(np.int32) if rows else np.zeros(0, np.int32)
    return TokenDataset(toks, offsets, np.asarray([lid[s] for s in labels], dtype=np.int64),
                        len(names), vocab_size)
